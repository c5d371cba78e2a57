#!/bin/bash
# Frames-in-flight sweep on one box, interleaved: CONFIGS x INFLIGHTS x REPS bench lines (no CPU baseline).
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp PYTHONUNBUFFERED=1
mkdir -p gpurun_out
TAG=${TAG:-ifs}
for rep in $(seq 1 ${REPS:-2}); do
  for cfg in ${CONFIGS:-C2 C3}; do
    for k in ${INFLIGHTS:-2 3 4}; do
      timeout -k 10 240 python bench.py --config $cfg --inflight $k --steps ${STEPS:-40} --warmup 5 --no-cpu-baseline --no-async-e2e \
        > gpurun_out/${TAG}_${cfg}_if${k}_$rep.log 2>&1 || { echo "$cfg if$k rc=$?"; tail -5 gpurun_out/${TAG}_${cfg}_if${k}_$rep.log; exit 1; }
      python3 -c "import json; d=json.loads(open('gpurun_out/${TAG}_${cfg}_if${k}_$rep.log').read().strip().splitlines()[-1]); print('$cfg if$k $rep', d['value'], d['ms_per_step'])"
    done
  done
done
echo done

#!/bin/bash
# Frames-in-flight sweep of the in-tree library: bench.py --inflight K for K in $KS per config, interleaved.
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp PYTHONUNBUFFERED=1
mkdir -p gpurun_out
TAG=${TAG:-if}
for rep in $(seq 1 ${REPS:-2}); do
  for cfg in ${CONFIGS:-C2 C3 C4}; do
    for k in ${KS:-2 3 4 5}; do
      timeout -k 10 240 python bench.py --config $cfg --steps ${STEPS:-40} --warmup 5 --inflight $k --no-cpu-baseline --no-async-e2e \
        > gpurun_out/${TAG}_${cfg}_k${k}_$rep.log 2>&1 || { echo "$cfg k$k rc=$?"; tail -5 gpurun_out/${TAG}_${cfg}_k${k}_$rep.log; exit 1; }
      python3 -c "import json; d=json.loads(open('gpurun_out/${TAG}_${cfg}_k${k}_$rep.log').read().strip().splitlines()[-1]); r=d['roofline']; print('$cfg k$k $rep', d['value'], d['ms_per_step'], r['kernel_us'])"
    done
  done
done
echo done

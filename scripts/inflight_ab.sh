#!/bin/bash
# Frames in flight at the settled clock (bench defaults: preroll + 1,000 timed steps), interleaved on one box.
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
for rep in 1 2; do
  for cfg in ${CONFIGS:-C2 C4}; do
    for k in ${INFLIGHT:-2 3 4}; do
      timeout -k 10 200 python bench.py --config $cfg --inflight $k --no-cpu-baseline --no-async-e2e > gpurun_out/ifab.log 2>&1 || { echo "rc=$?"; tail -5 gpurun_out/ifab.log; exit 1; }
      python3 -c "import json; d=json.loads(open('gpurun_out/ifab.log').read().strip().splitlines()[-1]); r=d['roofline']; print('$cfg if$k $rep', d['value'], d['ms_per_step'], r['kernel_us'])"
    done
  done
done

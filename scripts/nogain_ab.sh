#!/bin/bash
# What the per-frame gain feed costs beside the composites at the settled clock: bench with and without
# gain (--no-gain: the composite alone), interleaved on one box.
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
for rep in 1 2; do
  for cfg in C2 C4; do
    for a in "" "--no-gain"; do
      timeout -k 10 200 python bench.py --config $cfg $a --no-cpu-baseline --no-async-e2e > gpurun_out/ng.log 2>&1 || { echo "rc=$?"; tail -5 gpurun_out/ng.log; exit 1; }
      python3 -c "import json; d=json.loads(open('gpurun_out/ng.log').read().strip().splitlines()[-1]); r=d['roofline']; o=d['roofline_one_in_flight']; print('$cfg [$a] $rep', d['value'], d['ms_per_step'], r['kernel_us'], o['kernel_us'], o['step_us'])"
    done
  done
done

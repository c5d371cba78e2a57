#!/bin/bash
# Timed region against the GPU's clock ramp ("Clock ramp"): the default bench line without
# and with its untimed preroll, and a long timed region, interleaved on one box.
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
CFG=${CFG:-C2}
for rep in 1 2; do
  for a in "--preroll 0" "--preroll 0.5" "--preroll 0 --steps 4000" "--preroll 0 --warmup 10000"; do
    timeout -k 10 200 python bench.py --config $CFG $a --no-cpu-baseline --no-async-e2e > gpurun_out/warm.log 2>&1 || { echo "rc=$?"; tail -5 gpurun_out/warm.log; exit 1; }
    python3 -c "import json; d=json.loads(open('gpurun_out/warm.log').read().strip().splitlines()[-1]); r=d['roofline']; o=d['roofline_one_in_flight']; print('$CFG $a |', d['value'], d['ms_per_step'], d['host_issue_ms_per_step'], r['kernel_us'], o['kernel_us'], o['step_us'], d.get('preroll'))"
  done
done

#!/bin/bash
# Texture-convention mode on C2 / C3 (bench.py --remap texture), beside the default sampling.
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp PYTHONUNBUFFERED=1
mkdir -p gpurun_out
TAG=${TAG:-r5t}
for CFG in C2 C3; do
  for R in remap texture; do
    timeout -k 10 300 python bench.py --config $CFG --remap $R --steps 30 --warmup 5 --no-cpu-baseline --no-async-e2e \
      > gpurun_out/${TAG}_${CFG}_$R.json 2> gpurun_out/${TAG}_${CFG}_$R.err || { echo "$CFG $R rc=$?"; tail -5 gpurun_out/${TAG}_${CFG}_$R.err; exit 1; }
    python3 -c "import json; d=json.loads(open('gpurun_out/${TAG}_${CFG}_$R.json').read().strip().splitlines()[-1]); print('$CFG $R', d['value'], d['ms_per_step'], d['roofline']['kernel_us'])"
  done
done

#!/bin/bash
# Barrier cost bound: static item dealing (OCTVR_DYN=0) with and without the item barriers
# (OCTVR_DIAG_NOBAR: wrong output, timing only; every LDS / global address stays bounded).
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp PYTHONUNBUFFERED=1
mkdir -p gpurun_out
V=$PWD/opencv-octvr_amd/lib/variants
b() {  # name cfg [env...]
  local name=$1 cfg=$2; shift 2
  env "$@" timeout -k 10 240 python bench.py --config $cfg --steps 60 --warmup 5 --no-cpu-baseline --no-async-e2e \
      > gpurun_out/d3_$name.log 2>&1 || { echo "$name rc=$?"; tail -5 gpurun_out/d3_$name.log; exit 1; }
  python3 -c "import json; d=json.loads(open('gpurun_out/d3_$name.log').read().strip().splitlines()[-1]); r=d['roofline']; o=d.get('roofline_one_in_flight',{}); print('$name', d['value'], d['ms_per_step'], r['kernel_us'], r['frac_at_step_time'], o.get('kernel_us'), o.get('step_us'))"
}
for rep in 1 2; do
  b cur_$rep C2
  b dyn0_$rep C2 OCTVR_HIP_LIB=$V/dyn0.so
  b nobar_$rep C2 OCTVR_HIP_LIB=$V/nobar.so
done
echo done

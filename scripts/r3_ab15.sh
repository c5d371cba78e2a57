#!/bin/bash
# Round 3 A/B 15: multi-band blend register budget (MB_BLEND_WAVES 6 / 8 vs 7) and the collapse taps
# issued before the camera loop (MB_COLLAPSE_FIRST, re-measured now that most tiles take the owned path), C3.
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
V=$PWD/opencv-octvr_amd/lib/variants
b() {  # name cfg [env...]
  local name=$1 cfg=$2; shift 2
  env "$@" timeout -k 10 240 python bench.py --config $cfg --steps 30 --warmup 5 --no-cpu-baseline --no-async-e2e \
      > gpurun_out/ab15_$name.log 2>&1 || { echo "$name rc=$?"; tail -5 gpurun_out/ab15_$name.log; exit 1; }
  python3 -c "import json; d=json.loads(open('gpurun_out/ab15_$name.log').read().strip().splitlines()[-1]); r=d['roofline']; o=d.get('roofline_one_in_flight',{}); print('$name', d['value'], d['ms_per_step'], r['kernel_us'], o.get('kernel_us'), o.get('step_us'))"
}
for rep in 1 2 3; do
  b base_$rep C3
  b mbw6_$rep C3 OCTVR_HIP_LIB=$V/mbw6.so
  b mbw8_$rep C3 OCTVR_HIP_LIB=$V/mbw8.so
  b mbcf_$rep C3 OCTVR_HIP_LIB=$V/mbcf.so
done
echo done

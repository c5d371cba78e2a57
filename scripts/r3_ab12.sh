#!/bin/bash
# Round 3 A/B 12: RGB -> YUV420P as full-range BT.601 in 8-bit fixed point (v_dot4 per pixel) instead of
# the f32 definition (oracle changed with it) vs HEAD; then the whole GPU suite.
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp PYTHONUNBUFFERED=1
mkdir -p gpurun_out
V=$PWD/opencv-octvr_amd/lib/variants
b() {  # name cfg [env...]
  local name=$1 cfg=$2; shift 2
  env "$@" timeout -k 10 240 python bench.py --config $cfg --steps 60 --warmup 5 --no-cpu-baseline --no-async-e2e \
      > gpurun_out/ab12_$name.log 2>&1 || { echo "$name rc=$?"; tail -5 gpurun_out/ab12_$name.log; exit 1; }
  python3 -c "import json; d=json.loads(open('gpurun_out/ab12_$name.log').read().strip().splitlines()[-1]); r=d['roofline']; o=d.get('roofline_one_in_flight',{}); print('$name', d['value'], d['ms_per_step'], r['kernel_us'], o.get('kernel_us'), o.get('step_us'))"
}
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/ > gpurun_out/ab12_tests.log 2>&1 || { echo "tests rc=$?"; tail -30 gpurun_out/ab12_tests.log; exit 1; }
tail -1 gpurun_out/ab12_tests.log
for rep in 1 2 3; do
  b prev_$rep C2 OCTVR_HIP_LIB=$V/prev.so
  b yuv_$rep C2
done
b prev_C4 C4 OCTVR_HIP_LIB=$V/prev.so
b yuv_C4 C4
b prev_C3 C3 OCTVR_HIP_LIB=$V/prev.so
b yuv_C3 C3
echo done

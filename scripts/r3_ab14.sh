#!/bin/bash
# Round 3 A/B 14: multi-band level 0 and the scaled-output resize pack their 0..255 channels straight
# into quad_yuv (no float round trip) vs HEAD; C3; then the whole GPU suite.
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp PYTHONUNBUFFERED=1
mkdir -p gpurun_out
V=$PWD/opencv-octvr_amd/lib/variants
b() {  # name cfg [env...]
  local name=$1 cfg=$2; shift 2
  env "$@" timeout -k 10 240 python bench.py --config $cfg --steps 30 --warmup 5 --no-cpu-baseline --no-async-e2e \
      > gpurun_out/ab14_$name.log 2>&1 || { echo "$name rc=$?"; tail -5 gpurun_out/ab14_$name.log; exit 1; }
  python3 -c "import json; d=json.loads(open('gpurun_out/ab14_$name.log').read().strip().splitlines()[-1]); r=d['roofline']; o=d.get('roofline_one_in_flight',{}); print('$name', d['value'], d['ms_per_step'], r['kernel_us'], o.get('kernel_us'), o.get('step_us'))"
}
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/ > gpurun_out/ab14_tests.log 2>&1 || { echo "tests rc=$?"; tail -30 gpurun_out/ab14_tests.log; exit 1; }
tail -1 gpurun_out/ab14_tests.log
for rep in 1 2 3; do
  b prev_$rep C3 OCTVR_HIP_LIB=$V/prev.so
  b new_$rep C3
done
echo done

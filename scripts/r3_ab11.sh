#!/bin/bash
# Round 3 A/B 11: per-item gain table in LDS (MODE 0: a channel is one table read instead of a
# conversion, multiply, round and min) vs HEAD; blend / composite parity.
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp PYTHONUNBUFFERED=1
mkdir -p gpurun_out
V=$PWD/opencv-octvr_amd/lib/variants
b() {  # name cfg [env...]
  local name=$1 cfg=$2; shift 2
  env "$@" timeout -k 10 240 python bench.py --config $cfg --steps 60 --warmup 5 --no-cpu-baseline --no-async-e2e \
      > gpurun_out/ab11_$name.log 2>&1 || { echo "$name rc=$?"; tail -5 gpurun_out/ab11_$name.log; exit 1; }
  python3 -c "import json; d=json.loads(open('gpurun_out/ab11_$name.log').read().strip().splitlines()[-1]); r=d['roofline']; o=d.get('roofline_one_in_flight',{}); print('$name', d['value'], d['ms_per_step'], r['kernel_us'], o.get('kernel_us'), o.get('step_us'))"
}
OCTVR_HIP_LIB=$V/lut16.so timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_parity.py tests/test_gpu_fullsize.py > gpurun_out/ab11_tests.log 2>&1 || { echo "tests rc=$?"; tail -30 gpurun_out/ab11_tests.log; exit 1; }
tail -1 gpurun_out/ab11_tests.log
for rep in 1 2 3; do
  b prev_$rep C2 OCTVR_HIP_LIB=$V/prev.so
  b lut32_$rep C2 OCTVR_HIP_LIB=$V/lut32.so
  b lut16_$rep C2 OCTVR_HIP_LIB=$V/lut16.so
done
for rep in 1 2; do
  b prev_C4_$rep C4 OCTVR_HIP_LIB=$V/prev.so
  b lut32_C4_$rep C4 OCTVR_HIP_LIB=$V/lut32.so
  b lut16_C4_$rep C4 OCTVR_HIP_LIB=$V/lut16.so
done
echo done

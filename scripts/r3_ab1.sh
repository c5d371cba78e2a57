#!/bin/bash
# Round 3 A/B 1: composite VALU diet (entry layout with VOP2 weight decode, scalar finish / staging) vs
# the committed library, and an extra-VALU diagnostic; then the composite / multi-band parity tests.
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
V=$PWD/opencv-octvr_amd/lib/variants
b() {  # name cfg [env...]
  local name=$1 cfg=$2; shift 2
  env "$@" timeout -k 10 240 python bench.py --config $cfg --steps 60 --warmup 5 --no-cpu-baseline --no-async-e2e \
      > gpurun_out/ab1_$name.log 2>&1 || { echo "$name rc=$?"; tail -5 gpurun_out/ab1_$name.log; exit 1; }
  python3 -c "import json; d=json.loads(open('gpurun_out/ab1_$name.log').read().strip().splitlines()[-1]); r=d['roofline']; o=d.get('roofline_one_in_flight',{}); print('$name', d['value'], d['ms_per_step'], r['kernel_us'], r['frac_at_step_time'], o.get('kernel_us'), o.get('step_us'))"
}
for rep in 1 2; do
  b base_C2_$rep C2 OCTVR_HIP_LIB=$V/base.so
  b new_C2_$rep C2
  b xv4_C2_$rep C2 OCTVR_HIP_LIB=$V/xvalu4.so
done
b base_C4 C4 OCTVR_HIP_LIB=$V/base.so
b new_C4 C4
b base_C3 C3 OCTVR_HIP_LIB=$V/base.so
b new_C3 C3
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_parity.py tests/test_gpu_fullsize.py > gpurun_out/ab1_tests.log 2>&1 || { echo "tests rc=$?"; tail -20 gpurun_out/ab1_tests.log; exit 1; }
tail -2 gpurun_out/ab1_tests.log
echo done

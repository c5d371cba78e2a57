#!/bin/bash
# Round 3 A/B 13: the next item's entries loaded after this item's computation (OCTVR_ENT_LATE: no
# copy of in-flight entries across the compute, 10 fewer VALU per iteration) vs the default build.
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp PYTHONUNBUFFERED=1
mkdir -p gpurun_out
V=$PWD/opencv-octvr_amd/lib/variants
b() {  # name cfg [env...]
  local name=$1 cfg=$2; shift 2
  env "$@" timeout -k 10 240 python bench.py --config $cfg --steps 60 --warmup 5 --no-cpu-baseline --no-async-e2e \
      > gpurun_out/ab13_$name.log 2>&1 || { echo "$name rc=$?"; tail -5 gpurun_out/ab13_$name.log; exit 1; }
  python3 -c "import json; d=json.loads(open('gpurun_out/ab13_$name.log').read().strip().splitlines()[-1]); r=d['roofline']; o=d.get('roofline_one_in_flight',{}); print('$name', d['value'], d['ms_per_step'], r['kernel_us'], o.get('kernel_us'), o.get('step_us'))"
}
OCTVR_HIP_LIB=$V/entlate.so timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_parity.py tests/test_gpu_fullsize.py tests/test_gpu_vignette.py tests/test_gpu_scaled.py > gpurun_out/ab13_tests.log 2>&1 || { echo "tests rc=$?"; tail -30 gpurun_out/ab13_tests.log; exit 1; }
tail -1 gpurun_out/ab13_tests.log
for rep in 1 2 3; do
  b def_$rep C2
  b late_$rep C2 OCTVR_HIP_LIB=$V/entlate.so
done
for rep in 1 2; do
  b def_C4_$rep C4
  b late_C4_$rep C4 OCTVR_HIP_LIB=$V/entlate.so
done
echo done

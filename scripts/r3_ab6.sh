#!/bin/bash
# Round 3 A/B 6: min-only saturation (minonly) and scalar-offset stores (new) (clamped slot gains) vs the
# previous commit; more opcode prices (OCTVR_DIAG_XOP 8-15); composite / blend parity.
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp PYTHONUNBUFFERED=1
mkdir -p gpurun_out
V=$PWD/opencv-octvr_amd/lib/variants
b() {  # name cfg [env...]
  local name=$1 cfg=$2; shift 2
  env "$@" timeout -k 10 240 python bench.py --config $cfg --steps 60 --warmup 5 --no-cpu-baseline --no-async-e2e \
      > gpurun_out/ab6_$name.log 2>&1 || { echo "$name rc=$?"; tail -5 gpurun_out/ab6_$name.log; exit 1; }
  python3 -c "import json; d=json.loads(open('gpurun_out/ab6_$name.log').read().strip().splitlines()[-1]); r=d['roofline']; o=d.get('roofline_one_in_flight',{}); print('$name', d['value'], d['ms_per_step'], r['kernel_us'], o.get('kernel_us'), o.get('step_us'))"
}
timeout -k 10 120 python scripts/dbg_stitch.py rigA rigB | grep mismatches && \
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_parity.py tests/test_gpu_fullsize.py tests/test_gpu_vignette.py tests/test_gpu_morph.py tests/test_gpu_scaled.py > gpurun_out/ab6_tests.log 2>&1 || { echo "tests rc=$?"; tail -30 gpurun_out/ab6_tests.log; exit 1; }
tail -1 gpurun_out/ab6_tests.log
for rep in 1 2 3; do
  b prev_$rep C2 OCTVR_HIP_LIB=$V/prev.so
  b minonly_$rep C2 OCTVR_HIP_LIB=$V/minonly.so
  b new_$rep C2
done
for i in 8 9 10 11 12 13 14 15 16; do b x${i} C2 OCTVR_HIP_LIB=$V/x$i.so; done
b prev_4 C2 OCTVR_HIP_LIB=$V/prev.so
b new_4 C2
echo done

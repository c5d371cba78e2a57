#!/bin/bash
# C2 composite: next item's loads before the second barrier (OCTVR_ISSUE_EARLY) vs default
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp PYTHONUNBUFFERED=1
mkdir -p gpurun_out
V=$PWD/opencv-octvr_amd/lib/variants
OCTVR_HIP_LIB=$V/ie1.so timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_fullsize.py -m gpu -q -k "fullsize or c2 or frames_in_flight or vignette or golden" --timeout 250 --timeout-method thread -p no:cacheprovider > gpurun_out/p3_tests.log 2>&1 || { echo "tests rc=$?"; grep -E "FAILED|passed|failed" gpurun_out/p3_tests.log | tail; exit 1; }
grep -E "passed|failed" gpurun_out/p3_tests.log | tail -1
b() {
  local name=$1; shift
  env "$@" timeout -k 10 240 python bench.py --config ${CFG:-C2} --steps 60 --warmup 5 --no-cpu-baseline --no-async-e2e \
      > gpurun_out/p3_$name.log 2>&1 || { echo "$name rc=$?"; tail -5 gpurun_out/p3_$name.log; exit 1; }
  python3 -c "import json; d=json.loads(open('gpurun_out/p3_$name.log').read().strip().splitlines()[-1]); r=d['roofline']; o=d.get('roofline_one_in_flight',{}); print('$name', d['value'], d['ms_per_step'], r['kernel_us'], r['frac_at_step_time'], o.get('kernel_us'), o.get('step_us'))"
}
for rep in 1 2; do
  b default_$rep
  b ie1_$rep OCTVR_HIP_LIB=$V/ie1.so
done
CFG=C4 b c4default
CFG=C4 b c4ie1 OCTVR_HIP_LIB=$V/ie1.so
echo done

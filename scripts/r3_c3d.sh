#!/bin/bash
# C3: multi-band parity on the current library, then the packed pyrUp A/B (default vs nopack variant)
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp PYTHONUNBUFFERED=1
mkdir -p gpurun_out
V=opencv-octvr_amd/lib/variants
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_fullsize.py tests/test_gpu_scaled.py -m gpu -v \
  -k "multiband or frames_in_flight or fullsize or feather or scaled or preview" --timeout 300 --timeout-method thread \
  -p no:cacheprovider > gpurun_out/c3a_tests.log 2>&1 || { echo "tests rc=$?"; grep -E "FAILED|passed|failed" gpurun_out/c3a_tests.log | tail -20; exit 1; }
grep -E "passed|failed" gpurun_out/c3a_tests.log | tail -1
b() {
  local name=$1; shift
  env "$@" timeout -k 10 240 python bench.py --config C3 --steps 40 --warmup 5 --no-cpu-baseline --no-async-e2e \
      > gpurun_out/c3a_$name.log 2>&1 || { echo "$name rc=$?"; tail -5 gpurun_out/c3a_$name.log; exit 1; }
  python3 -c "import json; d=json.loads(open('gpurun_out/c3a_$name.log').read().strip().splitlines()[-1]); r=d['roofline']; print('$name', d['value'], d['ms_per_step'], r['kernel_us'], r.get('frac'), r.get('frac_at_step_time'))"
}
for rep in 1 2; do
  b cur_$rep
  b nolf_$rep OCTVR_HIP_LIB=$PWD/$V/nolf.so
  b cf_$rep OCTVR_HIP_LIB=$PWD/$V/cf.so
done
echo done

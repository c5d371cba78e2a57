#!/bin/bash
# Round 3 A/B 18: multi-band unread tiles (levels >= 1 read by no collapse: no blend, no Gaussian blocks)
# vs the r03h library.  Multi-band / full-size / deep tests first, then C3 interleaved.
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp PYTHONUNBUFFERED=1
mkdir -p gpurun_out
V=$PWD/opencv-octvr_amd/lib/variants
timeout -k 10 600 python -u -m pytest -x -q -s --timeout 400 --timeout-method thread -p no:cacheprovider -m gpu \
  tests/test_gpu_fullsize.py tests/test_gpu_parity.py tests/test_gpu_scaled.py tests/test_gpu_vignette.py tests/test_gpu_async.py \
  > gpurun_out/ab18_tests.log 2>&1; rc=$?
grep -E "passed|failed|\[\[|\{\(" gpurun_out/ab18_tests.log | tail -4
[ $rc -eq 0 ] || { grep -E "^E |FAILED" gpurun_out/ab18_tests.log | head -20; exit 1; }
b() {  # name cfg [env...]
  local name=$1 cfg=$2; shift 2
  env "$@" timeout -k 10 240 python bench.py --config $cfg --steps 30 --warmup 5 --no-cpu-baseline --no-async-e2e \
      > gpurun_out/ab18_$name.log 2>&1 || { echo "$name rc=$?"; tail -5 gpurun_out/ab18_$name.log; exit 1; }
  python3 -c "import json; d=json.loads(open('gpurun_out/ab18_$name.log').read().strip().splitlines()[-1]); r=d['roofline']; o=d.get('roofline_one_in_flight',{}); print('$name', d['value'], d['ms_per_step'], r['kernel_us'], o.get('kernel_us'), o.get('step_us'), [(t.get('owned_tiles'), t.get('deep_tiles'), t.get('unread_tiles'), t.get('down_items')) for t in d['mapper'].get('level_tiles', [])])"
}
for rep in 1 2 3; do
  b base_C3_$rep C3 OCTVR_HIP_LIB=$V/base.so
  b new_C3_$rep C3
done
echo done

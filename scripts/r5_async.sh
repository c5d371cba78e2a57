#!/bin/bash
# Round 5: AsyncMultiMapper footprint upload — the async GPU tests, then async_e2e on C2 interleaved
# between the in-tree library and VARIANTS (scripts/async_ab.py).
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp PYTHONUNBUFFERED=1
mkdir -p gpurun_out
TAG=${TAG:-r5a}
V=$PWD/opencv-octvr_amd/lib/variants
timeout -k 10 600 python -u -m pytest tests/test_gpu_async.py -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider \
  > gpurun_out/${TAG}_tests.log 2>&1 || { grep -E "^E |FAILED" gpurun_out/${TAG}_tests.log | head -20; exit 1; }
tail -1 gpurun_out/${TAG}_tests.log
for rep in $(seq 1 ${REPS:-2}); do
  for v in ${VARIANTS:-} cur; do
    lib=; [ "$v" != cur ] && lib="OCTVR_HIP_LIB=$V/$v.so"
    env $lib timeout -k 10 200 python scripts/async_ab.py ${FRAMES:-48} >> gpurun_out/${TAG}_ab.log 2>&1 || { echo "$v rc=$?"; tail -5 gpurun_out/${TAG}_ab.log; exit 1; }
  done
done
cat gpurun_out/${TAG}_ab.log

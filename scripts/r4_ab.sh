#!/bin/bash
# Round 4 box session: the GPU suite against variant $TV (OCTVR_HIP_LIB, if set), then scripts/ab.sh.
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp PYTHONUNBUFFERED=1
mkdir -p gpurun_out
TAG=${TAG:-ab}
if [ -n "$TV" ]; then
  OCTVR_HIP_LIB=$PWD/opencv-octvr_amd/lib/variants/$TV.so timeout -k 10 700 python -u -m pytest ${TESTS:-tests} -m gpu -x -q \
    --timeout 400 --timeout-method thread -p no:cacheprovider > gpurun_out/${TAG}_tests_$TV.log 2>&1; rc=$?
  grep -E "passed|failed" gpurun_out/${TAG}_tests_$TV.log | tail -1
  [ $rc -eq 0 ] || { grep -E "^E |FAILED" gpurun_out/${TAG}_tests_$TV.log | head -20; exit 1; }
fi
TESTS= bash scripts/ab.sh

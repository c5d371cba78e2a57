#!/bin/bash
# Round 3 check 17: the deep-tile shortcut against the pyrUp path on C3 noise frames, then the deep tests.
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp PYTHONUNBUFFERED=1
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -v -s --timeout 400 --timeout-method thread -p no:cacheprovider \
  tests/test_gpu_fullsize.py::test_gpu_c3_deep_tiles_equal_pyrup_path tests/test_gpu_parity.py::test_gpu_multiband_deep_tiles \
  > gpurun_out/ab17_tests.log 2>&1; rc=$?
grep -E "passed|failed|\[\[|\{\(" gpurun_out/ab17_tests.log | tail -5
[ $rc -eq 0 ] || { grep -E "^E " gpurun_out/ab17_tests.log | head -20; exit 1; }
echo done

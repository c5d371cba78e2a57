#!/bin/bash
# AsyncMultiMapper: GPU tests, then the copy/compute trace of C2 end to end
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp PYTHONUNBUFFERED=1
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_async.py tests/test_gpu_cpp_api.py -m gpu -v --timeout 240 --timeout-method thread \
  -p no:cacheprovider > gpurun_out/as_tests.log 2>&1 || { echo "tests rc=$?"; grep -E "FAILED|passed|failed" gpurun_out/as_tests.log | tail; exit 1; }
grep -E "passed|failed" gpurun_out/as_tests.log | tail -1
timeout -k 10 120 python3 scripts/async_trace.py --config C2 --frames 24 > gpurun_out/as_plain.log 2>&1 || { echo "plain rc=$?"; tail -3 gpurun_out/as_plain.log; exit 1; }
tail -1 gpurun_out/as_plain.log
timeout -s KILL 240 rocprofv3 --kernel-trace --memory-copy-trace --output-format csv -d gpurun_out/as_trace -o run -- \
  python3 scripts/async_trace.py --config C2 --frames 16 > gpurun_out/as_trace.log 2>&1 || { echo "trace rc=$?"; tail -5 gpurun_out/as_trace.log; exit 1; }
python3 scripts/async_trace.py --analyze gpurun_out/as_trace
echo done

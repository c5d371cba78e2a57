#!/bin/bash
# GPU tests on one box: `scripts/gpu_tests.sh [pytest args...]` (default: the whole -m gpu suite), the log
# under gpurun_out/tests_<tag>.log (TAG env, default "run").  Stops at the first failure.
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp PYTHONUNBUFFERED=1
mkdir -p gpurun_out
TAG=${TAG:-run}
if [ $# -eq 0 ]; then set -- tests -m gpu; fi
timeout -k 10 ${LIMIT:-900} python -u -m pytest "$@" -x -v --timeout 400 --timeout-method thread -p no:cacheprovider \
  > gpurun_out/tests_$TAG.log 2>&1
rc=$?
grep -E "passed|failed|error" gpurun_out/tests_$TAG.log | tail -3
[ $rc -ne 0 ] && grep -E "^E |FAILED|Error" gpurun_out/tests_$TAG.log | head -20
exit $rc

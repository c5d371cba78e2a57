#!/bin/bash
# Round 5: the GPU suite on the in-tree library (stops on the first failure), then an interleaved A/B of
# library variants (scripts/ab.sh; VARIANTS / CONFIGS / REPS) on the same box.
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp PYTHONUNBUFFERED=1
mkdir -p gpurun_out
TAG=${TAG:-r5}
if [ -n "${TESTS:-tests}" ] && [ "${TESTS}" != "none" ]; then
  timeout -k 10 900 python -u -m pytest ${TESTS:-tests} -m gpu -x -q --timeout 400 --timeout-method thread -p no:cacheprovider \
    > gpurun_out/${TAG}_tests.log 2>&1 || { grep -E "^E |FAILED" gpurun_out/${TAG}_tests.log | head -20; exit 1; }
  tail -1 gpurun_out/${TAG}_tests.log
fi
[ -n "$VARIANTS" ] || exit 0
TESTS= VARIANTS="$VARIANTS" CONFIGS="${CONFIGS:-C2}" REPS=${REPS:-2} TAG=$TAG bash scripts/ab.sh

#!/bin/bash
# round 3: GPU test suite (incl. the bit-exact LUT + full-size tests) then a short C2 bench
cd "$GRAFT_REPO_ROOT" || exit 1
export PYTHONUNBUFFERED=1
timeout -k 10 1080 python -u -m pytest tests -m gpu -v --maxfail=40 --timeout 400 --timeout-method thread \
    -p no:cacheprovider > gpurun_out/r3_t1_tests.log 2>&1
rc=$?
echo "tests rc=$rc" >> gpurun_out/r3_t1_tests.log
exit $rc

#!/bin/bash
# round 3 (session 2) final v5, part 1 (the library as committed): GPU test suite, PMC traffic for C2/C3/C4, and
# rocprofv3 kernel-trace --stats of the three bench configs.  Part 2 (bench lines) runs after the PMC
# summaries are written into profiles/ (scripts/pmc_summary.py), so `roofline.traffic` is filled.
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp PYTHONUNBUFFERED=1
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -v --timeout 400 --timeout-method thread -p no:cacheprovider \
  > gpurun_out/f11_tests.log 2>&1; rc=$?
grep -E "passed|failed" gpurun_out/f11_tests.log | tail -1
[ $rc -eq 0 ] || { grep -E "^FAILED" gpurun_out/f11_tests.log | head -20; exit 1; }
for CFG in C2 C3 C4; do
  CFG=$CFG bash scripts/pmc.sh > gpurun_out/f11_pmc_$CFG.log 2>&1 || { echo "pmc $CFG failed"; tail -5 gpurun_out/f11_pmc_$CFG.log; exit 1; }
done
echo pmc ok
for CFG in C2 C3 C4; do
  timeout -s KILL 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/f11_kt_$CFG -o run -- \
    python3 bench.py --config $CFG --steps 30 --warmup 5 --no-cpu-baseline --no-async-e2e > gpurun_out/f11_kt_$CFG.log 2>&1 \
    || { echo "kt $CFG rc=$?"; tail -5 gpurun_out/f11_kt_$CFG.log; exit 1; }
  timeout -s KILL 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/f11_kt1_$CFG -o run -- \
    python3 bench.py --config $CFG --steps 20 --warmup 3 --no-cpu-baseline --no-async-e2e --inflight 1 > gpurun_out/f11_kt1_$CFG.log 2>&1 \
    || { echo "kt1 $CFG rc=$?"; tail -5 gpurun_out/f11_kt1_$CFG.log; exit 1; }
done
echo done

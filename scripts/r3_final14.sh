#!/bin/bash
# round 3 final (deep + unread tiles library), one call: GPU test suite, PMC traffic for C2/C3/C4 summarised on the box
# into profiles/r03i_pmc_*.json (copied to gpurun_out/ to bring back), rocprofv3 kernel-trace --stats of the
# three configs (three frames in flight; C3 also one), then the bench lines, which read those summaries.
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp PYTHONUNBUFFERED=1
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -v --timeout 400 --timeout-method thread -p no:cacheprovider \
  > gpurun_out/f14_tests.log 2>&1; rc=$?
grep -E "passed|failed" gpurun_out/f14_tests.log | tail -1
[ $rc -eq 0 ] || { grep -E "^FAILED" gpurun_out/f14_tests.log | head -20; exit 1; }
for CFG in C2 C3 C4; do
  CFG=$CFG bash scripts/pmc.sh > gpurun_out/f14_pmc_$CFG.log 2>&1 || { echo "pmc $CFG failed"; tail -5 gpurun_out/f14_pmc_$CFG.log; exit 1; }
  python3 scripts/pmc_summary.py $CFG r03i > gpurun_out/f14_pmcsum_$CFG.log 2>&1 || { echo "pmc_summary $CFG failed"; tail -5 gpurun_out/f14_pmcsum_$CFG.log; exit 1; }
  cp profiles/r03i_pmc_$CFG.json gpurun_out/
done
echo pmc ok
for CFG in C2 C3 C4; do
  timeout -s KILL 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/f14_kt_$CFG -o run -- \
    python3 bench.py --config $CFG --steps 30 --warmup 5 --no-cpu-baseline --no-async-e2e > gpurun_out/f14_kt_$CFG.log 2>&1 \
    || { echo "kt $CFG rc=$?"; tail -5 gpurun_out/f14_kt_$CFG.log; exit 1; }
done
timeout -s KILL 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/f14_kt1_C3 -o run -- \
  python3 bench.py --config C3 --steps 20 --warmup 3 --no-cpu-baseline --no-async-e2e --inflight 1 > gpurun_out/f14_kt1_C3.log 2>&1 \
  || { echo "kt1 C3 rc=$?"; tail -5 gpurun_out/f14_kt1_C3.log; exit 1; }
echo kt ok
for CFG in C2 C3 C4; do
  timeout -k 10 400 python bench.py --config $CFG > gpurun_out/f14_bench_$CFG.json 2> gpurun_out/f14_bench_$CFG.err || { echo "$CFG rc=$?"; tail -5 gpurun_out/f14_bench_$CFG.err; exit 1; }
  tail -1 gpurun_out/f14_bench_$CFG.json | cut -c1-400
done
echo done

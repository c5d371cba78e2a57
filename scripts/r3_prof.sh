#!/bin/bash
# round 3 profiles of the current library: PMC traffic (FETCH/WRITE, separate passes) for C2, C3, C4,
# rocprofv3 kernel-trace --stats of each bench config, and the AsyncMultiMapper copy/compute trace.
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp PYTHONUNBUFFERED=1
mkdir -p gpurun_out
for CFG in C2 C3 C4; do
  CFG=$CFG bash scripts/pmc.sh > gpurun_out/prof_pmc_$CFG.log 2>&1 || { echo "pmc $CFG failed"; tail -5 gpurun_out/prof_pmc_$CFG.log; exit 1; }
  echo "pmc $CFG ok"
done
for CFG in C2 C3 C4; do
  timeout -s KILL 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_kt_$CFG -o run -- \
    python3 bench.py --config $CFG --steps 30 --warmup 5 --no-cpu-baseline --no-async-e2e > gpurun_out/prof_kt_$CFG.log 2>&1 \
    || { echo "kt $CFG rc=$?"; tail -5 gpurun_out/prof_kt_$CFG.log; exit 1; }
  echo "kt $CFG: $(tail -1 gpurun_out/prof_kt_$CFG.log | cut -c1-200)"
done
timeout -s KILL 240 rocprofv3 --kernel-trace --memory-copy-trace --output-format csv -d gpurun_out/prof_async -o run -- \
  python3 scripts/async_trace.py --config C2 --frames 12 > gpurun_out/prof_async.log 2>&1 || { echo "async rc=$?"; tail -5 gpurun_out/prof_async.log; exit 1; }
python3 scripts/async_trace.py --analyze gpurun_out/prof_async >> gpurun_out/prof_async.log 2>&1
echo done

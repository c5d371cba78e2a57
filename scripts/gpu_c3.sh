#!/bin/bash
# C3 (multi-band blend=16) bench + kernel trace on the GPU box.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python bench.py --config C3 --steps 20 --warmup 3 ${C3_BENCH_ARGS} > gpurun_out/bench_c3.log 2>&1 || { echo "bench rc=$?"; tail -20 gpurun_out/bench_c3.log; exit 1; }
tail -2 gpurun_out/bench_c3.log
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_c3 -o run --output-format csv -- python3 bench.py --config C3 --steps 10 --warmup 2 --no-cpu-baseline > gpurun_out/prof_c3.log 2>&1 || { echo "prof rc=$?"; tail -20 gpurun_out/prof_c3.log; exit 1; }
cat gpurun_out/prof_c3/run_kernel_stats.csv

#!/bin/bash
# bench one configuration (+ rocprof kernel stats): CFG=C4 bash scripts/gpu_cfg.sh
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
CFG=${CFG:-C2}
timeout -k 10 900 python bench.py --config $CFG --steps ${STEPS:-20} --warmup 3 ${BENCH_ARGS} > gpurun_out/bench_$CFG.log 2>&1 || { echo "bench rc=$?"; tail -20 gpurun_out/bench_$CFG.log; exit 1; }
tail -1 gpurun_out/bench_$CFG.log
[ -n "$NOPROF" ] && exit 0
timeout -k 10 900 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_$CFG -o run --output-format csv -- python3 bench.py --config $CFG --steps 10 --warmup 2 --no-cpu-baseline > gpurun_out/prof_$CFG.log 2>&1 || { echo "prof rc=$?"; tail -20 gpurun_out/prof_$CFG.log; exit 1; }
cat gpurun_out/prof_$CFG/run_kernel_stats.csv

#!/bin/bash
# C3 per-level breakdown: kernel trace with one frame in flight, SQ counters of every mb_blend dispatch
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp PYTHONUNBUFFERED=1
mkdir -p gpurun_out
timeout -s KILL 180 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/c3b_kt -o run -- \
  python3 bench.py --config C3 --steps 10 --warmup 3 --no-cpu-baseline --no-async-e2e --inflight 1 > gpurun_out/c3b_kt.log 2>&1 || { echo "kt rc=$?"; tail -5 gpurun_out/c3b_kt.log; exit 1; }
echo kt ok
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_SMEM SQ_ACTIVE_INST_SCA \
  --kernel-include-regex "mb_blend|mb_down|stitch_tiled" -d gpurun_out/c3b_sq -o run --output-format csv -- python3 bench.py --config C3 --pmc-child --steps 3 --inflight 1 > gpurun_out/c3b_sq.log 2>&1 || { echo "sq rc=$?"; tail -5 gpurun_out/c3b_sq.log; exit 1; }
echo sq ok
timeout -s KILL 180 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/c4b_kt -o run -- \
  python3 bench.py --config C4 --steps 10 --warmup 3 --no-cpu-baseline --no-async-e2e --inflight 1 > gpurun_out/c4b_kt.log 2>&1 || { echo "kt4 rc=$?"; tail -5 gpurun_out/c4b_kt.log; exit 1; }
echo done

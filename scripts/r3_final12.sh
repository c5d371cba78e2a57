#!/bin/bash
# round 3 (session 2) final v5, part 2: the bench lines (PMC summaries for this library already in profiles/)
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp PYTHONUNBUFFERED=1
mkdir -p gpurun_out
timeout -k 10 400 python bench.py > gpurun_out/f12_bench_C2.json 2> gpurun_out/f12_bench_C2.err || { echo "C2 rc=$?"; tail -5 gpurun_out/f12_bench_C2.err; exit 1; }
tail -1 gpurun_out/f12_bench_C2.json | cut -c1-300
for CFG in C3 C4; do
  timeout -k 10 400 python bench.py --config $CFG > gpurun_out/f12_bench_$CFG.json 2> gpurun_out/f12_bench_$CFG.err || { echo "$CFG rc=$?"; tail -5 gpurun_out/f12_bench_$CFG.err; exit 1; }
  tail -1 gpurun_out/f12_bench_$CFG.json | cut -c1-300
done
echo done

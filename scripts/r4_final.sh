#!/bin/bash
# Round 4 evidence session for the in-tree library: GPU suite, the default bench line (as the driver runs
# it) and one per config, then kernel traces + PMC passes (scripts/r4_prof.sh).  Any failure ends it.
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp PYTHONUNBUFFERED=1
mkdir -p gpurun_out
TAG=${TAG:-r04b}
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 400 --timeout-method thread -p no:cacheprovider \
  > gpurun_out/${TAG}_tests.log 2>&1 || { grep -E "^E |FAILED" gpurun_out/${TAG}_tests.log | head; exit 1; }
tail -1 gpurun_out/${TAG}_tests.log
timeout -k 10 400 python bench.py > gpurun_out/${TAG}_bench_default.json 2> gpurun_out/${TAG}_bench_default.err || { tail -5 gpurun_out/${TAG}_bench_default.err; exit 1; }
for CFG in ${CONFIGS:-C1 C2 C3 C4 F2}; do
  timeout -k 10 300 python bench.py --config $CFG --steps 50 --warmup 5 --no-async-e2e \
    > gpurun_out/${TAG}_bench_$CFG.json 2> gpurun_out/${TAG}_bench_$CFG.err || { echo "$CFG rc=$?"; tail -5 gpurun_out/${TAG}_bench_$CFG.err; exit 1; }
  python3 -c "import json; d=json.loads(open('gpurun_out/${TAG}_bench_$CFG.json').read().strip().splitlines()[-1]); print('$CFG', d['value'], d['ms_per_step'], d['roofline']['frac'], d['roofline'].get('frac_at_step_time'))"
done
TAG=$TAG CONFIGS="C3" INFLIGHTS="1 3" PASSES="FETCH WRITE SQ1" bash scripts/r4_prof.sh || exit 1
TAG=$TAG CONFIGS="C2 C4" INFLIGHTS="3" PASSES="FETCH WRITE SQ1 SQ2 TCC" bash scripts/r4_prof.sh || exit 1
TAG=$TAG CONFIGS="C1 F2" INFLIGHTS="3" PASSES="FETCH WRITE" bash scripts/r4_prof.sh || exit 1
echo done

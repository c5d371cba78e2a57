#!/bin/bash
# Round 4 box session: the GPU suite (or a subset: TESTS=...), then bench lines for CONFIGS (default C2 C3 C4).
# Each GPU step has its own time limit; any failure ends the script.
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp PYTHONUNBUFFERED=1
mkdir -p gpurun_out
TAG=${TAG:-chk}
TESTS=${TESTS:-tests}
if [ "$TESTS" != "none" ]; then
  timeout -k 10 700 python -u -m pytest $TESTS -m gpu -x -v --timeout 400 --timeout-method thread -p no:cacheprovider \
    > gpurun_out/${TAG}_tests.log 2>&1; rc=$?
  grep -E "passed|failed" gpurun_out/${TAG}_tests.log | tail -1
  [ $rc -eq 0 ] || { grep -E "^FAILED|^E " gpurun_out/${TAG}_tests.log | head -20; exit 1; }
fi
for CFG in ${CONFIGS:-C2 C3 C4}; do
  timeout -k 10 300 python bench.py --config $CFG --steps 30 --warmup 5 --no-cpu-baseline --no-async-e2e $BENCH_ARGS \
    > gpurun_out/${TAG}_bench_$CFG.json 2> gpurun_out/${TAG}_bench_$CFG.err || { echo "$CFG rc=$?"; tail -5 gpurun_out/${TAG}_bench_$CFG.err; exit 1; }
  python3 -c "import json,sys; d=json.loads(open('gpurun_out/${TAG}_bench_$CFG.json').read().strip().splitlines()[-1]); r=d['roofline']; o=d.get('roofline_one_in_flight',{}); print('$CFG', d['value'], d['ms_per_step'], r['kernel_us'], r['frac'], o.get('kernel_us'), o.get('step_us'))"
done
echo done

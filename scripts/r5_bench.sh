#!/bin/bash
# Bench lines of the in-tree library: optional GPU tests first, the default line (as the driver runs it),
# then per config (REPS each).  Every GPU step has its own time limit; any failure ends the script.
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp PYTHONUNBUFFERED=1
mkdir -p gpurun_out
TAG=${TAG:-r5}
if [ -n "$TESTS" ]; then
  timeout -k 10 900 python -u -m pytest $TESTS -m gpu -x -q --timeout 400 --timeout-method thread -p no:cacheprovider \
    > gpurun_out/${TAG}_tests.log 2>&1 || { grep -E "^E |FAILED" gpurun_out/${TAG}_tests.log | head -20; exit 1; }
  tail -1 gpurun_out/${TAG}_tests.log
fi
if [ -z "$NO_DEFAULT" ]; then
  timeout -k 10 500 python bench.py > gpurun_out/${TAG}_bench_default.json 2> gpurun_out/${TAG}_bench_default.err \
    || { tail -5 gpurun_out/${TAG}_bench_default.err; exit 1; }
  python3 -c "import json; d=json.loads(open('gpurun_out/${TAG}_bench_default.json').read().strip().splitlines()[-1]); print('default', d['value'], d['ms_per_step'], d.get('host_issue_ms_per_step'), d['roofline']['kernel_us'], d.get('async_e2e',{}).get('value'), d.get('cpu_baseline',{}).get('value'))"
fi
for rep in $(seq 1 ${REPS:-1}); do
for CFG in ${CONFIGS:-C2}; do
  n=${TAG}_bench_${CFG}_$rep
  timeout -k 10 300 python bench.py --config $CFG --steps ${STEPS:-50} --warmup 5 --no-cpu-baseline --no-async-e2e $BENCH_ARGS \
    > gpurun_out/$n.json 2> gpurun_out/$n.err || { echo "$CFG rc=$?"; tail -5 gpurun_out/$n.err; exit 1; }
  python3 -c "import json; d=json.loads(open('gpurun_out/$n.json').read().strip().splitlines()[-1]); print('$CFG $rep', d['value'], d['ms_per_step'], d.get('host_issue_ms_per_step'), d['roofline']['kernel_us'], d['roofline'].get('frac'))"
done
done
echo done

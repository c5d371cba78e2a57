#!/bin/bash
# Round-end rehearsal on one box: the GPU suite, smoke(), then the default bench line three times.
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp PYTHONUNBUFFERED=1
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 400 --timeout-method thread -p no:cacheprovider \
  > gpurun_out/final_tests.log 2>&1 || { grep -E "^E |FAILED" gpurun_out/final_tests.log | head; exit 1; }
tail -1 gpurun_out/final_tests.log
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" || exit 1
for rep in 1 2 3; do
  timeout -k 10 200 python bench.py --no-cpu-baseline --no-async-e2e > gpurun_out/final_bench_$rep.json 2>/dev/null || exit 1
  python3 -c "import json; d=json.loads(open('gpurun_out/final_bench_$rep.json').read().strip().splitlines()[-1]); r=d['roofline']; print('default', $rep, d['value'], d['ms_per_step'], r['kernel_us'], r['frac'], r.get('traffic_source'))"
done

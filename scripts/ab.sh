#!/bin/bash
# Interleaved A/B of library variants on one box (the only comparison this pool's box-to-box spread
# allows).  Variants are built beforehand with scripts/build_variant.sh NAME -D... (base = the default
# flags); the in-tree library is "cur".
#   VARIANTS="base cur x" CONFIGS="C2 C4" REPS=3 [TESTS=<pytest args>] [TAG=ab] bash scripts/ab.sh
# Optional TESTS runs those GPU tests first (against the in-tree library) and stops on a failure.
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp PYTHONUNBUFFERED=1
mkdir -p gpurun_out
TAG=${TAG:-ab}
V=$PWD/opencv-octvr_amd/lib/variants
if [ -n "$TESTS" ]; then
  timeout -k 10 600 python -u -m pytest -x -q --timeout 400 --timeout-method thread -p no:cacheprovider -m gpu $TESTS \
    > gpurun_out/${TAG}_tests.log 2>&1; rc=$?
  grep -E "passed|failed" gpurun_out/${TAG}_tests.log | tail -1
  [ $rc -eq 0 ] || { grep -E "^E |FAILED" gpurun_out/${TAG}_tests.log | head -20; exit 1; }
fi
for rep in $(seq 1 ${REPS:-3}); do
  for cfg in ${CONFIGS:-C2}; do
    for v in ${VARIANTS:-cur}; do
      lib=; [ "$v" != cur ] && lib="OCTVR_HIP_LIB=$V/$v.so"
      env $lib timeout -k 10 240 python bench.py --config $cfg --steps ${STEPS:-30} --warmup 5 --no-cpu-baseline --no-async-e2e $BENCH_ARGS \
        > gpurun_out/${TAG}_${v}_${cfg}_$rep.log 2>&1 || { echo "$v $cfg rc=$?"; tail -5 gpurun_out/${TAG}_${v}_${cfg}_$rep.log; exit 1; }
      python3 -c "import json; d=json.loads(open('gpurun_out/${TAG}_${v}_${cfg}_$rep.log').read().strip().splitlines()[-1]); r=d['roofline']; o=d.get('roofline_one_in_flight',{}); print('$v $cfg $rep', d['value'], d['ms_per_step'], r['kernel_us'], o.get('kernel_us'), o.get('step_us'))"
    done
  done
done
echo done

#!/bin/bash
# Round 3 A/B 16: multi-band deep tiles (R = G where one camera of weight 1 covers every pyrUp tap up the
# pyramid; mb_blend skips both pyrUps there) vs the committed library.  Full GPU suite first, then C3
# interleaved, then C2 once each (the composite is unchanged; a sanity check).
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp PYTHONUNBUFFERED=1
mkdir -p gpurun_out
V=$PWD/opencv-octvr_amd/lib/variants
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 400 --timeout-method thread -p no:cacheprovider -s \
  > gpurun_out/ab16_tests.log 2>&1 || { echo "tests rc=$?"; grep -E "FAILED|Error|assert" gpurun_out/ab16_tests.log | head -20; tail -5 gpurun_out/ab16_tests.log; exit 1; }
tail -1 gpurun_out/ab16_tests.log; grep "rigA" gpurun_out/ab16_tests.log | head -2
b() {  # name cfg [env...]
  local name=$1 cfg=$2; shift 2
  env "$@" timeout -k 10 240 python bench.py --config $cfg --steps 30 --warmup 5 --no-cpu-baseline --no-async-e2e \
      > gpurun_out/ab16_$name.log 2>&1 || { echo "$name rc=$?"; tail -5 gpurun_out/ab16_$name.log; exit 1; }
  python3 -c "import json; d=json.loads(open('gpurun_out/ab16_$name.log').read().strip().splitlines()[-1]); r=d['roofline']; o=d.get('roofline_one_in_flight',{}); print('$name', d['value'], d['ms_per_step'], r['kernel_us'], o.get('kernel_us'), o.get('step_us'), [(t.get('owned_tiles'), t.get('deep_tiles')) for t in d['mapper'].get('level_tiles', [])])"
}
for rep in 1 2 3; do
  b base_C3_$rep C3 OCTVR_HIP_LIB=$V/base.so
  b new_C3_$rep C3
done
b base_C2 C2 OCTVR_HIP_LIB=$V/base.so
b new_C2 C2
echo done

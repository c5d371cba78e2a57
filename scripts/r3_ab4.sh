#!/bin/bash
# Round 3 A/B 4: multi-band owned-tile fast path on every level (C3) vs the committed library; blend parity.
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
V=$PWD/opencv-octvr_amd/lib/variants
b() {  # name cfg [env...]
  local name=$1 cfg=$2; shift 2
  env "$@" timeout -k 10 240 python bench.py --config $cfg --steps 30 --warmup 5 --no-cpu-baseline --no-async-e2e \
      > gpurun_out/ab4_$name.log 2>&1 || { echo "$name rc=$?"; tail -5 gpurun_out/ab4_$name.log; exit 1; }
  python3 -c "import json; d=json.loads(open('gpurun_out/ab4_$name.log').read().strip().splitlines()[-1]); r=d['roofline']; o=d.get('roofline_one_in_flight',{}); print('$name', d['value'], d['ms_per_step'], r['kernel_us'], r['frac_at_step_time'], o.get('kernel_us'), o.get('step_us'), d['mapper'].get('level_tiles', [{}])[0])"
}
for rep in 1 2 3; do
  b base_C3_$rep C3 OCTVR_HIP_LIB=$V/base.so
  b new_C3_$rep C3
done
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_parity.py tests/test_gpu_fullsize.py tests/test_gpu_scaled.py tests/test_gpu_morph.py tests/test_gpu_vignette.py > gpurun_out/ab4_tests.log 2>&1 || { echo "tests rc=$?"; tail -30 gpurun_out/ab4_tests.log; exit 1; }
tail -2 gpurun_out/ab4_tests.log
echo done
# C2: staging phase at raised wave priority
for rep in 1 2; do
  b base_C2_$rep C2 OCTVR_HIP_LIB=$V/base.so
  b prio2_C2_$rep C2 OCTVR_HIP_LIB=$V/prio2.so
  b prio3_C2_$rep C2 OCTVR_HIP_LIB=$V/prio3.so
  b new_C2_$rep C2
done
echo done2

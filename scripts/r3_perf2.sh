#!/bin/bash
# C2 composite variants: XCD band balance by staging chunks, 5 workgroups per CU; plus smoke()
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp PYTHONUNBUFFERED=1
mkdir -p gpurun_out
V=opencv-octvr_amd/lib/variants
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/p2_smoke.log 2>&1 || { echo "smoke rc=$?"; tail -5 gpurun_out/p2_smoke.log; exit 1; }
tail -1 gpurun_out/p2_smoke.log
b() {
  local name=$1; shift
  env "$@" timeout -k 10 240 python bench.py --config ${CFG:-C2} --steps 60 --warmup 5 --no-cpu-baseline --no-async-e2e \
      > gpurun_out/p2_$name.log 2>&1 || { echo "$name rc=$?"; tail -5 gpurun_out/p2_$name.log; exit 1; }
  python3 -c "import json; d=json.loads(open('gpurun_out/p2_$name.log').read().strip().splitlines()[-1]); r=d['roofline']; print('$name', d['value'], d['ms_per_step'], r['kernel_us'], r['frac_at_step_time'], d.get('roofline_one_in_flight',{}).get('kernel_us'), d['mapper']['band_chunks'])"
}
for rep in 1 2; do
  b default_$rep
  b cw03_$rep OCTVR_HIP_LIB=$PWD/$V/cw03.so
  b cw1_$rep OCTVR_HIP_LIB=$PWD/$V/cw1.so
  b bpc5_$rep OCTVR_HIP_LIB=$PWD/$V/bpc5.so
done
echo done

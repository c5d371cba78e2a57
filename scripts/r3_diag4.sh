#!/bin/bash
# Price an opcode inside the composite loop: +4 independent instructions of one kind per pixel
# (OCTVR_DIAG_XOP 1 xor, 2 pk_mul_lo_u16, 3 perm, 4 mul_u32_u24, 5 dot2_u32_u16, 6 pk_add_u16,
# 7 cvt_pk_u8_f32) against the default build, interleaved, C2 one and three frames in flight.
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp PYTHONUNBUFFERED=1
mkdir -p gpurun_out
V=$PWD/opencv-octvr_amd/lib/variants
b() {  # name [env...]
  local name=$1; shift
  env "$@" timeout -k 10 240 python bench.py --config C2 --steps 60 --warmup 5 --no-cpu-baseline --no-async-e2e \
      > gpurun_out/d4_$name.log 2>&1 || { echo "$name rc=$?"; tail -5 gpurun_out/d4_$name.log; exit 1; }
  python3 -c "import json; d=json.loads(open('gpurun_out/d4_$name.log').read().strip().splitlines()[-1]); r=d['roofline']; o=d.get('roofline_one_in_flight',{}); print('$name', d['value'], d['ms_per_step'], r['kernel_us'], o.get('kernel_us'), o.get('step_us'))"
}
for rep in 1 2; do
  b def_$rep
  for i in 1 2 3 4 5 6 7; do b x${i}_$rep OCTVR_HIP_LIB=$V/x$i.so; done
done
echo done

#!/bin/bash
# round 3 perf batch 1: LDS row padding (bank spread) A/B on C2, phase shares, LDS conflict counters.
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
V=opencv-octvr_amd/lib/variants
b() {  # name, then env assignments (CFG overrides the config)
  local name=$1; shift
  env "$@" timeout -k 10 240 python bench.py --config ${CFG:-C2} --steps 60 --warmup 5 --no-cpu-baseline --no-async-e2e \
      > gpurun_out/p1_$name.log 2>&1 || { echo "$name rc=$?"; tail -5 gpurun_out/p1_$name.log; exit 1; }
  python3 -c "import json; d=json.loads(open('gpurun_out/p1_$name.log').read().strip().splitlines()[-1]); r=d['roofline']; print('$name', d['value'], d['ms_per_step'], r['kernel_us'], r['frac_at_step_time'], d.get('roofline_one_in_flight',{}).get('kernel_us'), d['mapper']['wide_tiles'])"
}
for rep in 1 2; do
  b default_$rep OCTVR_LDS_PAD=0
  b pad4_$rep OCTVR_LDS_PAD=4
  b b64pad2_$rep OCTVR_HIP_LIB=$PWD/$V/b64.so OCTVR_LDS_PAD=2
  b b64pad6_$rep OCTVR_HIP_LIB=$PWD/$V/b64.so OCTVR_LDS_PAD=6
  b b64pad0_$rep OCTVR_HIP_LIB=$PWD/$V/b64.so OCTVR_LDS_PAD=0
  b taps_$rep OCTVR_HIP_LIB=$PWD/$V/tapsfirst.so OCTVR_LDS_PAD=0
  b tapspad4_$rep OCTVR_HIP_LIB=$PWD/$V/tapsfirst.so OCTVR_LDS_PAD=4
done
for rep in 1 2; do
  CFG=C3 b c3arith_$rep OCTVR_LDS_PAD=0
  CFG=C3 b c3table_$rep OCTVR_HIP_LIB=$PWD/$V/tabtaps.so OCTVR_LDS_PAD=0
done
OCTVR_HIP_LIB=$PWD/$V/phases.so timeout -k 10 240 python scripts/phases.py --config C2 > gpurun_out/p1_phases.log 2>&1 || { echo "phases rc=$?"; tail -5 gpurun_out/p1_phases.log; }
OCTVR_LDS_PAD=4 OCTVR_HIP_LIB=$PWD/$V/phases.so timeout -k 10 240 python scripts/phases.py --config C2 > gpurun_out/p1_phases_pad4.log 2>&1 || { echo "phases rc=$?"; tail -5 gpurun_out/p1_phases_pad4.log; }
for P in 0 4; do
  OCTVR_LDS_PAD=$P timeout -s KILL 120 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_WAVE_CYCLES SQ_INSTS_VALU SQ_INSTS_LDS --kernel-include-regex stitch_tiled -d gpurun_out/p1_sq_pad$P -o run --output-format csv -- python3 bench.py --config C2 --pmc-child --steps 5 > gpurun_out/p1_sq_pad$P.log 2>&1 || { echo "sq pad$P rc=$?"; tail -5 gpurun_out/p1_sq_pad$P.log; exit 1; }
done
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_INSTS_SALU SQ_BUSY_CYCLES --kernel-include-regex "mb_blend|mb_down" -d gpurun_out/p1_sq_c3 -o run --output-format csv -- python3 bench.py --config C3 --pmc-child --steps 5 > gpurun_out/p1_sq_c3.log 2>&1 || { echo "sq c3 rc=$?"; tail -5 gpurun_out/p1_sq_c3.log; exit 1; }
for K in 3 4; do
  timeout -s KILL 180 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/p1_kt_if$K -o run -- python3 bench.py --config C2 --steps 30 --warmup 3 --no-cpu-baseline --no-async-e2e --inflight $K > gpurun_out/p1_kt_if$K.log 2>&1 || { echo "kt if$K rc=$?"; tail -5 gpurun_out/p1_kt_if$K.log; exit 1; }
done
echo done

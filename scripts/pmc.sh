#!/bin/bash
# PMC passes over the timed kernels (MI355X_MICROARCH.md "HBM" / "rocprofv3 PMC slots"), one
# rocprofv3 --pmc run per pass, each a short `bench.py --pmc-child` run; summarised by
# scripts/pmc_summary.py into profiles/<tag>_pmc_<cfg>[_if<k>].json.  The sha256 of the profiled
# liboctvr_hip.so is recorded beside the counters, so bench.py only uses a summary of the binary it times.
#   CFG=C2|C3|C4  PASSES="FETCH WRITE SQ1 SQ2 TCC"  INFLIGHT=<streams, default 3>  STEPS=<calls>  BATCH=<frames per launch>
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
CFG=${CFG:-C2}
STEPS=${STEPS:-6}
INFLIGHT=${INFLIGHT:-3}
PASSES=${PASSES:-FETCH WRITE}
if [ -z "$RE" ]; then
  case $CFG in C3) RE="stitch_tiled|mb_down|mb_blend|gain_feed" ;; F2) RE="fast_y|fast_uv" ;; *) RE="stitch_tiled|gain_feed" ;; esac
fi
declare -A P
P[FETCH]="FETCH_SIZE"
P[WRITE]="WRITE_SIZE"
P[SQ1]="SQ_WAVE_CYCLES SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_INSTS_VALU SQ_LDS_BANK_CONFLICT SQ_INSTS_LDS GRBM_GUI_ACTIVE"
P[SQ2]="SQ_WAVES SQ_BUSY_CYCLES SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_SALU SQ_INSTS_SMEM SQ_ACTIVE_INST_ANY SQ_INSTS_LDS GRBM_GUI_ACTIVE"
P[TCC]="TCC_HIT_sum TCC_MISS_sum GRBM_GUI_ACTIVE"
BATCH=${BATCH:-1}
D=pmc_${CFG}_if${INFLIGHT}${BATCH_TAG}
sha256sum opencv-octvr_amd/lib/liboctvr_hip.so | cut -d' ' -f1 > gpurun_out/${D}_so.sha
echo "$STEPS" > gpurun_out/${D}_frames  # calls of $BATCH frames
echo "$BATCH" > gpurun_out/${D}_batch
for p in $PASSES; do
  timeout -s KILL 120 rocprofv3 --pmc ${P[$p]} --kernel-include-regex "$RE" -d gpurun_out/${D}_$p -o run --output-format csv -- \
    python3 bench.py --config $CFG --pmc-child --steps $((STEPS * BATCH)) --inflight $INFLIGHT --batch $BATCH > gpurun_out/${D}_$p.log 2>&1 \
    || { echo "pmc $p rc=$?"; tail -5 gpurun_out/${D}_$p.log; exit 1; }
done
echo "pmc $CFG if$INFLIGHT: $PASSES ok"

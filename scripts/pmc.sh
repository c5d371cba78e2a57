#!/bin/bash
# HBM traffic of the timed kernels from PMC counters (MI355X_MICROARCH.md "HBM"): FETCH_SIZE and
# WRITE_SIZE in separate passes (TCC slots), each a short --pmc-child run of bench.py.  The sha256 of
# the profiled liboctvr_hip.so is recorded beside the counters, so bench.py only uses a summary of the
# binary it is timing.   CFG=C2|C3|C4  RE=<kernel regex>  STEPS=<frames>
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
CFG=${CFG:-C2}
STEPS=${STEPS:-5}
if [ -z "$RE" ]; then
  case $CFG in C3) RE="stitch_tiled|mb_down|mb_blend|gain_feed" ;; *) RE="stitch_tiled" ;; esac
fi
sha256sum opencv-octvr_amd/lib/liboctvr_hip.so | cut -d' ' -f1 > gpurun_out/pmc_${CFG}_so.sha
echo "$STEPS" > gpurun_out/pmc_${CFG}_frames
for C in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 120 rocprofv3 --pmc $C --kernel-include-regex "$RE" -d gpurun_out/pmc_${CFG}_$C -o run --output-format csv -- python3 bench.py --config $CFG --pmc-child --steps $STEPS > gpurun_out/pmc_${CFG}_$C.log 2>&1 || { echo "pmc $C rc=$?"; tail -5 gpurun_out/pmc_${CFG}_$C.log; exit 1; }
  ls gpurun_out/pmc_${CFG}_$C
done

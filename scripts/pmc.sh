#!/bin/bash
# HBM traffic of the dominant kernel from PMC counters (MI355X_MICROARCH.md "HBM"): FETCH_SIZE and
# WRITE_SIZE in separate passes (TCC slots), each a short --pmc-child run of bench.py.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
CFG=${CFG:-C2}
RE=${RE:-stitch_tiled}
for C in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 120 rocprofv3 --pmc $C --kernel-include-regex "$RE" -d gpurun_out/pmc_${CFG}_$C -o run --output-format csv -- python3 bench.py --config $CFG --pmc-child --steps 5 > gpurun_out/pmc_${CFG}_$C.log 2>&1 || { echo "pmc $C rc=$?"; tail -5 gpurun_out/pmc_${CFG}_$C.log; exit 1; }
  ls gpurun_out/pmc_${CFG}_$C
done

#!/bin/bash
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp PYTHONUNBUFFERED=1
V=$PWD/opencv-octvr_amd/lib/variants
for L in lfcn nolf; do
  TAG=$L OCTVR_HIP_LIB=$V/$L.so timeout -k 10 120 python scripts/dbg_mb.py > gpurun_out/dbg2_$L.log 2>&1 || { echo "$L rc=$?"; tail -3 gpurun_out/dbg2_$L.log; exit 1; }
  tail -1 gpurun_out/dbg2_$L.log
done

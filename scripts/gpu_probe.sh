#!/bin/bash
# Variant benches + the per-wave phase report of a diagnostic build in one GPU session.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
CFG=${CFG:-C2} bash scripts/bench_variants.sh || exit $?
for v in ${PHASE_LIBS:-phases}; do
  f=opencv-octvr_amd/lib/variants/$v.so
  [ -f $f ] || continue
  OCTVR_HIP_LIB=$PWD/$f timeout -k 10 300 python scripts/phases.py --config ${CFG:-C2} > gpurun_out/$v.log 2>&1 || { echo "$v rc=$?"; tail -5 gpurun_out/$v.log; exit 1; }
  echo "== $v"; head -8 gpurun_out/$v.log | tail -7
done

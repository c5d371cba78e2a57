#!/bin/bash
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp PYTHONUNBUFFERED=1
V=$PWD/opencv-octvr_amd/lib/variants
for L in lfcn lfg nolf; do
  OCTVR_HIP_LIB=$V/$L.so timeout -k 10 200 python -u -m pytest tests/test_gpu_parity.py -m gpu -q -k "multiband_bit_exact and rigA" --timeout 150 --timeout-method thread -p no:cacheprovider > gpurun_out/dbg_$L.log 2>&1
  echo "$L: $(grep -E 'passed|failed' gpurun_out/dbg_$L.log | tail -1)"
done

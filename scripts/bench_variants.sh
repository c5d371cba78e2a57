#!/bin/bash
# Bench the default library and every lib/variants/*.so on one config: CFG=C2 bash scripts/bench_variants.sh
# Per library: kernel time with one frame in flight (the kernel alone) and MP/s with the bench default.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
CFG=${CFG:-C2}
run() {
  for inf in 1 2; do
    timeout -k 10 300 python bench.py --config $CFG --steps 40 --warmup 3 --no-cpu-baseline --inflight $inf ${BENCH_ARGS} > gpurun_out/var_$1_$inf.log 2>&1 || { echo "$1 failed rc=$?"; tail -5 gpurun_out/var_$1_$inf.log; exit 1; }
    python3 -c "import json; d=json.loads(open('gpurun_out/var_$1_$inf.log').read().strip().splitlines()[-1]); print('$1 inflight=$inf', d['value'], d['ms_per_step'], d['roofline']['kernel_us'])"
  done
}
run default
for f in $(ls opencv-octvr_amd/lib/variants/*.so 2>/dev/null); do
  v=$(basename $f .so)
  OCTVR_HIP_LIB=$PWD/$f run $v
done

#!/bin/bash
# One GPU-box session: parity tests, smoke, bench, rocprof kernel trace.  Each GPU step has its own
# time limit; a fault / abort / timeout stops the script (no further GPU work), a plain test failure
# does not.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
step() {  # step NAME SECONDS CMD...
  local name=$1 secs=$2; shift 2
  echo "=== $name ($(date +%T))"
  timeout -k 10 "$secs" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  echo "=== $name rc=$rc"
  tail -n 5 "gpurun_out/$name.log"
  case $rc in
    0|1) return 0 ;;          # pass / test failures: keep going
    *) echo "STOP: $name exited $rc"; exit $rc ;;
  esac
}
STEPS=${STEPS:-"pytest smoke bench prof"}
for s in $STEPS; do
  case $s in
    pytest) step pytest_gpu 900 python -m pytest tests -m gpu -q -rf ;;
    smoke)  step smoke 300 python -c "import __graft_entry__ as g; g.smoke()" ;;
    bench)  step bench 600 python bench.py --steps 30 --warmup 5 ;;
    pmc)    step pmc_fetch 300 rocprofv3 --pmc FETCH_SIZE --kernel-include-regex stitch_tiled -d gpurun_out/pmc_fetch -o run --output-format csv -- python3 bench.py --pmc-child --steps 5
            step pmc_write 300 rocprofv3 --pmc WRITE_SIZE --kernel-include-regex stitch_tiled -d gpurun_out/pmc_write -o run --output-format csv -- python3 bench.py --pmc-child --steps 5
            step pmc_sq 300 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_LDS_BANK_CONFLICT --kernel-include-regex stitch_tiled -d gpurun_out/pmc_sq -o run --output-format csv -- python3 bench.py --pmc-child --steps 5
            step pmc_sq2 300 rocprofv3 --pmc SQ_ACTIVE_INST_VALU SQ_WAIT_INST_ANY SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS GRBM_GUI_ACTIVE SQ_INSTS_VMEM_WR --kernel-include-regex stitch_tiled -d gpurun_out/pmc_sq2 -o run --output-format csv -- python3 bench.py --pmc-child --steps 5 ;;
    prof)   step prof 600 rocprofv3 --kernel-trace --stats -d gpurun_out/prof -o run --output-format csv -- python3 bench.py --steps 20 --warmup 3 --no-cpu-baseline ;;
  esac
done
echo ALLDONE

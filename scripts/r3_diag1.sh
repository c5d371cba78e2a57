#!/bin/bash
# VALU instruction throughput on gfx950 (scripts/valu_rates.hip) and the composite's scalar / branch /
# VMEM issue counters on C2 (one SQ pass).
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 120 ./scripts/valu_rates.bin > gpurun_out/valu_rates.txt 2>&1 || { echo "valu rc=$?"; tail -5 gpurun_out/valu_rates.txt; exit 1; }
cat gpurun_out/valu_rates.txt
timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_SALU SQ_INSTS_SMEM SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_MISC SQ_ACTIVE_INST_VMEM SQ_INSTS_BRANCH SQ_WAIT_INST_LDS SQ_WAVE_CYCLES --kernel-include-regex stitch_tiled -d gpurun_out/d1_sq -o run --output-format csv -- python3 bench.py --config C2 --pmc-child --steps 5 > gpurun_out/d1_sq.log 2>&1 || { echo "sq rc=$?"; tail -5 gpurun_out/d1_sq.log; exit 1; }
python3 - <<'PY'
import csv, glob, collections
f = glob.glob("gpurun_out/d1_sq/run_counter_collection.csv") + glob.glob("gpurun_out/d1_sq/*/run_counter_collection.csv")
acc = collections.defaultdict(list)
for row in csv.DictReader(open(f[0])):
    acc[(row["Kernel_Name"][:60], row["Counter_Name"])].append(float(row["Counter_Value"]))
for k, v in sorted(acc.items()):
    print(k[0], k[1], sum(v) / len(v))
PY
echo done

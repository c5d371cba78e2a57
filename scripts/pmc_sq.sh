#!/bin/bash
# SQ issue/stall breakdown of one kernel (MI355X_MICROARCH.md "rocprofv3 PMC slots"): one pass, 8 SQ + 1 GRBM.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
CFG=${CFG:-C2}
RE=${RE:-stitch_tiled}
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_INSTS_VALU SQ_LDS_BANK_CONFLICT GRBM_GUI_ACTIVE --kernel-include-regex "$RE" -d gpurun_out/pmcsq_$CFG -o run --output-format csv -- python3 bench.py --config $CFG --pmc-child --steps 5 > gpurun_out/pmcsq_$CFG.log 2>&1 || { echo "pmc rc=$?"; tail -5 gpurun_out/pmcsq_$CFG.log; exit 1; }
python3 - <<'PY'
import csv, glob, collections
f = glob.glob("gpurun_out/pmcsq_*/run_counter_collection.csv") + glob.glob("gpurun_out/pmcsq_*/*/run_counter_collection.csv")
acc = collections.defaultdict(list)
for row in csv.DictReader(open(f[0])):
    acc[(row["Kernel_Name"][:60], row["Counter_Name"])].append(float(row["Counter_Value"]))
for k, v in sorted(acc.items()):
    print(k[0], k[1], sum(v) / len(v))
PY

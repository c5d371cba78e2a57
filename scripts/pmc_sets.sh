#!/bin/bash
# SQ counter passes over the stitch kernel (one rocprofv3 --pmc run per set: <= 8 SQ counters each),
# summarised per counter (mean over launches).  SETS="a b" picks sets; CFG / RE as pmc.sh.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
CFG=${CFG:-C2}
RE=${RE:-stitch_tiled}
declare -A S
S[issue]="SQ_INSTS_SALU SQ_ACTIVE_INST_SCA SQ_INST_CYCLES_SALU SQ_INSTS_SMEM SQ_ACTIVE_INST_ANY SQ_BUSY_CU_CYCLES SQ_ACTIVE_INST_MISC SQ_INSTS_BRANCH"
S[fifo]="SQ_VMEM_TA_ADDR_FIFO_FULL SQ_VMEM_TA_CMD_FIFO_FULL SQ_VMEM_WR_TA_DATA_FIFO_FULL SQ_LDS_CMD_FIFO_FULL SQ_LDS_DATA_FIFO_FULL SQ_LDS_IDX_ACTIVE SQ_INST_CYCLES_VMEM_WR SQ_INST_CYCLES_VMEM_RD"
S[core]="SQ_WAVE_CYCLES SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_INSTS_VALU SQ_LDS_BANK_CONFLICT SQ_INSTS_LDS"
S[mem1]="TCP_TCC_READ_REQ_LATENCY_sum TCP_TCC_READ_REQ_sum TCP_UTCL1_TRANSLATION_MISS_sum TCP_UTCL1_TRANSLATION_HIT_sum TA_TA_BUSY_sum TA_ADDR_STALLED_BY_TC_CYCLES_sum TD_TD_BUSY_sum TD_TC_STALL_sum"
S[mem2]="TCC_HIT_sum TCC_MISS_sum TCP_TCP_LATENCY_sum TCP_PENDING_STALL_CYCLES_sum TCP_TCR_TCP_STALL_CYCLES_sum TCP_READ_TAGCONFLICT_STALL_CYCLES_sum"
S[mem3]="TCP_TCC_WRITE_REQ_LATENCY_sum TCP_TCC_WRITE_REQ_sum TCP_UTCL1_TRANSLATION_MISS_UNDER_MISS_sum TCP_UTCL1_STALL_MULTI_MISS_sum TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_DRAM_sum"
for set in ${SETS:-issue fifo core}; do
  timeout -s KILL 120 rocprofv3 --pmc ${S[$set]} GRBM_GUI_ACTIVE --kernel-include-regex "$RE" -d gpurun_out/pmcs_$set -o run --output-format csv -- python3 bench.py --config $CFG --pmc-child --steps 5 > gpurun_out/pmcs_$set.log 2>&1 || { echo "pmc $set rc=$?"; tail -5 gpurun_out/pmcs_$set.log; exit 1; }
done
python3 - <<'PY'
import csv, glob, collections
for f in sorted(glob.glob("gpurun_out/pmcs_*/run_counter_collection.csv")):
    acc = collections.defaultdict(list)
    for row in csv.DictReader(open(f)):
        acc[row["Counter_Name"]].append(float(row["Counter_Value"]))
    print(f.split("/")[1], " ".join("%s=%.4g" % (k, sum(v) / len(v)) for k, v in sorted(acc.items())))
PY

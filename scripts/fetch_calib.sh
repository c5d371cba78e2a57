#!/bin/bash
# FETCH_SIZE calibration (scripts/fetch_calib.hip, built on the host: hipcc --offload-arch=gfx950 -O3
# scripts/fetch_calib.hip -o scripts/fetch_calib): one --pmc pass, then the reported KiB per kernel
# against the bytes each kernel reads.
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE -d gpurun_out/fetch_calib -o run --output-format csv -- ./scripts/fetch_calib \
  > gpurun_out/fetch_calib.log 2>&1 || { echo "rc=$?"; tail -5 gpurun_out/fetch_calib.log; exit 1; }
python3 - <<'PY'
import csv, glob, collections
f = glob.glob("gpurun_out/fetch_calib/**/run_counter_collection.csv", recursive=True)[0]
agg = collections.defaultdict(list)
for r in csv.DictReader(open(f)):
    agg[r["Kernel_Name"].split("(")[0]].append(float(r["Counter_Value"]))
known = {"stream_read<16>": 1 << 30, "stream_read<8>": 1 << 30, "stream_read<4>": 1 << 30,
         "segment_read<8>": (1 << 18) * 128, "segment_read<4>": (1 << 18) * 64}
for k, v in sorted(agg.items()):
    name = k.split("void ")[-1]
    b = sorted(v)[len(v) // 2] * 1024
    kb = [x for n, x in known.items() if name.endswith(n)]
    print("%-28s FETCH_SIZE %.4g B  read %.4g B  ratio %.3f" % (name, b, kb[0] if kb else 0, b / kb[0] if kb else 0))
PY

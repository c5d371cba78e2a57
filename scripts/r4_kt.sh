#!/bin/bash
# Per-kernel durations of library variants: rocprofv3 --kernel-trace of a short bench.py run per variant
# (one frame in flight), median duration per kernel@grid over the last frames.
#   VARIANTS="cur x" CFG=C3 bash scripts/r4_kt.sh
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp PYTHONUNBUFFERED=1
mkdir -p gpurun_out
TAG=${TAG:-kt}
V=$PWD/opencv-octvr_amd/lib/variants
for rep in $(seq 1 ${REPS:-1}); do
for v in ${VARIANTS:-cur}; do
  lib=; [ "$v" != cur ] && lib="OCTVR_HIP_LIB=$V/$v.so"
  d=gpurun_out/${TAG}_${v}_$rep
  env $lib timeout -s KILL 240 rocprofv3 --kernel-trace -d $d -o run --output-format csv -- \
    python3 bench.py --config ${CFG:-C3} --steps 20 --warmup 3 --inflight ${INFLIGHT:-1} --no-cpu-baseline --no-async-e2e > $d.log 2>&1 \
    || { echo "$v rc=$?"; tail -5 $d.log; exit 1; }
  python3 - "$d" "$v" <<'PY'
import csv, glob, sys, collections
f = glob.glob(sys.argv[1] + "/**/run_kernel_trace.csv", recursive=True)[0]
rows = [r for r in csv.DictReader(open(f)) if "octvr" in r["Kernel_Name"]]
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
agg = collections.defaultdict(list)
for r in rows[-160:]:
    n = r["Kernel_Name"].split("(")[0].split("::")[-1][:28]
    agg["%s@%s" % (n, r["Grid_Size_X"])].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
print(sys.argv[2], " ".join("%s=%.1f" % (k, sorted(v)[len(v) // 2]) for k, v in sorted(agg.items())))
PY
done
done
echo done

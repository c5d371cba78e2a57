#!/bin/bash
# C2 with and without the gain feed (how much the in-flight feed costs the composite); C3 per-kernel
# breakdown with one frame in flight after the owned-tile fast path.
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp PYTHONUNBUFFERED=1
mkdir -p gpurun_out
b() {  # name cfg [bench args...]
  local name=$1 cfg=$2; shift 2
  timeout -k 10 240 python bench.py --config $cfg --steps 60 --warmup 5 --no-cpu-baseline --no-async-e2e "$@" \
      > gpurun_out/d2_$name.log 2>&1 || { echo "$name rc=$?"; tail -5 gpurun_out/d2_$name.log; exit 1; }
  python3 -c "import json; d=json.loads(open('gpurun_out/d2_$name.log').read().strip().splitlines()[-1]); r=d['roofline']; o=d.get('roofline_one_in_flight',{}); print('$name', d['value'], d['ms_per_step'], r['kernel_us'], r['frac_at_step_time'], o.get('kernel_us'), o.get('step_us'))"
}
for rep in 1 2; do
  b gain_$rep C2
  b nogain_$rep C2 --no-gain
done
timeout -s KILL 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/d2_kt_C3 -o run -- \
  python3 bench.py --config C3 --steps 20 --warmup 3 --no-cpu-baseline --no-async-e2e --inflight 1 > gpurun_out/d2_kt_C3.log 2>&1 \
  || { echo "kt C3 rc=$?"; tail -5 gpurun_out/d2_kt_C3.log; exit 1; }
python3 - <<'PY'
import csv, glob
f = glob.glob("gpurun_out/d2_kt_C3/**/run_kernel_trace.csv", recursive=True)[0]
rows = list(csv.DictReader(open(f)))
import collections
by = collections.defaultdict(list)
for r in rows:
    n = r["Kernel_Name"]
    d = int(r["End_Timestamp"]) - int(r["Start_Timestamp"])
    key = n[:40]
    if "mb_blend" in n or "mb_down" in n:
        key = n[:24] + " grid=" + r.get("Grid_Size", r.get("Grid_Size_X", "?"))
    by[key].append(d)
for k, v in sorted(by.items(), key=lambda kv: -sum(kv[1])):
    if len(v) >= 10:
        print("%-60s n=%4d avg=%8.1f us" % (k, len(v), sum(v) / len(v) / 1e3))
PY
echo done

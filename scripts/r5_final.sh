#!/bin/bash
# Round 5 evidence session for the in-tree library, in two GPU calls (each under gpurun's 20-minute limit):
#   PART=A: the GPU suite, then the PMC passes per config (scripts/pmc.sh; raw CSVs into gpurun_out/,
#           summarised into profiles/ on this side by scripts/collect_profiles.py so that they travel with
#           the library they were taken from);
#   PART=B: the default bench line (as the driver runs it), one line per config (their `traffic` now
#           filled from those summaries), then rocprofv3 --kernel-trace --stats per config at one and at the
#           benched frames in flight, and the union of the timed launches' intervals from each trace
#           (scripts/trace_union.py: the basis of the lines' kernel_us with frames in flight).
# Every GPU step has its own time limit; any failure ends the script.
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp PYTHONUNBUFFERED=1
mkdir -p gpurun_out
TAG=${TAG:-r05}
if [ "${PART:-A}" = A ]; then
  timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 400 --timeout-method thread -p no:cacheprovider \
    > gpurun_out/${TAG}_tests.log 2>&1 || { grep -E "^E |FAILED" gpurun_out/${TAG}_tests.log | head; exit 1; }
  tail -1 gpurun_out/${TAG}_tests.log
  for CFG in C2 C4; do CFG=$CFG PASSES="FETCH WRITE SQ1 SQ2 TCC" bash scripts/pmc.sh || exit 1; done
  CFG=C3 PASSES="FETCH WRITE SQ1" bash scripts/pmc.sh || exit 1
  for CFG in C1 F2; do CFG=$CFG PASSES="FETCH WRITE SQ1" bash scripts/pmc.sh || exit 1; done
  echo done A
  exit 0
fi
timeout -k 10 500 python bench.py > gpurun_out/${TAG}_bench_default.json 2> gpurun_out/${TAG}_bench_default.err \
  || { tail -5 gpurun_out/${TAG}_bench_default.err; exit 1; }
for CFG in C1 C2 C3 C4 F2; do
  timeout -k 10 300 python bench.py --config $CFG --no-async-e2e --no-cpu-baseline \
    > gpurun_out/${TAG}_bench_$CFG.json 2> gpurun_out/${TAG}_bench_$CFG.err || { echo "$CFG rc=$?"; tail -5 gpurun_out/${TAG}_bench_$CFG.err; exit 1; }
  python3 -c "import json; d=json.loads(open('gpurun_out/${TAG}_bench_$CFG.json').read().strip().splitlines()[-1]); r=d['roofline']; print('$CFG', d['value'], d['ms_per_step'], r['kernel_us'], r['frac'], r.get('traffic'))"
done
# kernel traces: C2 / C4 / C1 / F2 benched with 3 in flight, C3 with 4; each also with 1
for spec in C2:1 C2:3 C4:1 C4:3 C3:1 C3:4 C1:3 F2:3; do
  CFG=${spec%:*}; IF=${spec#*:}
  d=gpurun_out/kt_${TAG}_${CFG}_if$IF
  timeout -s KILL 240 rocprofv3 --kernel-trace --stats -d $d -o run --output-format csv -- \
    python3 bench.py --config $CFG --steps 200 --warmup 5 --inflight $IF --no-cpu-baseline --no-async-e2e \
    > $d.log 2>&1 || { echo "kt $CFG if$IF rc=$?"; tail -5 $d.log; exit 1; }
  echo "kt $CFG if$IF ok"
done
echo done B

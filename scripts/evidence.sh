#!/bin/bash
# Evidence session for the in-tree library (every config at its benched settings), in two GPU calls:
#   PART=A: the GPU suite, then the PMC passes per config (scripts/pmc.sh; raw CSVs into gpurun_out/,
#           summarised into profiles/ on this side by scripts/collect_profiles.py, keyed to the library's
#           sha256 and the frames per launch);
#   PART=B: the default bench line (as the driver runs it), one line per config (their `traffic` filled from
#           those summaries), then rocprofv3 --kernel-trace --stats per config with one frame in flight and at
#           its benched settings (the trace union of the timed launches: scripts/union_check.py).
# Every GPU step has its own time limit; any failure ends the script.
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp PYTHONUNBUFFERED=1
mkdir -p gpurun_out
TAG=${TAG:-r06h}
# config: streams frames-per-launch (bench.py DEFAULT_INFLIGHT / DEFAULT_BATCH)
declare -A BENCHED=([C1]="2 4" [C2]="3 1" [C3]="4 1" [C4]="2 4" [F2]="1 4")
if [ "${PART:-A}" = A ]; then
  timeout -k 10 800 python -u -m pytest tests -m gpu -x -q --timeout 400 --timeout-method thread -p no:cacheprovider \
    > gpurun_out/${TAG}_tests.log 2>&1 || { grep -E "^E |FAILED" gpurun_out/${TAG}_tests.log | head; exit 1; }
  tail -1 gpurun_out/${TAG}_tests.log
  for CFG in C2 C4 C3 C1 F2; do
    set -- ${BENCHED[$CFG]}
    case $CFG in C2|C4) PS="FETCH WRITE SQ1 SQ2 TCC" ;; *) PS="FETCH WRITE SQ1" ;; esac
    CFG=$CFG INFLIGHT=$1 BATCH=$2 PASSES="$PS" bash scripts/pmc.sh || exit 1
  done
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
# kernel traces: one frame in flight (--batch 1 --inflight 1), then the benched settings
for CFG in C2 C4 C3 C1 F2; do
  set -- ${BENCHED[$CFG]}
  for IF in 1 $1; do
    if [ $IF = 1 ]; then B=1; else B=$2; fi
    [ $IF = 1 ] && [ $1 = 1 ] && B=$2  # F2's benched setting is itself one stream
    d=gpurun_out/kt_${TAG}_${CFG}_if${IF}b$B
    [ -d $d ] && continue
    timeout -s KILL 240 rocprofv3 --kernel-trace --stats -d $d -o run --output-format csv -- \
      python3 bench.py --config $CFG --steps 200 --warmup 5 --inflight $IF --batch $B --no-cpu-baseline --no-async-e2e \
      > $d.log 2>&1 || { echo "kt $CFG if$IF b$B rc=$?"; tail -5 $d.log; exit 1; }
    echo "kt $CFG if$IF b$B ok"
  done
done
echo done B

#!/bin/bash
# Round 4 profile session for the in-tree library: per config a rocprofv3 kernel trace + stats of a
# bench.py run (frames in flight $INFLIGHT, default 3; C3 also with 1), then the PMC passes
# (scripts/pmc.sh).  Every GPU step has its own time limit; any failure ends the script.
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp PYTHONUNBUFFERED=1
mkdir -p gpurun_out
TAG=${TAG:-r04}
for CFG in ${CONFIGS:-C2 C3 C4}; do
  for IF in ${INFLIGHTS:-3}; do
    timeout -s KILL 240 rocprofv3 --kernel-trace --stats -d gpurun_out/kt_${TAG}_${CFG}_if$IF -o run --output-format csv -- \
      python3 bench.py --config $CFG --steps 30 --warmup 5 --inflight $IF --no-cpu-baseline --no-async-e2e \
      > gpurun_out/kt_${TAG}_${CFG}_if$IF.log 2>&1 || { echo "kt $CFG if$IF rc=$?"; tail -5 gpurun_out/kt_${TAG}_${CFG}_if$IF.log; exit 1; }
    echo "kt $CFG if$IF ok"
  done
  if [ -n "$PASSES" ]; then
    CFG=$CFG PASSES="$PASSES" bash scripts/pmc.sh || exit 1
  fi
done
echo done

#!/bin/bash
# C4 frames-in-flight anatomy: bench lines at 1 / 2 / 3 frames in flight with and without the gain feed,
# then kernel traces (3 in flight, gain and --no-gain) analysed by scripts/overlap.py.
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp PYTHONUNBUFFERED=1
mkdir -p gpurun_out
TAG=${TAG:-c4}
CFG=${CFG:-C4}
for G in "" "--no-gain"; do
  for IF in ${INFLIGHTS:-1 2 3}; do
    n=${TAG}_${CFG}_if${IF}${G:+_nogain}
    timeout -k 10 300 python bench.py --config $CFG --steps 30 --warmup 5 --inflight $IF $G --no-cpu-baseline --no-async-e2e \
      > gpurun_out/$n.json 2> gpurun_out/$n.err || { echo "$n rc=$?"; tail -5 gpurun_out/$n.err; exit 1; }
    python3 -c "import json; d=json.loads(open('gpurun_out/$n.json').read().strip().splitlines()[-1]); print('$n', d['value'], d['ms_per_step'], d['roofline']['kernel_us'], d.get('roofline_one_in_flight',{}).get('kernel_us'))"
  done
done
for G in "" "--no-gain"; do
  n=kt_${TAG}_${CFG}_if3${G:+_nogain}
  timeout -s KILL 300 rocprofv3 --kernel-trace -d gpurun_out/$n -o run --output-format csv -- \
    python3 bench.py --config $CFG --steps 30 --warmup 5 --inflight 3 $G --no-cpu-baseline --no-async-e2e \
    > gpurun_out/$n.log 2>&1 || { echo "$n rc=$?"; tail -5 gpurun_out/$n.log; exit 1; }
  python3 scripts/overlap.py gpurun_out/$n 24
done
echo done

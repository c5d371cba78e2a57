#!/bin/bash
# Shader clock and power while the C2 composite runs back to back: a long bench run (STEPS frames,
# three in flight) in the background, rocm-smi sampled every half second beside it.  The samples taken
# while the timed loop runs give the clock the composite's cycle counts convert at.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
STEPS=${STEPS:-100000}
CFG=${CFG:-C2}
timeout -k 10 240 python3 -u bench.py --config "$CFG" --steps "$STEPS" --warmup 50 --no-cpu-baseline --no-async-e2e \
  > gpurun_out/clock_bench.log 2>&1 &
pid=$!
for i in $(seq 1 200); do
  kill -0 $pid 2>/dev/null || break
  echo "t=$(date +%s.%N)"
  rocm-smi --showclocks --showpower 2>&1 | grep -E "sclk|Power|mclk|fclk" || true
  sleep 0.5
done > gpurun_out/clock_samples.txt
wait $pid
rc=$?
tail -2 gpurun_out/clock_bench.log
exit $rc

#!/bin/bash
# gpurun_wait.sh OUTFILE TIMEOUT 'command' — re-submits only while no box / slot was available
# (exit 3, or a box lost while being prepared: nothing ran, nothing charged); any run that started
# is never retried.
out=$1; to=$2; cmd=$3
for i in $(seq 1 20); do
  /usr/local/graft/bin/gpurun --timeout "$to" -- "$cmd" > "$out" 2>&1
  rc=$?
  if [ $rc -eq 3 ] || { [ $rc -ne 0 ] && grep -q "while being prepared\|backing off" "$out"; }; then
    sleep 100; continue
  fi
  exit $rc
done
exit $rc

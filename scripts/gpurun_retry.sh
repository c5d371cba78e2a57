#!/bin/bash
# Retry a gpurun call only when the infrastructure reports a transient failure (nothing ran, nothing
# charged).  Any real run result (pass or fail) is returned as is.
for attempt in 1 2 3 4 5 6; do
  /usr/local/graft/bin/gpurun "$@"
  rc=$?
  st=$(python3 -c "import json;print(json.load(open('gpurun_out/.last_call.json')).get('status',''))" 2>/dev/null)
  if [ "$st" != "transient" ] && [ $rc -ne 3 ]; then exit $rc; fi
  echo "[retry] transient (attempt $attempt), sleeping 60s"
  sleep 60
done
exit $rc

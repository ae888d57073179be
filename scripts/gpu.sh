#!/bin/bash
# Runs one gpurun call; if the pool reports a transient infrastructure failure (the command
# never started: box not prepared / no slot), waits and asks again.  Command failures are
# never retried.
for attempt in 1 2 3 4 5; do
  /usr/local/graft/bin/gpurun "$@"
  rc=$?
  st=$(python3 -c "import json;print(json.load(open('gpurun_out/.last_call.json')).get('status',''))" 2>/dev/null)
  if [ "$st" = "transient" ] || [ $rc -eq 3 ]; then
    echo "[gpu.sh] transient ($st rc=$rc), retry $attempt after 40s" >&2
    sleep 40
    continue
  fi
  exit $rc
done
exit $rc

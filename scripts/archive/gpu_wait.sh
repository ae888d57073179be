#!/bin/bash
# Runs one gpurun call; if the pool reports a transient infrastructure failure (the command
# never started: box not prepared / no slot / backing off), waits as long as it asks and asks
# again.  Command failures are never retried.
for attempt in $(seq 1 40); do
  out=$(mktemp)
  /usr/local/graft/bin/gpurun "$@" 2>&1 | tee "$out"
  rc=${PIPESTATUS[0]}
  st=$(python3 -c "import json;print(json.load(open('gpurun_out/.last_call.json')).get('status',''))" 2>/dev/null)
  wait_s=$(grep -o 'retry in [0-9]*s' "$out" | tail -1 | grep -o '[0-9]*')
  rm -f "$out"
  if [ "$st" = "transient" ] || [ $rc -eq 3 ]; then
    sleep_s=$(( ${wait_s:-30} + 15 ))
    echo "[gpu.sh] transient ($st rc=$rc), retry $attempt after ${sleep_s}s" >&2
    sleep $sleep_s
    continue
  fi
  exit $rc
done
exit $rc

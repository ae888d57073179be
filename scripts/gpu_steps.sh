#!/bin/bash
# Runs GPU steps in order on the gpurun box; each step has its own time limit.  A step that
# times out, aborts or segfaults (exit >= 124) ends the script; ordinary failures (exit 1/2)
# are recorded and the next step runs.
# usage: scripts/gpu_steps.sh "<name>:<seconds>:<command>" ...
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
status=0
for spec in "$@"; do
  name="${spec%%:*}"; rest="${spec#*:}"; secs="${rest%%:*}"; cmd="${rest#*:}"
  echo "=== [$name] ($secs s) $cmd"
  start=$(date +%s)
  timeout -k 10 "$secs" bash -c "$cmd" > "gpurun_out/$name.log" 2>&1
  rc=$?
  echo "=== [$name] exit=$rc after $(( $(date +%s) - start )) s"
  tail -n 25 "gpurun_out/$name.log"
  if [ $rc -ne 0 ]; then status=$rc; fi
  if [ $rc -ge 124 ]; then echo "=== stopping: step $name ended with $rc"; exit $rc; fi
done
exit $status

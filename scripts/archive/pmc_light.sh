#!/bin/bash
# PMC passes over a short config-2 run (light/heavy task kernels), one rocprofv3 run per pass.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
mkdir -p gpurun_out/pmcl
export TMPDIR=/tmp
timeout -s KILL 60 rocprofv3 -L > gpurun_out/pmcl/counters.txt 2>&1 || true
i=0
for set in "$@"; do
  i=$((i+1))
  echo "=== pass $i: $set"
  timeout -s KILL 90 rocprofv3 --pmc $set --output-format csv -d gpurun_out/pmcl/p$i -o run -- python3 bench.py --pairs 300000 --steps 2 --warmup 1 --no-cpu-baseline --census 0 --bsi 0 --secondary none > gpurun_out/pmcl/p$i.log 2>&1
  rc=$?
  echo "exit=$rc"
  if [ $rc -ne 0 ]; then exit $rc; fi
done

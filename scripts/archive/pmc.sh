#!/bin/bash
# PMC passes over a short pairwise run (each pass its own run, counters within gfx950 slot limits).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
mkdir -p gpurun_out/pmc
export TMPDIR=/tmp
CMD="python bench.py --pairs ${PMC_PAIRS:-300000} --steps 2 --warmup 1 --no-cpu-baseline ${PMC_EXTRA:-}"
timeout -s KILL 60 rocprofv3 -L > gpurun_out/pmc/counters.txt 2>&1 || true
i=0
for set in "$@"; do
  i=$((i+1))
  echo "=== pass $i: $set"
  timeout -k 5 120 rocprofv3 --pmc $set --output-format csv -d gpurun_out/pmc/p$i -o run -- $CMD > gpurun_out/pmc/p$i.log 2>&1
  rc=$?
  echo "exit=$rc"
  if [ $rc -ge 124 ]; then exit $rc; fi
done

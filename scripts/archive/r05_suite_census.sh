#!/bin/bash
# The full GPU suite, then the census latency per op.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
O=gpurun_out/r5sc
mkdir -p $O
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > $O/gputests.txt 2>&1 || { tail -40 $O/gputests.txt; exit 1; }
tail -1 $O/gputests.txt
for kt in 0 1; do
  RBGPU_SMALL_KERNEL_TIMES=$kt timeout -k 10 120 python scripts/census_lat.py --calls 200 > $O/census_kt$kt.json || exit 1
  echo "kt=$kt $(cat $O/census_kt$kt.json)"
done

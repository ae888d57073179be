#!/bin/bash
# Small-batch merge walk (branch-free, one value ahead): parity, census timeline and latency.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
O=gpurun_out/r5merge3
mkdir -p $O
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 600 python -u -m pytest tests/test_gpu_pairwise.py tests/test_gpu_async.py tests/test_gpu_longlong.py tests/test_gpu_inplace.py -x -q --timeout 200 --timeout-method thread > $O/tests.txt 2>&1 || { tail -40 $O/tests.txt; exit 1; }
tail -1 $O/tests.txt
bash scripts/r05_stamps.sh stamps || exit 1
for round in 1 2; do
  timeout -k 10 120 python scripts/census_lat.py --calls 300 > $O/census_$round.json || exit 1
  echo "census main $round $(cat $O/census_$round.json)"
done

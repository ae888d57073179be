#!/bin/bash
# Small-batch Array x Array merge path: the pairwise / async / 64-bit / in-place parity tests, then the
# census latency per op (kernel times on and off).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
O=gpurun_out/r5merge
mkdir -p $O
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 600 python -u -m pytest tests/test_gpu_pairwise.py tests/test_gpu_async.py tests/test_gpu_longlong.py tests/test_gpu_inplace.py tests/test_gpu_configs.py -x -q --timeout 200 --timeout-method thread > $O/tests.txt 2>&1 || { tail -40 $O/tests.txt; exit 1; }
tail -1 $O/tests.txt
for kt in 0 1; do
  RBGPU_SMALL_KERNEL_TIMES=$kt timeout -k 10 120 python scripts/census_lat.py --calls 200 > $O/census_kt$kt.json || exit 1
  echo "kt=$kt $(cat $O/census_kt$kt.json)"
done

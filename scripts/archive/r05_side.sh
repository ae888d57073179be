#!/bin/bash
# Small-batch Array pairs with one side of <= 64 values by closed-form placement (main) or the merged walk
# (abvar/noside): parity, then the census latency per op, interleaved.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
O=gpurun_out/r5side
mkdir -p $O
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 400 python -u -m pytest tests/test_gpu_pairwise.py tests/test_gpu_bsi.py tests/test_gpu_async.py -x -q --timeout 200 --timeout-method thread > $O/tests.txt 2>&1 || { tail -30 $O/tests.txt; exit 1; }
tail -1 $O/tests.txt
for round in 1 2 3; do
  for v in main noside; do
    lib=abvar/$v/librbgpu.so; [ "$v" = main ] && lib=roaringbitmap_amd/librbgpu.so
    RBGPU_LIB=$lib timeout -k 10 120 python scripts/census_lat.py --calls 300 > $O/c_$v$round.json || exit 1
    echo "census $v $round $(cat $O/c_$v$round.json)"
  done
done

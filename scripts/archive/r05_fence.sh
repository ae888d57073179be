#!/bin/bash
# Census: the result-word hand-off with a system-scope release (main) or a vmcnt(0) wait (nofence).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
O=gpurun_out/r5fence
mkdir -p $O
export HSA_ENABLE_IPC_MODE_LEGACY=0
RBGPU_LIB=abvar/nofence/librbgpu.so timeout -k 10 300 python -u -m pytest tests/test_gpu_pairwise.py tests/test_gpu_async.py -x -q --timeout 200 --timeout-method thread > $O/tests.txt 2>&1 || { tail -30 $O/tests.txt; exit 1; }
tail -1 $O/tests.txt
bash scripts/r05_stamps.sh stamps stamps_nf || exit 1
for round in 1 2; do
  for v in main nofence; do
    lib=abvar/$v/librbgpu.so; [ "$v" = main ] && lib=roaringbitmap_amd/librbgpu.so
    RBGPU_LIB=$lib timeout -k 10 120 python scripts/census_lat.py --calls 300 > $O/census_$v$round.json || exit 1
    echo "census $v $round $(cat $O/census_$v$round.json)"
  done
done

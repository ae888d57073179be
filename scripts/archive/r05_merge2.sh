#!/bin/bash
# Array x Array merge: pairwise parity suite, then config-2 ops (main vs abvar/nolm, interleaved), then the
# census timeline per block (abvar/stamps vs abvar/stamps_nm).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
O=gpurun_out/r5merge2
mkdir -p $O
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 600 python -u -m pytest tests/test_gpu_pairwise.py tests/test_gpu_async.py tests/test_gpu_longlong.py tests/test_gpu_inplace.py tests/test_gpu_configs.py tests/test_gpu_type_pins.py tests/test_gpu_roaring_api.py -x -q --timeout 200 --timeout-method thread > $O/tests.txt 2>&1 || { tail -40 $O/tests.txt; exit 1; }
tail -1 $O/tests.txt
RBGPU_LIB=abvar/img/librbgpu.so timeout -k 10 300 python -u -m pytest tests/test_gpu_pairwise.py -x -q --timeout 200 --timeout-method thread > $O/tests_img.txt 2>&1 || { tail -40 $O/tests_img.txt; exit 1; }
tail -1 $O/tests_img.txt
bash scripts/r05_ab_ops.sh main nolm img || exit 1
bash scripts/r05_stamps.sh stamps stamps_nm || exit 1
for round in 1 2; do
  for v in main nopoll; do
    lib=abvar/$v/librbgpu.so; [ "$v" = main ] && lib=roaringbitmap_amd/librbgpu.so
    RBGPU_LIB=$lib timeout -k 10 120 python scripts/census_lat.py --calls 300 > $O/census_$v$round.json || exit 1
    echo "census $v $round $(cat $O/census_$v$round.json)"
  done
done

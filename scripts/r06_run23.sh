#!/bin/bash
# Lopsided merges (one side <= 64 values) publishing their slot word before the store sweep (RBG_LOPSIDED=1,
# abvar/lop): parity tests under that build, study (OR), census A/B against the product.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0
o=gpurun_out/r6lop; mkdir -p $o
RBGPU_LIB=$PWD/abvar/lop/librbgpu.so timeout -k 10 600 python -u -m pytest tests/test_gpu_pairwise.py tests/test_gpu_configs.py tests/test_gpu_type_pins.py tests/test_gpu_roaring_api.py -m gpu -x -q --timeout 120 --timeout-method thread > $o/gputests.txt 2>&1 || { echo "TESTS FAILED"; tail -30 $o/gputests.txt; exit 1; }
tail -1 $o/gputests.txt
RBGPU_LIB=$PWD/abvar/lopst/librbgpu.so timeout -k 10 120 python3 scripts/micro/small_study.py OR > $o/study_OR.txt 2>&1 || { echo "STUDY FAILED"; tail -20 $o/study_OR.txt; exit 1; }
head -9 $o/study_OR.txt
timeout -k 10 600 python3 scripts/micro/census_ab.py 3 base lop > $o/census_ab.txt 2>&1 || { echo "AB FAILED"; tail -20 $o/census_ab.txt; exit 1; }
cat $o/census_ab.txt

#!/bin/bash
# Small-batch pair lookup in one round (np <= 256): pairwise GPU tests, study (OR), census A/B against HEAD (cbase2).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0
o=gpurun_out/r6look; mkdir -p $o
timeout -k 10 600 python -u -m pytest tests/test_gpu_pairwise.py tests/test_gpu_configs.py tests/test_gpu_async.py -m gpu -x -q --timeout 120 --timeout-method thread > $o/gputests.txt 2>&1 || { echo "TESTS FAILED"; tail -30 $o/gputests.txt; exit 1; }
tail -1 $o/gputests.txt
RBGPU_LIB=$PWD/abvar/sstudy/librbgpu.so timeout -k 10 120 python3 scripts/micro/small_study.py OR > $o/study_OR.txt 2>&1 || { echo "STUDY FAILED"; tail -20 $o/study_OR.txt; exit 1; }
head -9 $o/study_OR.txt
timeout -k 10 600 python3 scripts/micro/census_ab.py 3 cbase2 base > $o/census_ab.txt 2>&1 || { echo "AB FAILED"; tail -20 $o/census_ab.txt; exit 1; }
cat $o/census_ab.txt

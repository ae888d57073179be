#!/bin/bash
# Early slot words: compaction block by id (product) vs by start ticket (abvar/tick) vs the previous build (cbase).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0
o=gpurun_out/r6early2; mkdir -p $o
timeout -k 10 600 python -u -m pytest tests/test_gpu_pairwise.py tests/test_gpu_configs.py -m gpu -x -q --timeout 120 --timeout-method thread > $o/gputests.txt 2>&1 || { echo "TESTS FAILED"; tail -30 $o/gputests.txt; exit 1; }
tail -1 $o/gputests.txt
timeout -k 10 600 python3 scripts/micro/census_ab.py 3 cbase base tick > $o/census_ab.txt 2>&1 || { echo "AB FAILED"; tail -20 $o/census_ab.txt; exit 1; }
cat $o/census_ab.txt

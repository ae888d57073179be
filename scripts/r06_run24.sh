#!/bin/bash
# Double-buffered small-batch slot words (resets spread over the next call's blocks instead of the compaction's
# tail): GPU tests of the pairwise paths, census A/B against HEAD (cbase3).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0
o=gpurun_out/r6dbuf; mkdir -p $o
timeout -k 10 600 python -u -m pytest tests/test_gpu_pairwise.py tests/test_gpu_configs.py tests/test_gpu_async.py tests/test_gpu_type_pins.py tests/test_gpu_roaring_api.py tests/test_gpu_inplace.py -m gpu -x -q --timeout 120 --timeout-method thread > $o/gputests.txt 2>&1 || { echo "TESTS FAILED"; tail -30 $o/gputests.txt; exit 1; }
tail -1 $o/gputests.txt
timeout -k 10 600 python3 scripts/micro/census_ab.py 4 cbase3 base > $o/census_ab.txt 2>&1 || { echo "AB FAILED"; tail -20 $o/census_ab.txt; exit 1; }
cat $o/census_ab.txt

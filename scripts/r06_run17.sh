#!/bin/bash
# Small-batch kernel with early slot words (published before each key's payload stores, polled by the last block to
# START): GPU suite, then census interleaved against the previous build (abvar/cbase).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0
o=gpurun_out/r6early; mkdir -p $o
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $o/gputests.txt 2>&1 || { echo "TESTS FAILED"; tail -30 $o/gputests.txt; exit 1; }
tail -2 $o/gputests.txt
timeout -k 10 600 python3 scripts/micro/census_ab.py 3 cbase base > $o/census_ab.txt 2>&1 || { echo "AB FAILED"; tail -20 $o/census_ab.txt; exit 1; }
cat $o/census_ab.txt

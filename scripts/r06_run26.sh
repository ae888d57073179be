#!/bin/bash
# Last sanity run on the final product commit: smoke + the full GPU suite.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0
o=gpurun_out/r6last; mkdir -p $o
timeout -k 10 120 python -c 'import __graft_entry__ as g; g.smoke()' > $o/smoke.txt 2>&1 || { echo "SMOKE FAILED"; tail -20 $o/smoke.txt; exit 1; }
tail -1 $o/smoke.txt
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > $o/gputests.txt 2>&1 || { echo "TESTS FAILED"; tail -30 $o/gputests.txt; exit 1; }
tail -1 $o/gputests.txt

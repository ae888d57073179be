#!/bin/bash
# The GPU suite on the in-tree library, then an interleaved A/B of the config-2 headline and the OR
# line against abvar/prev (the tree before the change).
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/join
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 600 python -u -m pytest -x -q -m gpu --timeout 120 --timeout-method thread tests \
  > gpurun_out/join/tests.txt 2>&1 || { tail -30 gpurun_out/join/tests.txt; exit 1; }
tail -2 gpurun_out/join/tests.txt
OPAB_WORKLOADS="pairwise_and pairwise_or" bash scripts/opab.sh prev main prev main

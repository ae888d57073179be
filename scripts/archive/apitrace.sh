#!/bin/bash
# HIP API + kernel trace of a short config-2 bench (host-side call costs between the kernels);
# summarise with scripts/api_summary.py gpurun_out/apitrace/p_results.db
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/apitrace
export HSA_ENABLE_IPC_MODE_LEGACY=0
cd /tmp && export TMPDIR=/tmp
timeout -k 10 240 rocprofv3 --kernel-trace --hip-trace --memory-copy-trace -d $GRAFT_REPO_ROOT/gpurun_out/apitrace -o p -- \
  python $GRAFT_REPO_ROOT/bench.py --secondary none --steps 5 --warmup 2 --no-cpu-baseline \
  > $GRAFT_REPO_ROOT/gpurun_out/apitrace/bench.json 2>&1

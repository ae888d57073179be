#!/bin/bash
# Round-4 check: the GPU suite, then a headline A/B of the variants given as arguments.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
mkdir -p gpurun_out/r4base
export HSA_ENABLE_IPC_MODE_LEGACY=0
scripts/gpu_steps.sh \
  "gputests:700:python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread" \
  "ab:500:bash scripts/r04_ab.sh $*"

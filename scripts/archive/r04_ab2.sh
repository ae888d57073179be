#!/bin/bash
# One call: config-2 headline A/B (main vs the variants given).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
export HSA_ENABLE_IPC_MODE_LEGACY=0
mkdir -p gpurun_out/ab
scripts/gpu_steps.sh "ab_c2:400:bash scripts/r04_ab.sh main $*"

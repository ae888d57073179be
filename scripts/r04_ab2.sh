#!/bin/bash
# One call: config-2 headline A/B (main vs $1...) and config-4 XOR A/B (main vs noslot).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
export HSA_ENABLE_IPC_MODE_LEGACY=0
mkdir -p gpurun_out/ab
scripts/gpu_steps.sh \
  "ab_c2:400:bash scripts/r04_ab.sh main $*" \
  "ab_c4:400:C4AB_ROUNDS=2 bash scripts/c4ab.sh main noslot"

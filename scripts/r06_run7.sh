#!/bin/bash
# workShyAnd on the SoA: keys per wave (8 / 16 / 32) and the load ring depth (2 / 3 / 4), interleaved A/B.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0
scripts/gpu_steps.sh \
  "andab:600:scripts/r06_ab.sh r6andab3 2 'wide_runs_and' '--workload wide_and_runs --secondary none --steps 3 --warmup 1 --no-cpu-baseline' base ak32 ak8 ar4 ar2"

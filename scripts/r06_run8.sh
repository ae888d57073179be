#!/bin/bash
# workShyAnd keys per wave 32 / 64 and ring depth at 32; naive_xor's two stretch heuristics (union-stretch floor,
# shortest pair-bounded stretch); interleaved A/B by kernel trace.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0
scripts/gpu_steps.sh \
  "andab:600:scripts/r06_ab.sh r6andab4 2 'wide_runs_and' '--workload wide_and_runs --secondary none --steps 3 --warmup 1 --no-cpu-baseline' base ak32 ak64 ak32r4 ak32r2" \
  "xorab:600:scripts/r06_ab.sh r6xorab4 2 'wide_runs_xor' '--workload wide_xor_runs --secondary none --steps 3 --warmup 1 --no-cpu-baseline' base xu256 xu4k xf4 xf16"

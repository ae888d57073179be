#!/bin/bash
# workShyAnd at 32 keys per wave / ring 2 (the new default): wide parity, A/B against ring 1; the emit kernel at
# 5 waves per SIMD (abvar/ew5) against the unbounded build on the headline.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0
scripts/gpu_steps.sh \
  "widetests:400:python -u -m pytest tests/test_gpu_wide.py tests/test_gpu_configs.py -m gpu -x -q --timeout 200 --timeout-method thread" \
  "andab:300:scripts/r06_ab.sh r6andab5 2 'wide_runs_and' '--workload wide_and_runs --secondary none --steps 3 --warmup 1 --no-cpu-baseline' base ar1" \
  "emitab:400:scripts/r06_ab.sh r6emitab 3 'k_pair_emit|k_pair_count|k_compact' '--secondary none --steps 20 --warmup 3 --no-cpu-baseline' base ew5"

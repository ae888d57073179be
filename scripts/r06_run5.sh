#!/bin/bash
# Balanced register-path emission (RBG_BAL_EMIT): parity of the pairwise suites, then an interleaved A/B of the
# task kernels per op against the per-word loops (abvar/bal0).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0
scripts/gpu_steps.sh \
  "baltests:400:python -u -m pytest tests/test_gpu_pairwise.py tests/test_gpu_type_pins.py tests/test_gpu_inplace.py tests/test_gpu_configs.py tests/test_gpu_longlong.py tests/test_gpu_roaring_api.py -m gpu -x -q --timeout 200 --timeout-method thread" \
  "balab_or:400:scripts/r06_ab.sh r6bal_or 2 'k_pair_tasks' '--workload pairwise_or --secondary none --steps 5 --warmup 2 --no-cpu-baseline' base bal0" \
  "balab_xor:400:scripts/r06_ab.sh r6bal_xor 2 'k_pair_tasks' '--workload pairwise_xor --secondary none --steps 5 --warmup 2 --no-cpu-baseline' base bal0" \
  "balab_and:400:scripts/r06_ab.sh r6bal_and 2 'k_pair_tasks' '--workload pairwise_and --secondary none --steps 10 --warmup 3 --no-cpu-baseline' base bal0"

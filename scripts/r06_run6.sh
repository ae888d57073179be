#!/bin/bash
# OR / XOR of two small Arrays by a merge in the register-path kernel (RBG_HEAVY_MERGE): parity, then an
# interleaved A/B against the register path (abvar/hm0).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0
scripts/gpu_steps.sh \
  "hmtests:400:python -u -m pytest tests/test_gpu_pairwise.py tests/test_gpu_type_pins.py tests/test_gpu_inplace.py tests/test_gpu_configs.py tests/test_gpu_longlong.py tests/test_gpu_roaring_api.py tests/test_gpu_async.py -m gpu -x -q --timeout 200 --timeout-method thread" \
  "hmab_or:400:scripts/r06_ab.sh r6hm_or 2 'k_pair_tasks' '--workload pairwise_or --secondary none --steps 5 --warmup 2 --no-cpu-baseline' base hm0" \
  "hmab_xor:400:scripts/r06_ab.sh r6hm_xor 2 'k_pair_tasks' '--workload pairwise_xor --secondary none --steps 5 --warmup 2 --no-cpu-baseline' base hm0"

#!/bin/bash
# GPU suite + the headline A/B (main vs base) + the headline with the async line.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
mkdir -p gpurun_out/r4
export HSA_ENABLE_IPC_MODE_LEGACY=0
scripts/gpu_steps.sh \
  "async_tests:300:python -u -m pytest tests/test_gpu_async.py -x -v --timeout 120 --timeout-method thread" \
  "ab_c2:400:bash scripts/r04_ab.sh main base" \
  "gputests:700:python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread" \
  "h_async:300:python bench.py --secondary pairwise_async --steps 20 --no-cpu-baseline > gpurun_out/r4/h_async.json"

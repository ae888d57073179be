#!/bin/bash
# Pipelined async pairwise and the 64-bit formats: their tests, then the headline with the async line (twice).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
mkdir -p gpurun_out/r4
export HSA_ENABLE_IPC_MODE_LEGACY=0
scripts/gpu_steps.sh \
  "async_tests:300:python -u -m pytest tests/test_gpu_async.py tests/test_gpu_longlong.py tests/test_gpu_configs.py -x -v --timeout 120 --timeout-method thread" \
  "h_async1:300:python bench.py --secondary pairwise_async --steps 20 --no-cpu-baseline > gpurun_out/r4/h_async1.json" \
  "h_async2:300:python bench.py --secondary pairwise_async --steps 20 --no-cpu-baseline > gpurun_out/r4/h_async2.json"

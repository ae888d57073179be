#!/bin/bash
# Round-4 check: the GPU suite, then the headline twice and the default bench.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
mkdir -p gpurun_out/r4base
export HSA_ENABLE_IPC_MODE_LEGACY=0
scripts/gpu_steps.sh \
  "gputests:700:python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread" \
  "h1:200:python bench.py --secondary none --steps 20 --no-cpu-baseline > gpurun_out/r4base/h1.json" \
  "h2:200:python bench.py --secondary none --steps 20 --no-cpu-baseline > gpurun_out/r4base/h2.json" \
  "def:400:python bench.py --no-cpu-baseline > gpurun_out/r4base/default.json"

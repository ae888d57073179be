#!/bin/bash
# Round 6, first GPU call: the stream-contract tests, the whole GPU suite, the default bench, the naive_xor counters.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0
mkdir -p gpurun_out/r6
scripts/gpu_steps.sh \
  "contract:300:python -u -m pytest tests/test_gpu_async.py tests/test_gpu_bsi.py -m gpu -x -v --timeout 120 --timeout-method thread" \
  "gputests:600:python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread" \
  "bench:400:python bench.py > gpurun_out/r6/bench_default.json" \
  "xorpmc:900:scripts/r06_xor_pmc.sh xdup1 xdup2 xdup3"

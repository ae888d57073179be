#!/bin/bash
# naive_xor with the next window's LDS-DMA issued from inline asm (no compiler vmcnt(0) at every window's
# first LDS access): wide parity, then A/B against the builtin DMA (abvar/xdma0).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0
scripts/gpu_steps.sh \
  "widetests:400:python -u -m pytest tests/test_gpu_wide.py tests/test_gpu_configs.py -m gpu -x -q --timeout 200 --timeout-method thread" \
  "xorab:400:scripts/r06_ab.sh r6xordma 3 'wide_runs_xor' '--workload wide_xor_runs --secondary none --steps 3 --warmup 1 --no-cpu-baseline' base xdma0"

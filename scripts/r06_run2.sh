#!/bin/bash
# naive_xor core-run de-duplication: parity tests, then an interleaved A/B against RBG_XOR_CORE=0 and a PMC pass.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0
scripts/gpu_steps.sh \
  "xortests:300:python -u -m pytest tests/test_gpu_configs.py tests/test_gpu_wide.py -m gpu -x -q --timeout 200 --timeout-method thread" \
  "xorab:600:scripts/r06_ab.sh r6xorab 2 'wide_runs_xor' '--workload wide_xor_runs --secondary none --steps 3 --warmup 1 --no-cpu-baseline' base xcore0" \
  "xorpmc:300:PMC_OUT=gpurun_out/r6xor_core scripts/r06_xor_pmc.sh"

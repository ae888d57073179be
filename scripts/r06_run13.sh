#!/bin/bash
# naive_xor mark-pass variants: the core run marked once per stretch (xcm), 4 mask copies (xmc4), both (xcm4);
# plus the SoA run-count normalization test on the product.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0
scripts/gpu_steps.sh \
  "wtest:300:python -u -m pytest tests/test_gpu_wide.py -m gpu -x -q --timeout 200 --timeout-method thread -k 'soa_run_count or runs_only or dense_run'" \
  || exit $?
scripts/gpu_steps.sh \
  "xorab:600:scripts/r06_ab.sh r6xormark 2 'wide_runs_xor' '--workload wide_xor_runs --secondary none --steps 3 --warmup 1 --no-cpu-baseline' base xcm xmc4 xcm4"

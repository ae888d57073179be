#!/bin/bash
# OR pairs with a large Bitmap operand on the copy + filter kernel (RBG_OR_BITS): pairwise parity, then (only if
# green) the config-2 OR / AND lines A/B against the register-path build (abvar/orbits0).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0
mkdir -p gpurun_out/r6orbits
scripts/gpu_steps.sh \
  "ortests:500:python -u -m pytest tests/test_gpu_or_bits.py tests/test_gpu_inplace.py tests/test_gpu_pairwise.py tests/test_gpu_type_pins.py tests/test_gpu_configs.py -m gpu -x -q --timeout 200 --timeout-method thread" \
  || exit $?
scripts/gpu_steps.sh \
  "orab:500:scripts/r06_ab.sh r6orbits 2 'k_pair_tasks' '--workload pairwise_or --secondary none --steps 5 --warmup 2 --no-cpu-baseline' base orbits0" \
  "benchor:200:python bench.py --workload pairwise_or --secondary none --steps 10 --warmup 3 --no-cpu-baseline > gpurun_out/r6orbits/bench_or.json" \
  "benchand:200:python bench.py --secondary none --steps 10 --warmup 3 --no-cpu-baseline > gpurun_out/r6orbits/bench_and.json"

#!/bin/bash
# naive_xor on 4-B member records (card summed from the runs): wide + config parity (stops if red), then the
# config-4 XOR line under rocprofv3 (kernel and setup times) and the plain bench line.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0
mkdir -p gpurun_out/r6xrec
scripts/gpu_steps.sh \
  "xtests:500:python -u -m pytest tests/test_gpu_wide.py tests/test_gpu_configs.py tests/test_gpu_type_pins.py tests/test_gpu_or_bits.py -m gpu -x -q --timeout 200 --timeout-method thread" \
  || exit $?
scripts/gpu_steps.sh \
  "xorprof:300:timeout -k 10 250 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r6xrec/prof -o run -- python3 bench.py --workload wide_xor_runs --secondary none --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/r6xrec/prof.log 2>&1" \
  "xorbench:300:python bench.py --workload wide_xor_runs --secondary none --steps 5 --warmup 2 --no-cpu-baseline > gpurun_out/r6xrec/bench_xor.json"

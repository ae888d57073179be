#!/bin/bash
# naive_xor's first-call record build overlapped with the kernel (two key chunks, side stream): wide parity (stops
# if red), then the config-4 XOR line with and without the overlap (RBGPU_KREC_NO_OVERLAP=1), twice each.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0
mkdir -p gpurun_out/r6kov
scripts/gpu_steps.sh \
  "wtests:500:python -u -m pytest tests/test_gpu_wide.py tests/test_gpu_configs.py -m gpu -x -q --timeout 200 --timeout-method thread" \
  || exit $?
scripts/gpu_steps.sh \
  "ov1:200:python bench.py --workload wide_xor_runs --secondary none --steps 5 --warmup 2 --no-cpu-baseline > gpurun_out/r6kov/ov1.json" \
  "seq1:200:RBGPU_KREC_NO_OVERLAP=1 python bench.py --workload wide_xor_runs --secondary none --steps 5 --warmup 2 --no-cpu-baseline > gpurun_out/r6kov/seq1.json" \
  "ov2:200:python bench.py --workload wide_xor_runs --secondary none --steps 5 --warmup 2 --no-cpu-baseline > gpurun_out/r6kov/ov2.json" \
  "seq2:200:RBGPU_KREC_NO_OVERLAP=1 python bench.py --workload wide_xor_runs --secondary none --steps 5 --warmup 2 --no-cpu-baseline > gpurun_out/r6kov/seq2.json" \
  "trace:300:timeout -k 10 250 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/r6kov/trace -o run -- python3 bench.py --workload wide_xor_runs --secondary none --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/r6kov/trace.log 2>&1"

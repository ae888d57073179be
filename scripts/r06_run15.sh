#!/bin/bash
# Small-batch kernel: block -> pair lookup by 64 parallel probes, compaction stores in slot order.  Parity of every
# small-path test (stops if red), the phase study (abvar/sstudy) and the census line.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0
mkdir -p gpurun_out/r6small
scripts/gpu_steps.sh \
  "stests:600:python -u -m pytest tests/test_gpu_pairwise.py tests/test_gpu_inplace.py tests/test_gpu_type_pins.py tests/test_gpu_async.py tests/test_gpu_roaring_api.py tests/test_gpu_longlong.py tests/test_gpu_configs.py -m gpu -x -q --timeout 200 --timeout-method thread" \
  || exit $?
scripts/gpu_steps.sh \
  "study:300:for op in OR AND XOR ANDNOT; do RBGPU_LIB=\$PWD/abvar/sstudy/librbgpu.so timeout -k 10 120 python scripts/micro/small_study.py \$op || exit 1; done > gpurun_out/r6small/study.txt 2>&1" \
  "census:300:python bench.py --workload pairwise_and --secondary census --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/r6small/census.json" \
  "census2:300:python bench.py --workload pairwise_and --secondary census --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/r6small/census2.json"

#!/bin/bash
# One GPU call: bench.py over librbgpu's one-rank RCCL communicator (the C-ABI exchange path at N = 1)
# for pairwise, BSI and wide lines, then the RBG_STUDY build on the OR line (per-phase heavy/light timing).
set -o pipefail
mkdir -p gpurun_out/comm
export HSA_ENABLE_IPC_MODE_LEGACY=0
RBGPU_BENCH_COMM=rccl1 timeout -k 10 240 python -u bench.py --workload pairwise_and \
  --secondary bsi_range,wide_or,wide_and_runs --steps 5 --warmup 2 --no-cpu-baseline \
  > gpurun_out/comm/rccl1.json 2> gpurun_out/comm/rccl1.err || exit $?
RBGPU_LIB=abvar/study/librbgpu.so RBG_STUDY=1 timeout -k 10 180 python -u bench.py --workload pairwise_or \
  --secondary none --steps 2 --warmup 1 --no-cpu-baseline \
  > gpurun_out/comm/study_or.json 2> gpurun_out/comm/study_or.err || exit $?
RBGPU_LIB=abvar/study/librbgpu.so RBG_STUDY=1 timeout -k 10 180 python -u bench.py --workload pairwise_andnot \
  --secondary none --steps 2 --warmup 1 --no-cpu-baseline \
  > gpurun_out/comm/study_andnot.json 2> gpurun_out/comm/study_andnot.err

#!/bin/bash
# naive_xor occupancy sensitivity (RBG_XOR_LDS_PAD: 2 waves/SIMD) and the core dedupe again; workShyAnd reading the
# SoA directly (RBG_AND_SOA) against the packed records: parity and an interleaved A/B with the records pass.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0
scripts/gpu_steps.sh \
  "asoatests:300:RBGPU_LIB=$PWD/abvar/asoa1/librbgpu.so python -u -m pytest tests/test_gpu_configs.py tests/test_gpu_wide.py -m gpu -x -q --timeout 200 --timeout-method thread -k 'config4 or wide'" \
  "xorab:600:scripts/r06_ab.sh r6xorab3 2 'wide_runs_xor' '--workload wide_xor_runs --secondary none --steps 3 --warmup 1 --no-cpu-baseline' base xpad2 xcore1" \
  "andab:600:scripts/r06_ab.sh r6andab 2 'wide_runs_and|pack_records' '--workload wide_and_runs --secondary none --steps 3 --warmup 1 --no-cpu-baseline' base asoa1" || { rc=$?; [ $rc -ge 124 ] && exit $rc; }
mkdir -p gpurun_out/r6calib
scripts/gpu_steps.sh \
  "calib_time:120:scripts/micro/fetch_calib > gpurun_out/r6calib/time.txt" \
  "calib_fetch:120:timeout -s KILL 100 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/r6calib/p1 -o run -- scripts/micro/fetch_calib" \
  "calib_req:120:timeout -s KILL 100 rocprofv3 --pmc TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_32B_sum TCC_BUBBLE_sum --output-format csv -d gpurun_out/r6calib/p2 -o run -- scripts/micro/fetch_calib"

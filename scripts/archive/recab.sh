#!/bin/bash
# Task-record prefetch check: the pairwise GPU tests on the in-tree library, then an interleaved A/B of
# the config-2 bench (abvar/base = previous tree) and OR/XOR/ANDNOT lines, then the RBG_STUDY phase
# split of the AND line.  Every GPU step has its own limit; the first failure ends the call.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/rec
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread \
  tests/test_gpu_pairwise.py tests/test_gpu_type_pins.py tests/test_gpu_configs.py \
  > gpurun_out/rec/tests.txt 2>&1 || { tail -30 gpurun_out/rec/tests.txt; exit 1; }
tail -2 gpurun_out/rec/tests.txt
scripts/ab.sh base1 abvar/base/librbgpu.so new1 default base2 abvar/base/librbgpu.so new2 default || exit 1
for t in base1 new1 base2 new2; do
  python -c "import json;d=json.loads(open('gpurun_out/ab/$t.json').read().splitlines()[-1]);r=d['roofline'];print('$t',d['ms_per_step'],r.get('kernel_ms'),r['frac'])"
done
OPAB_WORKLOADS="pairwise_or pairwise_xor pairwise_andnot" bash scripts/opab.sh base main || exit 1
RBGPU_LIB=abvar/study/librbgpu.so RBG_STUDY=1 timeout -k 10 180 python -u bench.py --workload pairwise_and \
  --secondary none --steps 2 --warmup 1 --no-cpu-baseline \
  > gpurun_out/rec/study_and.json 2> gpurun_out/rec/study_and.err

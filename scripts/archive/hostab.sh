#!/bin/bash
# Host-phase kernels after a change: the GPU test suite on the in-tree library, an interleaved
# A/B of the config-2 bench against abvar/base (the previous tree), and a kernel-trace profile of each
# library (per-kernel averages of the count / scan / emit / compaction launches).  Every GPU step has
# its own limit; the first failure ends the call.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/host
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 600 python -u -m pytest -x -q -m gpu --timeout 120 --timeout-method thread tests \
  > gpurun_out/host/tests.txt 2>&1 || { tail -30 gpurun_out/host/tests.txt; exit 1; }
tail -2 gpurun_out/host/tests.txt
scripts/ab.sh base1 abvar/base/librbgpu.so new1 default base2 abvar/base/librbgpu.so new2 default || exit 1
for t in base1 new1 base2 new2; do
  python -c "import json;d=json.loads(open('gpurun_out/ab/$t.json').read().splitlines()[-1]);r=d['roofline'];print('$t',d['ms_per_step'],r.get('kernel_ms'),r['frac'],d['config']['roofline_pct_whole_step'])"
done
cd /tmp && export TMPDIR=/tmp
for v in base new; do
  lib=$GRAFT_REPO_ROOT/abvar/base/librbgpu.so; [ $v = new ] && lib=$GRAFT_REPO_ROOT/roaringbitmap_amd/librbgpu.so
  RBGPU_LIB=$lib timeout -k 10 240 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/host/prof_$v -o p -- \
    python $GRAFT_REPO_ROOT/bench.py --secondary none --steps 5 --warmup 2 --no-cpu-baseline \
    > $GRAFT_REPO_ROOT/gpurun_out/host/prof_$v.json 2>&1 || exit 1
done

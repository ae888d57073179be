#!/bin/bash
# The GPU suite on the in-tree library, then the BSI RANGE line against abvar/prev (the tree before).
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/bsi
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 600 python -u -m pytest -x -q -m gpu --timeout 120 --timeout-method thread tests \
  > gpurun_out/bsi/tests.txt 2>&1 || { tail -30 gpurun_out/bsi/tests.txt; exit 1; }
tail -2 gpurun_out/bsi/tests.txt
for v in prev main prev main; do
  lib=abvar/$v/librbgpu.so; [ $v = main ] && lib=roaringbitmap_amd/librbgpu.so
  RBGPU_LIB=$lib timeout -k 10 200 python -u bench.py --workload bsi_range --secondary none --no-cpu-baseline \
    > gpurun_out/bsi/$v.json 2>/dev/null || exit 1
  python -c "import json;d=json.loads([x for x in open('gpurun_out/bsi/$v.json') if x.startswith('{')][-1]);r=d['roofline'];print('$v',d['ms_per_step'],r['kernel_ms'],r['frac'],d['value'])"
done

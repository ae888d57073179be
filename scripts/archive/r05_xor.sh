#!/bin/bash
# Config-4 naive_xor: its parity tests, then the wide_xor_runs bench line (in-tree library).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
O=gpurun_out/r5xor
mkdir -p $O
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 400 python -u -m pytest tests/test_gpu_wide.py tests/test_gpu_configs.py -x -q --timeout 200 --timeout-method thread -k "xor or XOR or runs or config4" > $O/tests.txt 2>&1 || { tail -30 $O/tests.txt; exit 1; }
tail -1 $O/tests.txt
for v in "$@"; do
  lib=abvar/$v/librbgpu.so; [ "$v" = main ] && lib=roaringbitmap_amd/librbgpu.so
  RBGPU_LIB=$lib timeout -k 10 300 python bench.py --no-cpu-baseline --secondary none --workload wide_xor_runs --steps 10 > $O/$v.json 2>$O/$v.err || { tail $O/$v.err; exit 1; }
  python - $O/$v.json $v <<'PY'
import json, sys
for l in open(sys.argv[1]):
    if l.startswith('{'): d = json.loads(l)
print(sys.argv[2], d.get('ms_per_step'), d.get('roofline', {}).get('kernel_ms'), d.get('roofline', {}).get('frac'), d.get('ms_per_step_with_setup'))
PY
done

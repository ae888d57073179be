#!/bin/bash
# BSI RANGE (config 5): parity, then the line with the key count from the host CSR (main) against the
# read-back build (abvar/bsiold), interleaved.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
O=gpurun_out/r5bsi
mkdir -p $O
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 600 python -u -m pytest tests/test_gpu_bsi.py tests/test_gpu_configs.py tests/test_gpu_comm.py -x -q --timeout 200 --timeout-method thread > $O/tests.txt 2>&1 || { tail -30 $O/tests.txt; exit 1; }
tail -1 $O/tests.txt
for round in 1 2 3; do
  for v in main bsiold; do
    lib=abvar/$v/librbgpu.so; [ "$v" = main ] && lib=roaringbitmap_amd/librbgpu.so
    RBGPU_LIB=$lib timeout -k 10 300 python bench.py --no-cpu-baseline --secondary none --workload bsi_range --steps 20 > $O/${v}_$round.json 2>$O/${v}_$round.err || { tail $O/${v}_$round.err; exit 1; }
    python - $O/${v}_$round.json $v $round <<'PY'
import json, sys
d = [json.loads(l) for l in open(sys.argv[1]) if l.startswith('{')][-1]
print(sys.argv[2], sys.argv[3], d["ms_per_step"], d["roofline"]["frac"], d["roofline"].get("kernel_ms"))
PY
  done
done

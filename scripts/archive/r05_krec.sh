#!/bin/bash
# naive_xor key-major record build (k_records_direct) by tile shape: the config-4 XOR line's setup parts.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
O=gpurun_out/r5krec
mkdir -p $O
export HSA_ENABLE_IPC_MODE_LEGACY=0
for t in "$@"; do
  RBGPU_KREC_GROUP=$t timeout -k 10 300 python bench.py --no-cpu-baseline --secondary none --workload wide_xor_runs --steps 3 > $O/t$t.json 2>$O/t$t.err || { tail $O/t$t.err; exit 1; }
  python - $O/t$t.json $t <<'PY'
import json, sys
d = [json.loads(l) for l in open(sys.argv[1]) if l.startswith('{')][-1]
print("tile", sys.argv[2], d["ms_per_step"], json.dumps(d["config"]["setup"]["parts"]))
PY
done
RBGPU_KREC_GROUP=${KEEP:-8} timeout -k 10 300 python -u -m pytest tests/test_gpu_configs.py tests/test_gpu_wide.py -x -q --timeout 200 --timeout-method thread -k "xor or XOR or config4" > $O/tests.txt 2>&1; tail -1 $O/tests.txt

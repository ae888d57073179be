#!/bin/bash
# BSI / sharding parity, the BSI line, then the N=2 rehearsals (default command and per workload).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
O=gpurun_out/r5fn2
mkdir -p $O
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 600 python -u -m pytest tests/test_gpu_bsi.py tests/test_gpu_configs.py tests/test_gpu_comm.py tests/test_gpu_wide.py -x -q --timeout 200 --timeout-method thread > $O/tests.txt 2>&1 || { tail -30 $O/tests.txt; exit 1; }
tail -1 $O/tests.txt
timeout -k 10 300 python bench.py --no-cpu-baseline --secondary none --workload bsi_range --steps 20 > $O/bsi.json 2>$O/bsi.err || { tail $O/bsi.err; exit 1; }
python - $O/bsi.json <<'PY'
import json, sys
d = [json.loads(l) for l in open(sys.argv[1]) if l.startswith('{')][-1]
print("bsi", d["ms_per_step"], d["roofline"]["frac"], d["roofline"]["kernel_ms"], d["config"]["ms_per_step_with_setup"])
PY
bash scripts/r05_rehearse_default.sh || exit 1
bash scripts/rehearse_n2.sh || exit 1

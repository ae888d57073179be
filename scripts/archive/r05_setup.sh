#!/bin/bash
# Config-4 setup: naive_xor / workShyAnd parity tests, then both wide lines with their fresh-set setup.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
O=gpurun_out/r5setup
mkdir -p $O
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 400 python -u -m pytest tests/test_gpu_wide.py tests/test_gpu_configs.py tests/test_gpu_comm.py -x -q --timeout 200 --timeout-method thread > $O/tests.txt 2>&1 || { tail -30 $O/tests.txt; exit 1; }
tail -1 $O/tests.txt
timeout -k 10 400 python bench.py --no-cpu-baseline --secondary wide_xor_runs,wide_and_runs --steps 5 > $O/bench.json 2>$O/bench.err || { tail $O/bench.err; exit 1; }
python - $O/bench.json <<'PY'
import json, sys
d = [json.loads(l) for l in open(sys.argv[1]) if l.startswith('{')][-1]
for k in ("wide_xor_runs", "wide_and_runs"):
    w = d["secondary"][k]
    print(k, w["ms_per_step"], w["roofline"]["kernel_ms"], w["roofline"]["frac"], "setup", json.dumps(w["setup"]["parts"]),
          "with_setup", w["ms_per_step_with_setup"], w["value_with_setup"])
PY

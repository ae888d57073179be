#!/bin/bash
# Setup parts timed from an empty dispatch (DeriveTimer): the wide lines and the BSI line, with their
# setup-inclusive steps.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
O=gpurun_out/r5setup2
mkdir -p $O
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 600 python bench.py --no-cpu-baseline --secondary wide_xor_runs,wide_and_runs,bsi_range --steps 5 > $O/bench.json 2>$O/bench.err || { tail $O/bench.err; exit 1; }
python - $O/bench.json <<'PY'
import json, sys
d = [json.loads(l) for l in open(sys.argv[1]) if l.startswith('{')][-1]
for k in ("wide_xor_runs", "wide_and_runs", "bsi_range"):
    w = d["secondary"][k]
    print(k, "step", w["ms_per_step"], "kernel", w["roofline"]["kernel_ms"], "frac", w["roofline"]["frac"], "setup",
          json.dumps(w["setup"].get("parts", w["setup"]["ms"])), "with_setup", w["ms_per_step_with_setup"], w["value_with_setup"])
PY

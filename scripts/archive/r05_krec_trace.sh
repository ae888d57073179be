#!/bin/bash
# Config-4 XOR line under a kernel trace: the key-major record build's kernel time against the setup timer.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
O=gpurun_out/r5kt
mkdir -p $O
export HSA_ENABLE_IPC_MODE_LEGACY=0 TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof -o run -- python3 bench.py --no-cpu-baseline --secondary none --workload wide_xor_runs --steps 3 > $O/bench.json 2>$O/bench.err || { tail $O/bench.err; exit 1; }
python3 - $O <<'PY'
import json, sys, glob, csv
O = sys.argv[1]
d = [json.loads(l) for l in open(O + "/bench.json") if l.startswith('{')][-1]
print("timer", json.dumps(d["config"]["setup"]["parts"]))
for f in glob.glob(O + "/prof/**/*kernel_stats.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        if "records" in r["Name"] or "dense" in r["Name"]:
            print(r["Name"][:60], r["Calls"], float(r["AverageNs"]) / 1e6, "ms")
PY

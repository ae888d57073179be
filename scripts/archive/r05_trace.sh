#!/bin/bash
# Kernel trace of one bench workload (rocprofv3 --kernel-trace, sqlite output): the last steps' kernels with
# their gaps.  usage: r05_trace.sh WORKLOAD STEPS
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
W=${1:-bsi_range}; N=${2:-5}
O=gpurun_out/r5trace_$W
mkdir -p $O
export HSA_ENABLE_IPC_MODE_LEGACY=0 TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace -d $O/prof -o run -- python3 bench.py --no-cpu-baseline --secondary none --workload $W --steps $N --warmup 2 > $O/bench.json 2>$O/bench.err || { tail $O/bench.err; exit 1; }
python3 - $O <<'PY'
import glob, json, sqlite3, sys
O = sys.argv[1]
d = [json.loads(l) for l in open(O + "/bench.json") if l.startswith('{')][-1]
print("ms_per_step", d["ms_per_step"])
db = glob.glob(O + "/prof/**/*.db", recursive=True)[0]
rows = list(sqlite3.connect(db).execute("select name,start,end from kernels order by start"))
tail = rows[-60:]
t0 = tail[0][1]; prev = None
for n, s, e in tail:
    gap = (s - prev) / 1e3 if prev else 0.0
    print(f"{(s - t0) / 1e3:10.1f} gap {gap:7.1f} dur {(e - s) / 1e3:8.1f}  {n[:70]}")
    prev = e
PY

#!/bin/bash
# Instruction-cache counters of the task kernels (config 2 OR) and the small-batch kernel (census OR): are the
# 70-83 KB kernels fetch-bound?  One pass per counter set.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0
o=gpurun_out/r6icache; mkdir -p $o
run() { # name counters... -- command
  local n=$1; shift; local c=(); while [ "$1" != "--" ]; do c+=("$1"); shift; done; shift
  timeout -s KILL 150 rocprofv3 --pmc "${c[@]}" --output-format csv -d $o/$n -o run -- "$@" > $o/$n.log 2>&1 || { echo "FAIL $n"; tail -3 $o/$n.log; return 1; }
}
B="python3 bench.py --workload pairwise_or --secondary none --steps 2 --warmup 1 --no-cpu-baseline"
S="python3 scripts/micro/small_study.py OR"
run or_ic SQC_ICACHE_HITS SQC_ICACHE_MISSES SQC_ICACHE_MISSES_DUPLICATE -- $B && \
run or_wait SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_IFETCH -- $B && \
run sm_ic SQC_ICACHE_HITS SQC_ICACHE_MISSES SQC_ICACHE_MISSES_DUPLICATE -- $S && \
run sm_wait SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_IFETCH -- $S && \
python3 - $o > $o/summary.txt 2>&1 <<'PY'
import csv, glob, sys, collections, os
root = sys.argv[1]
for d in sorted(glob.glob(f"{root}/*/run_counter_collection.csv")):
    agg = collections.defaultdict(lambda: collections.defaultdict(list))
    for row in csv.DictReader(open(d)):
        name = row["Kernel_Name"].split("(")[0].replace("void ", "")
        if not any(k in name for k in ("k_pair_tasks", "k_pair_small")): continue
        agg[name][row["Counter_Name"]].append(float(row["Counter_Value"]))
        agg[name]["_dur_ns"].append(float(row["End_Timestamp"]) - float(row["Start_Timestamp"]))
    print("==", os.path.basename(os.path.dirname(d)))
    for name, cs in agg.items():
        print(" ", name, " ".join(f"{k}={sum(v)/len(v):.4g}" for k, v in sorted(cs.items())))
PY
cat $o/summary.txt

#!/bin/bash
# Interleaved A/B of kernel variants by rocprofv3 kernel trace (one box): for each round, each library in turn runs
# the given bench command; the per-kernel average of the named kernels is printed per run.
# usage: scripts/r06_ab.sh <out> <rounds> "<kernel regex>" "<bench args>" lib1 lib2 ...   (lib "base" = the product)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
out=gpurun_out/$1; rounds=$2; pat=$3; args=$4; shift 4
mkdir -p $out
export TMPDIR=/tmp
for r in $(seq 1 $rounds); do
  for v in "$@"; do
    if [ "$v" = base ]; then unset RBGPU_LIB; else export RBGPU_LIB=$PWD/abvar/$v/librbgpu.so; fi
    d=$out/$v.$r
    timeout -k 10 150 rocprofv3 --kernel-trace --stats --output-format csv -d $d -o run -- python3 bench.py $args > $d.log 2>&1 || { echo "FAIL $v $r"; tail -5 $d.log; exit 1; }
    python3 - "$d" "$v" "$r" "$pat" <<'PY'
import csv, re, sys
d, v, r, pat = sys.argv[1:5]
for row in csv.DictReader(open(f"{d}/run_kernel_stats.csv")):
    if re.search(pat, row["Name"]):
        print(f"{v:10s} r{r} {row['Name'][:44]:44s} n={row['Calls']:>4s} avg {float(row['AverageNs'])/1e6:.4f} ms")
PY
  done
done | tee $out/summary.txt

#!/bin/bash
# naive_xor per-key trace (RBG_STUDY builds): stretch counts and phase cycles of three keys.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
O=gpurun_out/r5xor
mkdir -p $O
export HSA_ENABLE_IPC_MODE_LEGACY=0
for v in "$@"; do
  RBGPU_LIB=abvar/$v/librbgpu.so timeout -k 10 300 python bench.py --no-cpu-baseline --secondary none --workload wide_xor_runs --steps 1 --warmup 0 > $O/$v.study.txt 2>&1 || { tail $O/$v.study.txt; exit 1; }
  echo "== $v"; grep "xor trace" $O/$v.study.txt | sort | uniq | head -6
done

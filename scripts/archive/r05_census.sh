#!/bin/bash
# Census (config 1) latency variants: per-call wall time and kernel split (RBGPU_SMALL_KERNEL_TIMES=1).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
O=gpurun_out/r5census
mkdir -p $O
export HSA_ENABLE_IPC_MODE_LEGACY=0
for v in "$@"; do
  for kt in 0 1; do
    env $v RBGPU_SMALL_KERNEL_TIMES=$kt timeout -k 10 120 python scripts/census_lat.py --calls 200 > $O/${v//[=]/_}_kt$kt.json || exit 1
    echo "$v kt=$kt $(cat $O/${v//[=]/_}_kt$kt.json)"
  done
done

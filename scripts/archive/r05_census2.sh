#!/bin/bash
# Census latency vs batch size (1 / 10 / 50 / 199 pairs), with the kernel split.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
O=gpurun_out/r5census
mkdir -p $O
export HSA_ENABLE_IPC_MODE_LEGACY=0
for v in "$@"; do
  for np in 1 10 50 199; do
    env $v RBGPU_SMALL_KERNEL_TIMES=1 timeout -k 10 120 python scripts/census_lat.py --calls 100 --npairs $np > $O/np${np}_${v//[=]/_}.json || exit 1
    echo "$v np=$np $(cat $O/np${np}_${v//[=]/_}.json)"
  done
done

#!/bin/bash
# Census call timeline per block (study builds abvar/<name>, scripts/small_stamps_variant.py), then the
# census latency of the same builds without stamps' output.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
O=gpurun_out/r5stamps
mkdir -p $O
export HSA_ENABLE_IPC_MODE_LEGACY=0
for v in "$@"; do
  RBGPU_LIB=abvar/$v/librbgpu.so RBGPU_SMALL_STAMPS=1 timeout -k 10 120 python scripts/census_lat.py --calls 3 > $O/$v.json 2> $O/$v.err || { tail $O/$v.err; exit 1; }
  echo "== $v"; grep -A4 "stamps blocks" $O/$v.err | tail -10
done
for v in "$@"; do
  RBGPU_LIB=abvar/$v/librbgpu.so timeout -k 10 120 python scripts/census_lat.py --calls 200 > $O/$v.lat.json || exit 1
  echo "$v $(cat $O/$v.lat.json)"
done

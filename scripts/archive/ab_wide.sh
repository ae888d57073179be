#!/bin/bash
# A/B of kernel variants on config 3 (FastAggregation.or of 1024 dense bitmaps): scripts/ab_wide.sh <tag> <lib|default> ...
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
mkdir -p gpurun_out/ab
while [ $# -ge 2 ]; do
  tag=$1; lib=$2; shift 2
  if [ "$lib" = default ]; then unset RBGPU_LIB; else export RBGPU_LIB=$lib; fi
  timeout -k 10 240 python -u bench.py --workload wide_or --secondary none --census 0 --bsi 0 --no-cpu-baseline --steps 5 --warmup 2 > gpurun_out/ab/$tag.json 2> gpurun_out/ab/$tag.err || exit 1
done

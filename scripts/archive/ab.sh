#!/bin/bash
# A/B of kernel variants on the config-2 bench: scripts/ab.sh <tag> <lib-or-default> [env...] (repeated pairs)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
mkdir -p gpurun_out/ab
while [ $# -ge 2 ]; do
  tag=$1; lib=$2; shift 2
  if [ "$lib" = default ]; then unset RBGPU_LIB; else export RBGPU_LIB=$lib; fi
  timeout -k 10 200 python -u bench.py --secondary none --no-cpu-baseline > gpurun_out/ab/$tag.json 2> gpurun_out/ab/$tag.err || exit 1
done

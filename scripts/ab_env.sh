#!/bin/bash
# A/B of runtime knobs on the config-2 bench: scripts/ab_env.sh <tag> "<VAR=val ...|->" ... (pairs)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
mkdir -p gpurun_out/ab
while [ $# -ge 2 ]; do
  tag=$1; envs=$2; shift 2
  [ "$envs" = "-" ] && envs=""
  env $envs timeout -k 10 200 python -u bench.py --secondary none --census 0 --bsi 0 --no-cpu-baseline > gpurun_out/ab/$tag.json 2> gpurun_out/ab/$tag.err || exit 1
done

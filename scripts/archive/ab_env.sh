#!/bin/bash
# A/B of runtime knobs on the config-2 bench: scripts/ab_env.sh <tag> "<VAR=val ...|->" ... (pairs)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
mkdir -p gpurun_out/ab
while [ $# -ge 2 ]; do
  tag=$1; envs=$2; shift 2
  [ "$envs" = "-" ] && envs=""
  env $envs timeout -k 10 200 python -u bench.py --secondary none --no-cpu-baseline > gpurun_out/ab/$tag.json 2> gpurun_out/ab/$tag.err || exit 1
  python -c "import json;d=json.loads(open('gpurun_out/ab/$tag.json').read().splitlines()[-1]);r=d['roofline'];print('$tag',d['ms_per_step'],d['step_ms'],r.get('kernel_ms'),r['frac'],d['config']['roofline_pct_whole_step'])"
done

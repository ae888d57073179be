#!/bin/bash
# A/B of config-2 headline variants: abvar/<name>/librbgpu.so ("main" = the in-tree library),
# interleaved, each a full bench run of the headline (20 steps).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
mkdir -p gpurun_out/ab
export HSA_ENABLE_IPC_MODE_LEGACY=0
for round in 1 2; do
  for v in "$@"; do
    lib=abvar/$v/librbgpu.so; [ "$v" = main ] && lib=roaringbitmap_amd/librbgpu.so
    RBGPU_LIB=$lib timeout -k 10 150 python bench.py --no-cpu-baseline --secondary none --steps 20 > gpurun_out/ab/c2_${v}_$round.json || exit 1
    python -c "import json;d=json.loads(open('gpurun_out/ab/c2_${v}_$round.json').read().splitlines()[-1]);r=d['roofline'];k=r['kernels'];print('$v', $round, d['ms_per_step'],r['kernel_ms'],r['frac'],d['config']['roofline_pct_whole_step'],k['k_pair_tasks<light>']['ms'],k['k_pair_tasks<heavy>']['ms'])"
  done
done

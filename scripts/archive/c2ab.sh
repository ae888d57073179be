# A/B timing of config-2 (headline) kernel variants: abvar/<name>/librbgpu.so, "main" = the in-tree library
cd $GRAFT_REPO_ROOT
for v in "$@"; do
  lib=abvar/$v/librbgpu.so; [ "$v" = main ] && lib=roaringbitmap_amd/librbgpu.so
  RBGPU_LIB=$lib timeout -k 10 120 python bench.py --no-cpu-baseline --secondary none > gpurun_out/c2_$v.json || exit 1
  python -c "import json;d=json.loads(open('gpurun_out/c2_$v.json').read().splitlines()[-1]);r=d['roofline'];k=r['kernels'];print('$v',d['ms_per_step'],r['kernel_ms'],r['frac'],k['k_pair_tasks<light>']['ms'],k['k_pair_tasks<heavy>']['ms'])"
done

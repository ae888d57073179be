# A/B timing of config-4 XOR kernel variants (abvar/<name>/librbgpu.so; "main" = the in-tree library)
cd $GRAFT_REPO_ROOT
for v in "$@"; do
  lib=abvar/$v/librbgpu.so; [ "$v" = main ] && lib=roaringbitmap_amd/librbgpu.so
  RBGPU_LIB=$lib timeout -k 10 120 python bench.py --workload wide_xor_runs --steps 5 --warmup 2 --no-cpu-baseline --secondary none > gpurun_out/c4_$v.json || exit 1
  python -c "import json;d=json.loads(open('gpurun_out/c4_$v.json').read().splitlines()[-1]);print('$v',d['ms_per_step'],d['roofline']['kernel_ms'])"
done

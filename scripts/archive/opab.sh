# A/B of the pairwise OR / XOR secondary lines: abvar/<name>/librbgpu.so, "main" = the in-tree library
cd $GRAFT_REPO_ROOT
for v in "$@"; do
  lib=abvar/$v/librbgpu.so; [ "$v" = main ] && lib=roaringbitmap_amd/librbgpu.so
  for w in ${OPAB_WORKLOADS:-pairwise_or pairwise_xor}; do
    RBGPU_LIB=$lib timeout -k 10 120 python bench.py --workload $w --steps 3 --warmup 1 --no-cpu-baseline --secondary none > gpurun_out/op_${v}_$w.json || exit 1
    python -c "import json;d=json.loads(open('gpurun_out/op_${v}_$w.json').read().splitlines()[-1]);print('$v','$w',d['ms_per_step'],d['roofline']['kernel_ms'],d['roofline']['frac'])"
  done
done

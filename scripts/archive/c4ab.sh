#!/bin/bash
# A/B timing of config-4 kernel variants (abvar/<name>/librbgpu.so; "main" = the in-tree library),
# interleaved: C4AB_WORKLOAD (default wide_xor_runs), C4AB_ROUNDS rounds over the variants.
cd $GRAFT_REPO_ROOT
wl=${C4AB_WORKLOAD:-wide_xor_runs}
for r in $(seq ${C4AB_ROUNDS:-1}); do
for v in "$@"; do
  lib=abvar/$v/librbgpu.so; [ "$v" = main ] && lib=roaringbitmap_amd/librbgpu.so
  RBGPU_LIB=$lib timeout -k 10 120 python bench.py --workload $wl --steps 5 --warmup 2 --no-cpu-baseline --secondary none > gpurun_out/c4_${v}_$r.json || exit 1
  python -c "import json;d=json.loads([l for l in open('gpurun_out/c4_${v}_$r.json') if l.startswith('{')][-1]);print('$wl $v',d['ms_per_step'],d['roofline']['kernel_ms'])"
done
done

#!/bin/bash
# A/B of library variants on the four config-2 ops: abvar/<name>/librbgpu.so ("main" = in-tree), interleaved.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
O=gpurun_out/r5ops
mkdir -p $O
export HSA_ENABLE_IPC_MODE_LEGACY=0
for round in 1 2; do
  for v in "$@"; do
    lib=abvar/$v/librbgpu.so; [ "$v" = main ] && lib=roaringbitmap_amd/librbgpu.so
    RBGPU_LIB=$lib timeout -k 10 300 python bench.py --no-cpu-baseline --secondary pairwise_ops --steps 10 > $O/${v}_$round.json || exit 1
    python - "$O/${v}_$round.json" "$v" "$round" <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().splitlines()[-1])
out = [f"AND {d['ms_per_step']} {d['roofline']['frac']}"]
for k, w in d["secondary"].items():
    out.append(f"{k[9:]} {w['ms_per_step']} {w['roofline']['frac']}")
print(sys.argv[2], sys.argv[3], " | ".join(out))
PY
  done
done

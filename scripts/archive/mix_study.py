"""Light / heavy kernel time per container-type mix of config 2 (kernel study, not the bench).

usage: python scripts/mix_study.py [--pairs N]
"""
import argparse
import ctypes as C
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import roaringbitmap_amd as rb  # noqa: E402
from roaringbitmap_amd import _lib as L  # noqa: E402

p = argparse.ArgumentParser()
p.add_argument("--pairs", type=int, default=300_000)
args = p.parse_args()
lib = L.lib()
lib.rbgpu_internal_set_mix.argtypes = [C.c_int] * 4
MIXES = {  # (filter A, A+B, posting A, A+B) cumulative per mille
    "default": (400, 700, 700, 800),
    "F_bitmap__P_array": (0, 1000, 1000, 1000),
    "F_run__P_array": (0, 0, 1000, 1000),
    "F_array__P_array": (1000, 1000, 1000, 1000),
    "F_bitmap__P_bitmap": (0, 1000, 0, 1000),
    "F_run__P_run": (0, 0, 0, 0),
    "F_bitmap__P_run": (0, 1000, 0, 0),
}
ctx = rb.Context(0)
out = {}
for name, m in MIXES.items():
    lib.rbgpu_internal_set_mix(*m)
    a, b = ctx.generate(rb.WL_FILTER_POSTING, args.pairs, seed=42)
    for _ in range(2):
        ctx.pairwise(rb.AND, a, b).close()
    ks = {}
    for _ in range(5):
        ctx.pairwise(rb.AND, a, b).close()
        for k in ctx.stats()["kernels"]:
            ks.setdefault(k["name"], []).append((k["ms"], k["bytes"], k["items"]))
    out[name] = {n: {"ms": round(sorted(v)[2][0], 4), "items": v[0][2], "GB/s": round(v[0][1] / sorted(v)[2][0] / 1e6, 1),
                     "ns_per_task": round(sorted(v)[2][0] * 1e6 / max(v[0][2], 1), 1)} for n, v in ks.items()}
    a.close()
    b.close()
lib.rbgpu_internal_set_mix(*MIXES["default"])
print(json.dumps(out, indent=1))

"""Roofline study for the pairwise task kernel (config 2): times the product kernel, its read-only
twin (same schedule and payload loads, no compute) and a streaming read of one arena.

usage: [RBGPU_LIB=scratch/<variant>/librbgpu.so] python scripts/probe.py [--pairs N] [--op 0]
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
p.add_argument("--pairs", type=int, default=1_000_000)
p.add_argument("--op", type=int, default=0)
p.add_argument("--reps", type=int, default=5)
args = p.parse_args()
lib = L.lib()
lib.rbgpu_internal_probe.restype = C.c_int
lib.rbgpu_internal_probe.argtypes = [C.c_void_p, C.c_int, C.c_void_p, C.c_void_p, C.c_uint32, C.c_int]
ctx = rb.Context(0)
a, b = ctx.generate(rb.WL_FILTER_POSTING, args.pairs, seed=42)
res = {"lib": os.environ.get("RBGPU_LIB", "default")}
for name, mode in (("product", 0), ("task_reads", 1), ("stream_read", 2)):
    ms = []
    for _ in range(args.reps):
        if mode == 0:
            ctx.pairwise(args.op, a, b).close()
        else:
            L.check(lib.rbgpu_internal_probe(ctx.h, args.op, a.h, b.h, args.pairs, mode))
        ms.append(ctx.stats()["main_kernel_ms"])
    ms_med = sorted(ms)[len(ms) // 2]
    byts = ctx.stats()["main_kernel_bytes"]
    res[name] = {"ms": round(ms_med, 4), "bytes": int(byts), "GB/s": round(byts / ms_med / 1e6, 1)}
print(json.dumps(res))

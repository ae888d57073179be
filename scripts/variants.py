"""Builds kernel variants of librbgpu as abvar/<name>/librbgpu.so (select one with RBGPU_LIB=...).

usage: python scripts/variants.py name:DEF=1,DEF2=3 ...
"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from roaringbitmap_amd import build as b  # noqa: E402

for spec in sys.argv[1:]:
    name, _, defs = spec.partition(":")
    os.makedirs(os.path.join(ROOT, "abvar", name), exist_ok=True)
    # the .so goes to abvar/ (travels with gpurun; git-ignored), objects to scratch/ (stays here)
    out = b.build(defines=[x for x in defs.split(",") if x], out=os.path.join(ROOT, "abvar", name, "librbgpu.so"),
                  obj=os.path.join(ROOT, "scratch", name, "obj"))
    print(out)

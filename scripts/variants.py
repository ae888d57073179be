"""Builds kernel variants of librbgpu under scratch/<name>/ (select one with RBGPU_LIB=...).

usage: python scripts/variants.py name:DEF=1,DEF2=3 ...
"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from roaringbitmap_amd import build as b  # noqa: E402

for spec in sys.argv[1:]:
    name, _, defs = spec.partition(":")
    d = os.path.join(ROOT, "scratch", name)
    out = b.build(defines=[x for x in defs.split(",") if x], out=os.path.join(d, "librbgpu.so"),
                  obj=os.path.join(d, "obj"))
    print(out)

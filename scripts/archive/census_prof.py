"""Config 1 (census1881, 199 consecutive pairs x and/or/xor/andNot) in a loop, for rocprofv3 runs
of the small-batch pairwise kernels.  usage: python scripts/census_prof.py [iterations]"""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402
import roaringbitmap_amd as rb  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 50
ctx = rb.Context(0)
vals = bench.load_census()
s = ctx.upload_values(vals)
ai = np.arange(len(vals) - 1, dtype=np.uint32)
bi = ai + 1
for _ in range(n):
    for op in (rb.AND, rb.OR, rb.XOR, rb.ANDNOT):
        ctx.pairwise(op, s, s, ai, bi).close()
ctx.synchronize()
print("done", n)

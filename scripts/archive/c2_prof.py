"""Config 2 (1M generated filter/posting pairs) batched pairwise calls in a loop, for rocprofv3 runs of
the general pipeline's kernels.  usage: python scripts/c2_prof.py [op 0-3] [iterations] [pairs]"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import roaringbitmap_amd as rb  # noqa: E402

op = int(sys.argv[1]) if len(sys.argv) > 1 else 0
n = int(sys.argv[2]) if len(sys.argv) > 2 else 5
pairs = int(sys.argv[3]) if len(sys.argv) > 3 else 1_000_000
ctx = rb.Context(0)
a, b = ctx.generate(rb.WL_FILTER_POSTING, pairs, seed=42)
for _ in range(n):
    ctx.pairwise(op, a, b).close()
ctx.synchronize()
print("done", op, n, pairs)

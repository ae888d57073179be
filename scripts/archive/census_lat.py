"""Small-batch latency study (config 1 shape): per-call wall time of one pairwise op over the 199
census1881 pairs, with the stats read-back, for latency work on the launch / sync sequence.
usage: python scripts/census_lat.py [--calls N]"""
import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
import roaringbitmap_amd as rb  # noqa: E402
from datasets import load_realdata  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--calls", type=int, default=400)
    ap.add_argument("--npairs", type=int, default=0, help="first N pairs only (0: all 199)")
    args = ap.parse_args()
    ctx = rb.Context(0)
    vals = load_realdata("census1881")
    s = ctx.upload_values(vals)
    n = args.npairs or len(vals) - 1
    ai = np.arange(n, dtype=np.uint32)
    bi = ai + 1
    res = {}
    for name, op in (("AND", rb.AND), ("OR", rb.OR), ("XOR", rb.XOR), ("ANDNOT", rb.ANDNOT)):
        for _ in range(20):
            ctx.pairwise(op, s, s, ai, bi).close()
        t = []
        for _ in range(args.calls):
            t0 = time.perf_counter()
            r = ctx.pairwise(op, s, s, ai, bi)
            t.append(time.perf_counter() - t0)
            r.close()
        st = ctx.stats()
        res[name] = {"median_us": round(1e6 * float(np.median(t)), 1), "min_us": round(1e6 * min(t), 1),
                     "gpu_total_us": round(1e3 * st["total_ms"], 1),
                     "kernels_us": {k["name"]: round(1e3 * k["ms"], 1) for k in st["kernels"]}}
    print(json.dumps(res))


if __name__ == "__main__":
    main()

"""Host-side cost of one config-2 pairwise call, split the way bench.py's step loop spends it:
the rbgpu_pairwise call itself (its wall time against the device span between its first and last
event, stats total_ms), rbgpu_get_stats, and the result's rbgpu_set_free.  Run on the GPU box:
    python scripts/host_overhead.py [--pairs N] [--steps K]"""
import argparse
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import roaringbitmap_amd as rb  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--pairs", type=int, default=1_000_000)
    ap.add_argument("--steps", type=int, default=20)
    args = ap.parse_args()
    with rb.Context(0) as ctx:
        a, b = ctx.generate(rb.WL_FILTER_POSTING, args.pairs, seed=42)  # bench.py's config-2 sets
        for _ in range(3):
            ctx.pairwise(rb.AND, a, b).close()
        ctx.synchronize()
        call, dev, stats, free, step = [], [], [], [], []
        for _ in range(args.steps):
            t0 = time.perf_counter()
            r = ctx.pairwise(rb.AND, a, b, npairs=args.pairs)
            t1 = time.perf_counter()
            s = ctx.stats_raw()
            t2 = time.perf_counter()
            r.close()
            t3 = time.perf_counter()
            call.append(t1 - t0)
            stats.append(t2 - t1)
            free.append(t3 - t2)
            step.append(t3 - t0)
            dev.append(s.total_ms * 1e-3)
        us = lambda v: round(1e6 * float(np.median(v)), 1)  # noqa: E731
        print({"call_us": us(call), "device_span_us": us(dev), "call_minus_device_us": us(np.subtract(call, dev)),
               "get_stats_us": us(stats), "set_free_us": us(free), "step_us": us(step)})


if __name__ == "__main__":
    main()

"""Light/heavy task-kernel study on config 2: materialising AND vs cardinality-only AND (same
staging and filter, no result stores) — separates the cost of the output path.
usage: python scripts/light_study.py [--pairs N] [--reps R]"""
import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import roaringbitmap_amd as rb  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--pairs", type=int, default=1_000_000)
    ap.add_argument("--reps", type=int, default=5)
    args = ap.parse_args()
    ctx = rb.Context(0)
    a, b = ctx.generate(rb.WL_FILTER_POSTING, args.pairs, seed=42)
    out = {}
    for name in ("materialise", "card_only"):
        ks = []
        for _ in range(args.reps + 2):
            if name == "materialise":
                ctx.pairwise(rb.AND, a, b).close()
            else:
                ctx.pairwise_cardinality(rb.AND, a, b)
            ks.append({k["name"]: k["ms"] for k in ctx.stats()["kernels"]})
        ks = ks[2:]
        out[name] = {k: round(sorted(x[k] for x in ks)[len(ks) // 2], 4) for k in ks[0]}
    print(json.dumps(out))


if __name__ == "__main__":
    main()

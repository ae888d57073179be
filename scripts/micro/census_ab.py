"""Census1881 small-batch calls, interleaved across library builds (A/B of k_pair_small variants): per lib and round,
the four ops' sweep time through Python (bench.py run_census's measure) and the C calls' median wall time, with the
golden cardinality sums checked.  Each library runs in its own process (RBGPU_LIB), rounds alternate.
usage: python scripts/micro/census_ab.py <rounds> lib1 lib2 ...   (lib "base" = the in-tree product)"""
import json
import os
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))

CHILD = r"""
import json, os, sys, time
import numpy as np
sys.path.insert(0, %r)
import bench
import roaringbitmap_amd as rb
vals = bench.load_census()
ops = {k: getattr(rb, k) for k in ("AND", "OR", "XOR", "ANDNOT")}
out = {}
with rb.Context(0) as ctx:
    s = ctx.upload_values(vals)
    ai = np.arange(len(vals) - 1, dtype=np.uint32); bi = ai + 1
    cards = {k: int(ctx.pairwise(op, s, s, ai, bi).cardinalities().sum()) for k, op in ops.items()}
    out["golden_ok"] = cards == bench.CENSUS_EXPECTED
    for k, op in ops.items():
        us = []
        for _ in range(40):
            r = ctx.pairwise(op, s, s, ai, bi)
            us.append(ctx.stats()["call_us"])
            r.close()
        out[k] = float(np.median(us[5:]))
    for _ in range(5):
        for op in ops.values():
            ctx.pairwise(op, s, s, ai, bi).close()
    ctx.synchronize()
    t0 = time.perf_counter()
    for _ in range(100):
        for op in ops.values():
            ctx.pairwise(op, s, s, ai, bi).close()
    ctx.synchronize()
    out["sweep_us"] = (time.perf_counter() - t0) / 400 * 1e6
print(json.dumps(out))
""" % ROOT


def main():
    rounds, libs = int(sys.argv[1]), sys.argv[2:]
    for r in range(rounds):
        for lib in libs:
            env = dict(os.environ)
            if lib == "base":
                env.pop("RBGPU_LIB", None)
            else:
                env["RBGPU_LIB"] = os.path.join(ROOT, "abvar", lib, "librbgpu.so")
            p = subprocess.run([sys.executable, "-c", CHILD], env=env, capture_output=True, text=True, timeout=300)
            if p.returncode != 0:
                print(f"FAIL {lib} r{r}: {p.stderr[-800:]}", flush=True)
                sys.exit(1)
            d = json.loads(p.stdout.strip().splitlines()[-1])
            print(f"{lib:12s} r{r} sweep {d['sweep_us']:6.1f} us | C calls AND {d['AND']:5.1f} OR {d['OR']:5.1f} "
                  f"XOR {d['XOR']:5.1f} ANDNOT {d['ANDNOT']:5.1f} | golden {d['golden_ok']}", flush=True)


if __name__ == "__main__":
    main()

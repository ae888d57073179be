"""Debug: FastAggregation.xor over the config-4 generator (4096 members) for a few keys, device vs oracle,
printing per-key container metadata on mismatch (with and without the fast-forward)."""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import roaringbitmap_amd as rb  # noqa: E402
from oracle import rbref as R  # noqa: E402

nb = int(sys.argv[1]) if len(sys.argv) > 1 else 4096
lo, hi = 0, 8
with rb.Context(0) as ctx:
    small = ctx.generate_keys(rb.WL_WIDE_RUNS, nb, lo, hi, seed=42)
    refs = [R.RefBitmap.deserialize(b) for b in small.serialize()]
    want = R.wide(R.FAST_XOR, refs)
    wc = want.containers()
    for ff in ("0", "1"):
        os.environ["RBGPU_XOR_NO_FASTFWD"] = ff
        got = ctx.wide(rb.FAST_XOR, small)
        h = got.download()
        gc = list(zip(h.key.tolist(), h.type.tolist(), h.card.tolist(), h.nruns.tolist()))
        ok = got.serialize()[0] == want.serialize()
        print("no_fastfwd" if ff == "1" else "fastfwd", "OK" if ok else "MISMATCH")
        if not ok:
            for a, b in zip(gc, wc):
                print("  dev", a, "ref", b, "" if tuple(a) == tuple(b) else "<--")

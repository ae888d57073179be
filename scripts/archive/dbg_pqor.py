"""Debug: priorityqueue_or device vs oracle per key (synthetic seed 6 members [32, 31])."""
import os, sys
import numpy as np
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT); sys.path.insert(0, os.path.join(ROOT, "tests"))
import roaringbitmap_amd as rb
from oracle import rbref as R
from datasets import synthetic_bitmaps
bms = synthetic_bitmaps(60, seed=6, max_keys=6, key_space=6)
rng = np.random.default_rng(6)
ctx = rb.Context(0)
for ro in (False, True):
    s = ctx.upload_values(bms, run_optimize=ro)
    refs = [R.RefBitmap.deserialize(b) for b in s.serialize()]
    for n in (1, 2, 3, 5, 11, 15, 16, 17, 40):
        members = rng.integers(0, len(bms), size=n).astype(np.uint32)
        got = ctx.wide(rb.PQ_OR, s, members)
        want = R.wide(R.PQ_OR, [refs[m] for m in members])
        if got.serialize()[0] != want.serialize():
            h = got.download()
            print("ro", ro, "members", list(members))
            print(" device:", [(int(h.key[i]), int(h.type[i]), int(h.card[i]), int(h.nruns[i])) for i in range(h.n_containers)])
            print(" oracle:", [(k, c.type_name() if hasattr(c, 'type_name') else None) for k, c in []])
            wb = want.serialize()
            w = ctx.upload_serialized([wb]) if hasattr(ctx, "upload_serialized") else None
            if w is not None:
                hw = w.download()
                print(" oracle:", [(int(hw.key[i]), int(hw.type[i]), int(hw.card[i]), int(hw.nruns[i])) for i in range(hw.n_containers)])
            hs = s.download()
            for m in members:
                b0, b1 = int(hs.begin[m]), int(hs.begin[m + 1])
                print(" member", int(m), [(int(hs.key[i]), int(hs.type[i]), int(hs.card[i]), int(hs.nruns[i])) for i in range(b0, b1)],
                      "size", s.summaries()[m]["size_in_bytes"] if "size_in_bytes" in s.summaries()[m] else None)
            sys.exit(0)
print("all equal")

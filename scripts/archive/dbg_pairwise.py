import sys, numpy as np
sys.path.insert(0, '.'); sys.path.insert(0, 'tests')
import roaringbitmap_amd as rb
from oracle import rbref as R
from datasets import synthetic_bitmaps
ctx = rb.Context(0)
names = {0:'A',1:'B',2:'R'}
for opname, op in (('AND',0),('OR',1),('XOR',2),('ANDNOT',3)):
  for ro in (False, True):
    bms = synthetic_bitmaps(80, seed=1)
    s = ctx.upload_values(bms, run_optimize=ro)
    h = s.download()
    refs = [R.RefBitmap.deserialize(b) for b in s.serialize()]
    rng = np.random.default_rng(101)
    a_idx = rng.integers(0, len(bms), size=300).astype(np.uint32)
    b_idx = rng.integers(0, len(bms), size=300).astype(np.uint32)
    out = ctx.pairwise(op, s, s, a_idx, b_idx)
    ho = out.download()
    bad = 0
    for i in range(len(a_idx)):
        ref = R.op(op, refs[a_idx[i]], refs[b_idx[i]])
        rc = ref.containers()
        lo, hi = int(ho.begin[i]), int(ho.begin[i+1])
        gc = list(zip(ho.key[lo:hi].tolist(), ho.type[lo:hi].tolist(), ho.card[lo:hi].tolist(), ho.nruns[lo:hi].tolist()))
        gv = ho.values(i); rv = ref.to_array()
        if gc != rc or not np.array_equal(gv, rv):
            bad += 1
            if bad <= 3:
                ia, ib = int(a_idx[i]), int(b_idx[i])
                ca = [(int(h.key[j]), names[int(h.type[j])], int(h.card[j]), int(h.nruns[j])) for j in range(int(h.begin[ia]), int(h.begin[ia+1]))]
                cb = [(int(h.key[j]), names[int(h.type[j])], int(h.card[j]), int(h.nruns[j])) for j in range(int(h.begin[ib]), int(h.begin[ib+1]))]
                print(f"{opname} ro={ro} pair {i}: A={ca}\n   B={cb}\n   got={gc}\n   ref={rc}")
                # per container value diff
                for (k,t,c,r) in rc:
                    gvk = gv[(gv>>16)==k] & 0xFFFF; rvk = rv[(rv>>16)==k] & 0xFFFF
                    if not np.array_equal(gvk, rvk):
                        d1 = np.setdiff1d(rvk, gvk); d2 = np.setdiff1d(gvk, rvk)
                        print(f"   key {k}: missing {len(d1)} e.g. {d1[:10]}, extra {len(d2)} e.g. {d2[:10]}")
    print(opname, ro, 'bad', bad, flush=True)

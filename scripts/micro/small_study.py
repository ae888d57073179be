"""Study build (RBG_SMALL_STUDY=1): per-block phase times of k_pair_small (s_memrealtime) on census1881's 199 pairs,
one op, copied out of the device by rbgpu_internal_small_study (only that build exports it).
usage: RBGPU_LIB=abvar/sstudy/librbgpu.so python scripts/micro/small_study.py OR"""
import ctypes as C
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import bench  # noqa: E402
import roaringbitmap_amd as rb  # noqa: E402
from roaringbitmap_amd import _lib as L  # noqa: E402

W = 32
op = getattr(rb, sys.argv[1] if len(sys.argv) > 1 else "OR")
vals = bench.load_census()
with rb.Context(0) as ctx:
    s = ctx.upload_values(vals)
    ai = np.arange(len(vals) - 1, dtype=np.uint32)
    bi = ai + 1
    for i in range(5):
        ctx.pairwise(op, s, s, ai, bi).close()
        ctx.synchronize()
    buf = np.zeros(8192 * W, np.uint64)
    f = L.lib().rbgpu_internal_small_study
    f.argtypes = [C.c_void_p, C.c_uint64]
    assert f(buf.ctypes.data, buf.size) == 0
    st = ctx.stats()
b = buf.reshape(-1, W)
cp = b[8191, :5].astype(np.int64).copy()
b = b[:8191]
b = b[b[:, 0] > 0]
t0 = int(b[:, 0].min())
last = b[b[:, 15] == 1]
print(f"op {sys.argv[1] if len(sys.argv) > 1 else 'OR'}: {len(b)} blocks, call device span {st['total_ms'] * 1e3:.1f} us "
      f"(s_memrealtime ticks: 10 ns at 100 MHz)")
rel = lambda x: (x.astype(np.int64) - t0) / 100.0  # us
start = rel(b[:, 0]); align = (b[:, 1].astype(np.int64) - b[:, 0].astype(np.int64)) / 100.0
wend = (b[:, 2:6].astype(np.int64) - b[:, [0]].astype(np.int64)) / 100.0
done = (b[:, 10].astype(np.int64) - b[:, 0].astype(np.int64)) / 100.0
q = lambda v: f"median {np.median(v):6.2f} p90 {np.percentile(v, 90):6.2f} max {np.max(v):6.2f}"
print("block start after the first block (us):", q(start))
print("alignment + work order (us)           :", q(align))
print("slowest wave of the block done (us)   :", q(wend.max(1)))
print("block done, counters added (us)       :", q(done))
print("block end, absolute (us)              :", q(start + done))
print("keys per wave (max in block)           :", q(b[:, 6:10].max(1)))
if len(last):
    l0 = last[0]
    print(f"last block: starts {rel(np.array([l0[0]]))[0]:.2f}, its keys done {(int(l0[10]) - int(l0[0])) / 100:.2f}, "
          f"compaction {(int(l0[11]) - int(l0[10])) / 100:.2f} us -> ends {rel(np.array([l0[11]]))[0]:.2f} us")
order = np.argsort(-(start + done))[:6]
for i in order:
    print(f"  slow block pair {int(b[i, 12])} sub {int(b[i, 13]) & 0xFFFFFFFF}/{int(b[i, 13]) >> 32} nu {int(b[i, 14])}: "
          f"start {start[i]:.2f} align {align[i]:.2f} waves {np.round(wend[i], 2).tolist()} keys {b[i, 6:10].tolist()} "
          f"done {done[i]:.2f}")
print("compaction phases (us): metas loaded + scanned + written %.2f, rbegin %.2f, pcard %.2f, counters + host words + "
      "release %.2f" % tuple((cp[1:] - cp[:-1]) / 100.0))

# the slowest single keys of the call: operands (type, card, runs) -> result (type, card, runs)
TN = {0: "A", 1: "B", 2: "R", 3: "-", 255: "empty"}
keys = []
for blk in b:
    for w in range(4):
        d, d1, d2, d3 = int(blk[16 + 4 * w]), int(blk[17 + 4 * w]), int(blk[18 + 4 * w]), int(blk[19 + 4 * w])
        if d:
            keys.append((d / 100.0, d1, d2, d3, int(blk[31 - w])))
keys.sort(reverse=True)
print("slowest keys (us): operands A | B -> result")
for d, d1, d2, d3, d4 in keys[:12]:
    ta, tb, ty, nr, c = d1 & 3, (d1 >> 2) & 3, (d1 >> 8) & 0xFF, (d1 >> 16) & 0xFFFF, d1 >> 32
    ca, cb, ra, rb = d2 & 0xFFFFF, (d2 >> 20) & 0xFFFFF, (d2 >> 40) & 0xFFF, (d2 >> 52) & 0xFFF
    mp = [((d3 >> (10 * i)) & 0x3FF) / 100.0 for i in range(6)] if d3 else None
    ph = (f"  merge: start {mp[0]:.2f} load+stage+search {mp[1]:.2f} walk {mp[2]:.2f} scan+copy {mp[3]:.2f} "
          f"out {mp[4]:.2f} return {mp[5]:.2f} after {d4 / 100.0:.2f}") if mp else ""
    print(f"  {d:6.2f}  {TN[ta]}(c={ca},r={ra}) | {TN[tb]}(c={cb},r={rb}) -> {TN.get(ty, ty)}(c={c},r={nr}){ph}")
ds = np.array([k[0] for k in keys])
print("key durations (us):", q(ds))

"""Pairwise OR with a large Bitmap operand on the general pipeline (round 6): such a pair's result type is
known before the OR — a Bitmap, or the full Run (BitmapContainer.or, BitmapContainer.java:1073-1110;
RunContainer.or(Bitmap)), a Bitmap even when full for BitmapContainer.ior(ArrayContainer) (:749-766).  Every
ordered pair of a container zoo (large, near-full and full Bitmaps; Arrays that fill a gap; Runs of <= 2047
and of 32768 runs, the > 8 KiB staging path), static, in place and cardinality-only, byte-exact against the
oracle.  The default build keeps these pairs on the register path; RBG_OR_BITS=1 builds (a study: slower) send
them to the copy + filter kernel — the same bytes either way."""
import numpy as np
import pytest

from type_pins import ARRAY, BITMAP, RUN, one_container_soa, oracle_bitmap, r, u

pytestmark = pytest.mark.gpu


@pytest.fixture
def general(monkeypatch):
    monkeypatch.setenv("RBGPU_NO_SMALL_PAIRS", "1")


def _zoo():
    rng = np.random.default_rng(61)
    gap = r(1000, 1700)
    near_full = np.setdiff1d(r(0, 65536), gap).astype(np.uint32)
    return [
        (BITMAP, np.sort(rng.choice(65536, 30000, replace=False)).astype(np.uint32)),
        (BITMAP, near_full),
        (BITMAP, r(0, 65536)),                       # a full Bitmap (non-canonical: the canonical form is a Run)
        (ARRAY, gap),                                # fills near_full
        (ARRAY, np.sort(rng.choice(65536, 2500, replace=False)).astype(np.uint32)),
        (RUN, u(r(900, 1800), r(40000, 41000))),     # covers the gap too
        (RUN, r(0, 65536, 2)),                       # 32768 runs: staged from global memory
        (RUN, u(*[r(k, k + 17) for k in range(5, 65000, 40)])),
        (BITMAP, np.setdiff1d(r(0, 65536), r(0, 65536, 2)).astype(np.uint32)),  # the odd values: + the Run = full
    ]


def _pairs(n):
    a = np.repeat(np.arange(n), n).astype(np.uint32)
    b = np.tile(np.arange(n), n).astype(np.uint32)
    keep = a != b
    return a[keep], b[keep]


def test_or_with_large_bitmap_static_inplace_cardinality(ctx, oracle, general):
    import roaringbitmap_amd as rb
    conts = _zoo()
    s = ctx.upload_soa(one_container_soa(conts))
    refs = [oracle_bitmap(oracle, t, v) for t, v in conts]
    ai, bi = _pairs(len(conts))
    # the general pipeline takes batches above the small-batch limit: repeat the pairs
    rep = 50
    ai_r, bi_r = np.tile(ai, rep), np.tile(bi, rep)
    got = ctx.pairwise(rb.OR, s, s, ai_r, bi_r).serialize()
    got_i = ctx.pairwise_inplace(rb.OR, s, s, ai_r, bi_r).serialize()
    cards = ctx.pairwise_cardinality(rb.OR, s, s, ai_r, bi_r)
    table = {}
    for x, y in zip(ai.tolist(), bi.tolist()):
        want = oracle.op(rb.OR, refs[x], refs[y])
        ref_i = refs[x].clone()
        oracle.op_inplace(rb.OR, ref_i, refs[y])
        table[(x, y)] = (want.serialize(), ref_i.serialize(), want.cardinality())
    for k in range(len(ai_r)):
        x, y = int(ai_r[k]), int(bi_r[k])
        want_s, want_i, want_c = table[(x, y)]
        assert got[k] == want_s, (k, x, y)
        assert got_i[k] == want_i, ("inplace", k, x, y)
        assert int(cards[k]) == want_c, ("card", k, x, y)


def test_or_full_results_types(ctx, oracle, general):
    """The full unions: a Run [0, 65535] from the static or(), a Bitmap from Bitmap.ior(Array) only."""
    import roaringbitmap_amd as rb
    conts = _zoo()
    s = ctx.upload_soa(one_container_soa(conts))
    pairs = [(1, 3), (3, 1), (1, 5), (5, 1), (8, 6), (6, 8), (2, 4), (4, 2)]
    ai = np.array([p[0] for p in pairs] * 600, np.uint32)
    bi = np.array([p[1] for p in pairs] * 600, np.uint32)
    hs = ctx.pairwise(rb.OR, s, s, ai, bi).download()
    hi = ctx.pairwise_inplace(rb.OR, s, s, ai, bi).download()
    for k, (x, y) in enumerate(pairs):
        assert int(hs.card[k]) == 65536 and int(hs.type[k]) == RUN and int(hs.nruns[k]) == 1, (x, y)
        keeps = conts[x][0] == BITMAP and conts[y][0] == ARRAY
        assert int(hi.type[k]) == (BITMAP if keeps else RUN), ("inplace", x, y)

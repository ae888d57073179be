"""Parity of the fused MI355X BSI compare (rbgpu_bsi_compare) with the oracle's restatement of
Roaring64BitmapSliceIndex.compare: identical RoaringFormatSpec bytes for every operation, with and
without foundSet, over dense / sparse / run-optimized slices, plus the reference's own known answers."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu
OPS = ["EQ", "NEQ", "LE", "LT", "GE", "GT", "RANGE"]


def _device_bsi(ctx, oracle, slices, ebm, run_optimize):
    vals = [s.to_array() for s in slices] + [ebm.to_array()]
    d = ctx.upload_values(vals, run_optimize=run_optimize)
    refs = [oracle.RefBitmap.deserialize(b) for b in d.serialize()]  # the exact containers uploaded
    return d, refs[:-1], refs[-1]


def _case(rng, n, nbits, universe):
    cols = np.unique(rng.integers(0, universe, size=n))
    vals = rng.integers(0, 2**nbits, size=len(cols), dtype=np.uint64) if nbits < 64 else \
        rng.integers(0, 2**63, size=len(cols), dtype=np.uint64)
    return cols, vals


@pytest.mark.parametrize("seed", [1, 2, 3])
def test_bsi_all_ops_bytes(ctx, oracle, seed):
    import roaringbitmap_amd as rb
    rng = np.random.default_rng(seed)
    shapes = [(3000, 10, 1 << 18), (200000, 20, 1 << 18), (50000, 40, 1 << 22), (500, 63, 1 << 17)]
    for n, nbits, uni in shapes:
        cols, vals = _case(rng, n, nbits, uni)
        sl, ebm, mn, mx = oracle.bsi_build(cols, vals)
        for ro in (False, True):
            d, rsl, rebm = _device_bsi(ctx, oracle, sl, ebm, ro)
            fcols = np.unique(rng.choice(cols, size=max(1, len(cols) // 3)))
            fcols = np.concatenate([fcols, rng.integers(0, uni, size=50)]).astype(np.uint32)  # some not in ebM
            found_ref = oracle.RefBitmap.of(np.unique(fcols))
            found = ctx.upload_serialized([found_ref.serialize()])
            preds = [int(v) for v in rng.choice(vals, size=3)] + [0, int(mn), int(mx), int(mx) + 1]
            for name in OPS:
                op = getattr(rb, "BSI_" + name)
                for p in preds:
                    end = p + int(rng.integers(0, max(1, int(mx) - p + 2)))
                    for f_dev, f_ref in ((None, None), (found, found_ref)):
                        got = ctx.bsi_compare(op, d, p, end, int(mn), int(mx), f_dev).serialize()[0]
                        want = oracle.bsi_compare(rsl, rebm, op, p, end, f_ref, int(mn), int(mx)).serialize()
                        assert got == want, (name, n, nbits, ro, p, end, f_dev is not None)
            # the index's key tables were built once and reused by every compare above (a foundSet's row
            # rebuilt per call in their scratch row)
            assert d.setup_parts()["bsi_tables"]["bytes"] > 0


def test_bsi_reference_known_answers(ctx, oracle):
    """R64BSITest.java testGT / testGE / testLT / testLE / testRANGE / testNEQ / testValueZero
    through the Python mirror of the reference API."""
    import roaringbitmap_amd as rb
    bsi = rb.Roaring64BitmapSliceIndex(1, 99)
    for x in range(1, 100):
        bsi.setValue(x, x)
    q = lambda op, a, b=0, f=None: list(bsi.compare(op, a, b, f).toArray())  # noqa: E731
    O = rb.Operation
    assert q(O.GT, 50) == list(range(51, 100)) and q(O.GT, 99) == []
    assert q(O.GE, 50) == list(range(50, 100)) and q(O.GE, 100) == []
    assert q(O.LT, 50) == list(range(1, 50)) and q(O.LT, 1) == []
    assert q(O.LE, 50) == list(range(1, 51)) and q(O.LE, 0) == []
    assert q(O.RANGE, 10, 20) == list(range(10, 21)) and q(O.RANGE, 1000, 2000) == []
    assert q(O.GE, 50, 0, rb.RoaringBitmap.bitmapOf([51, 52, 53])) == [51, 52, 53]
    z = rb.Roaring64BitmapSliceIndex()
    for c, v in ((0, 0), (1, 0), (2, 1)):
        z.setValue(c, v)
    assert list(z.compare(O.EQ, 0).toArray()) == [0, 1] and list(z.compare(O.EQ, 1).toArray()) == [2]
    n = rb.Roaring64BitmapSliceIndex()
    for c, v in ((1, 99), (2, 1), (3, 50)):
        n.setValue(c, v)
    assert list(n.compare(O.NEQ, 99).toArray()) == [2, 3]


def test_generated_bsi_sample(ctx, oracle):
    """The config-5 generator's shape (random value bits, full ebM, runOptimize'd), reduced."""
    import roaringbitmap_amd as rb
    d = ctx.generate_bsi(24, 3 * 65536 + 1234, seed=4)
    refs = [oracle.RefBitmap.deserialize(b) for b in d.serialize()]
    sl, ebm = refs[:-1], refs[-1]
    lo, hi = 3 << 20, 11 << 20
    for name in OPS:
        op = getattr(rb, "BSI_" + name)
        got = ctx.bsi_compare(op, d, lo, hi, 0, (1 << 24) - 1).serialize()[0]
        want = oracle.bsi_compare(sl, ebm, op, lo, hi, None, 0, (1 << 24) - 1).serialize()
        assert got == want, name


def test_bsi_key_range_shards(ctx, oracle):
    """rbgpu_bsi_compare_keys / rbgpu_generate_bsi_keys: the key-range shards of the
    answer, computed from the whole index and from per-shard generated indexes, reassemble
    (serialize_parts) to the whole answer's bytes — O'Neil path and min/max shortcut, with foundSet."""
    import roaringbitmap_amd as rb
    from roaringbitmap_amd.sharding import serialize_parts
    nrows, nbits = 5 * 65536 + 77, 20
    d = ctx.generate_bsi(nbits, nrows, seed=9)
    fvals = np.arange(0, nrows, 3, dtype=np.uint32)
    found = ctx.upload_values([fvals])
    parts = [(0, 2), (2, 3), (3, 65536)]
    shards = [ctx.generate_bsi(nbits, nrows, seed=9, key_range=kr) for kr in parts]
    whole = d.download()
    for s, (klo, khi) in zip(shards, parts):  # a generated shard holds exactly the index's containers
        h = s.download()
        for b in range(nbits + 1):
            sel = [i for i in range(int(whole.begin[b]), int(whole.begin[b + 1])) if klo <= whole.key[i] < khi]
            assert list(h.key[int(h.begin[b]):int(h.begin[b + 1])]) == [int(whole.key[i]) for i in sel]
            for j, i in zip(range(int(h.begin[b]), int(h.begin[b + 1])), sel):
                assert bytes(h.container_payload(j)) == bytes(whole.container_payload(i))
    vmax = (1 << nbits) - 1
    for name, lo, hi in (("RANGE", 1 << 17, 5 << 17), ("GE", 4321, 0), ("NEQ", 7, 0), ("LE", vmax, 0),
                         ("GT", 1 << 30, 0)):  # LE vmax / GT above max: the min/max shortcut
        op = getattr(rb, "BSI_" + name)
        for f in (None, found):
            want = ctx.bsi_compare(op, d, lo, hi, 0, vmax, f).serialize()[0]
            for src in ("whole", "shards"):
                hs = []
                for i, kr in enumerate(parts):
                    r = ctx.bsi_compare(op, d if src == "whole" else shards[i], lo, hi, 0, vmax, f, key_range=kr)
                    assert len(r) == 1
                    hs.append(r.download())
                assert serialize_parts(hs) == want, (name, src, f is not None)
    with pytest.raises(rb.InvalidArgument):
        ctx.bsi_compare(rb.BSI_GE, d, 3, 0, 0, vmax, key_range=(5, 70000))


def test_bsi_range_one_launch_handoff(ctx, oracle):
    """RANGE runs as one launch whose last block hands the result count and counters to host-visible
    words, behind a per-context sequence number that the small-batch pairwise path shares: empty and
    one-key answers, and RANGE calls interleaved with small pairwise calls on the same context, all equal
    the oracle; the call's device times are read when the stats are asked for."""
    import roaringbitmap_amd as rb
    rng = np.random.default_rng(5)
    cols, vals = _case(rng, 70000, 12, 1 << 20)
    sl, ebm, mn, mx = oracle.bsi_build(cols, vals)
    d, rsl, rebm = _device_bsi(ctx, oracle, sl, ebm, False)
    one_key = oracle.RefBitmap.of(np.unique(cols[cols < 65536]).astype(np.uint32))
    found1 = ctx.upload_serialized([one_key.serialize()])
    absent = int(max(set(range(int(mn), int(mx) + 1)) - set(int(v) for v in vals), default=int(mn)))
    pair_bms = [np.unique(rng.integers(0, 1 << 18, size=n)).astype(np.uint32) for n in (100, 3000, 20000, 5)]
    p = ctx.upload_values(pair_bms)
    prefs = [oracle.RefBitmap.deserialize(b) for b in p.serialize()]
    cases = [(absent, absent, None, None), (int(mn), int(mx), None, None), (int(vals[0]), int(vals[0]), found1, one_key),
             (absent, absent, found1, one_key)]
    for it in range(6):
        lo, hi, f_dev, f_ref = cases[it % len(cases)]
        r = ctx.bsi_compare(rb.BSI_RANGE, d, lo, hi, int(mn), int(mx), f_dev)
        st = ctx.stats()
        want = oracle.bsi_compare(rsl, rebm, rb.BSI_RANGE, lo, hi, f_ref, int(mn), int(mx))
        assert r.serialize()[0] == want.serialize(), (it, lo, hi)
        assert st["result_cardinality"] == want.cardinality()  # the shortcut's answer too
        assert st["result_containers"] == r.n_containers
        if (lo, hi) != (int(mn), int(mx)):  # (the whole value range is compareUsingMinMax's shortcut: no kernel)
            assert st["total_ms"] > 0.0 and st["main_kernel_ms"] > 0.0
        else:
            assert st["tasks"] == 0
        r.wait()  # the one-launch kernel's end (rbgpu_set_wait), then its SoA through the device view
        v = r.device_view()
        assert v["n_containers"] == r.n_containers and v["n_bitmaps"] == 1
        for op in (rb.AND, rb.OR):  # small batches on the same context between the compares
            got = ctx.pairwise(op, p, p, [0, 1, 2], [1, 2, 3]).serialize()
            assert got == [oracle.op(op, prefs[i], prefs[i + 1]).serialize() for i in range(3)]
            assert ctx.stats()["total_ms"] > 0.0

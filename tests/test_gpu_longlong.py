"""The 64-bit front end on the device (rbgpu_set64 / rbgpu_pairwise64): Roaring64NavigableMap and
Roaring64Bitmap set algebra byte-exact against the oracle's restatement (oracle/rbref64.py), the
reference's 64-bit portable fixtures, and the Python mirror classes."""
import numpy as np
import pytest

from test_oracle64 import FIXTURES64, read

pytestmark = pytest.mark.gpu
OPS = {"AND": 0, "OR": 1, "XOR": 2, "ANDNOT": 3}


def _values64(rng, n_highs=4, dense=False):
    highs = rng.choice([0, 1, 2, 7, 1 << 20, (1 << 32) - 2, (1 << 32) - 1], size=n_highs, replace=False)
    parts = []
    for h in highs:
        k = int(rng.integers(1, 4))
        for key in rng.choice(16, size=k, replace=False):
            base = (int(h) << 32) | (int(key) << 16)
            kind = int(rng.integers(0, 3))
            if kind == 0:
                lows = rng.choice(65536, size=int(rng.integers(1, 3000)), replace=False)
            elif kind == 1:
                lows = rng.choice(65536, size=int(rng.integers(5000, 40000)), replace=False)
            else:
                s = int(rng.integers(0, 60000))
                lows = np.arange(s, s + int(rng.integers(1, 5000))) % 65536
            parts.append(np.uint64(base) + np.asarray(lows, np.uint64))
    return np.unique(np.concatenate(parts))


@pytest.mark.parametrize("name,card,nb,sel", FIXTURES64, ids=[f[0] for f in FIXTURES64])
def test_portable_fixtures_on_device(ctx, name, card, nb, sel):
    data = read(name)
    s = ctx.upload_portable64([data])
    assert s.serialize_portable() == [data]
    assert int(s.cardinalities()[0]) == card and len(s.highs(0)) == nb


def _pool(ctx, oracle, seed, n=12):
    from oracle import rbref64 as R64
    rng = np.random.default_rng(seed)
    vals = [_values64(rng, n_highs=int(rng.integers(1, 5))) for _ in range(n)]
    refs = [R64.Ref64.of(v) for v in vals]
    for r in refs[::3]:  # some buckets runOptimize'd (Run containers in the mix)
        for _, b in r.buckets:
            b.run_optimize()
    s = ctx.upload_portable64([r.to_portable() for r in refs])
    return s, refs


@pytest.mark.parametrize("seed", [1, 2, 3])
def test_roaring64_ops(ctx, oracle, seed):
    import roaringbitmap_amd as rb
    from oracle import rbref64 as R64
    s, refs = _pool(ctx, oracle, seed)
    n = len(refs)
    ai = np.array([i for i in range(n) for j in range(n)], np.uint32)
    bi = np.array([j for i in range(n) for j in range(n)], np.uint32)  # includes i == j
    for opname, op in OPS.items():
        got_s = ctx.pairwise64(rb.RB64_BITMAP, op, s, s, ai, bi).serialize_portable()
        got_i = ctx.pairwise64(rb.RB64_BITMAP, op, s, s, ai, bi, inplace=True).serialize_portable()
        got_n = ctx.pairwise64(rb.RB64_NAVIGABLE, op, s, s, ai, bi, inplace=True).serialize_portable()
        for k in range(len(ai)):
            i, j = int(ai[k]), int(bi[k])
            assert got_s[k] == R64.bitmap_op(op, refs[i], refs[j], False).to_portable(), ("static", opname, i, j)
            assert got_i[k] == R64.bitmap_op(op, refs[i], refs[j], True, same=i == j).to_portable(), \
                ("in place", opname, i, j)
            assert got_n[k] == R64.navigable_op(op, refs[i], refs[j], same=i == j).to_portable(), \
                ("navigable", opname, i, j)


def test_roaring64_empty_xor_containers_and_buckets(ctx, oracle):
    """Roaring64Bitmap.xor keeps an empty container under its key (card - 1 written as 0xFFFF in the
    bucket's RoaringFormatSpec bytes); Roaring64NavigableMap.xor leaves an empty bucket; both from equal
    containers, through the register path of the 32-bit engine (one shared Bitmap, one shared Run)."""
    import roaringbitmap_amd as rb
    from oracle import rbref64 as R64
    same = np.concatenate([np.arange(0, 30000, 3, dtype=np.uint64),                       # Bitmap at key 0
                           (1 << 16) + np.arange(100, 20000, dtype=np.uint64)])          # Run at key 1
    x = R64.Ref64.of(np.concatenate([same, (5 << 32) + np.arange(10, dtype=np.uint64)]))
    y = R64.Ref64.of(np.concatenate([same, (6 << 32) + np.arange(10, dtype=np.uint64)]))
    for r in (x, y):
        for _, b in r.buckets:
            b.run_optimize()
    s = ctx.upload_portable64([x.to_portable(), y.to_portable()])
    for inplace in (False, True):
        got = ctx.pairwise64(rb.RB64_BITMAP, rb.XOR, s, s, [0], [1], inplace=inplace).serialize_portable()[0]
        want = R64.bitmap_op(rb.XOR, x, y, inplace)
        assert got == want.to_portable()
        assert [c[2] for c in want.buckets[0][1].containers()] == [0, 0]
    got = ctx.pairwise64(rb.RB64_NAVIGABLE, rb.XOR, s, s, [0], [1], inplace=True)
    assert got.serialize_portable()[0] == R64.navigable_op(rb.XOR, x, y).to_portable()
    assert list(got.highs(0)) == [0, 5, 6]


def test_roaring64_large_batch_general_path(ctx, oracle):
    """More bucket pairs than the small-batch path takes: the general pipeline with RB_EMPTY_BITMAP pairs."""
    import roaringbitmap_amd as rb
    from oracle import rbref64 as R64
    s, refs = _pool(ctx, oracle, 9, n=40)
    rng = np.random.default_rng(4)
    ai = rng.integers(0, 40, 3000).astype(np.uint32)
    bi = rng.integers(0, 40, 3000).astype(np.uint32)
    for opname, op in OPS.items():
        got = ctx.pairwise64(rb.RB64_BITMAP, op, s, s, ai, bi).serialize_portable()
        for k in range(0, 3000, 37):
            assert got[k] == R64.bitmap_op(op, refs[ai[k]], refs[bi[k]], False).to_portable(), (opname, k)


def test_roaring64_python_mirror(ctx, oracle):
    import roaringbitmap_amd as rb
    from oracle import rbref64 as R64
    rng = np.random.default_rng(12)
    va, vb = _values64(rng), _values64(rng)
    for cls, flavor in ((rb.Roaring64NavigableMap, "nav"), (rb.Roaring64Bitmap, "art")):
        a, b = cls.bitmapOf(va), cls.bitmapOf(vb)
        ra, rb_ = R64.Ref64.of(va), R64.Ref64.of(vb)
        assert a.getLongCardinality() == len(va)
        assert np.array_equal(a.toArray(), va)
        assert a.serializePortable() == ra.to_portable()
        for opname, op in OPS.items():
            x = a.clone()
            getattr(x, {"AND": "and_", "OR": "or_", "XOR": "xor", "ANDNOT": "andNot"}[opname])(b)
            want = R64.navigable_op(op, ra, rb_) if flavor == "nav" else R64.bitmap_op(op, ra, rb_, True)
            assert x.serializePortable() == want.to_portable(), (flavor, opname)
    r = rb.Roaring64Bitmap.and_(rb.Roaring64Bitmap.bitmapOf(va), rb.Roaring64Bitmap.bitmapOf(vb))
    assert r.serializePortable() == R64.bitmap_op(rb.AND, R64.Ref64.of(va), R64.Ref64.of(vb), False).to_portable()
    fx = rb.Roaring64NavigableMap.deserializePortable(read("64mapspreadvals.bin"))
    assert fx.select(90) == (9 << 32) and fx.select(99) == (9 << 32) + 9
    with pytest.raises(rb.InvalidArgument):  # Roaring64NavigableMap has no static and/or/xor/andNot
        ctx.pairwise64(rb.RB64_NAVIGABLE, rb.AND, fx._set, fx._set, [0], [0])


def test_roaring64_kept_empty_container_through_later_ops(ctx, oracle):
    """A Roaring64Bitmap keeps the empty container an xor leaves (Roaring64Bitmap.java:392-460).  Later
    in-place and static ops treat it like any other container: an andNot / or / xor against a bitmap
    without that high (or without that key under it) leaves it untouched or clones it (:319-343, 599-628,
    630-650), a matched and / andNot drops it, a matched or fills it."""
    import roaringbitmap_amd as rb
    from oracle import rbref64 as R64
    same = np.concatenate([np.arange(0, 30000, 3, dtype=np.uint64),                       # Bitmap at key 0
                           (1 << 16) + np.arange(100, 200, dtype=np.uint64)])            # Array at key 1
    x = R64.Ref64.of(np.concatenate([same, (1 << 32) + np.arange(10, dtype=np.uint64)]))
    y = R64.Ref64.of(same)
    z_other_high = R64.Ref64.of((9 << 32) + np.arange(5, dtype=np.uint64))
    z_other_key = R64.Ref64.of((5 << 16) + np.arange(5, dtype=np.uint64))
    z_matched = R64.Ref64.of(np.arange(0, 90, 3, dtype=np.uint64))
    s = ctx.upload_portable64([r.to_portable() for r in (x, y, z_other_high, z_other_key, z_matched)])
    xy = ctx.pairwise64(rb.RB64_BITMAP, rb.XOR, s, s, [0], [1], inplace=True)
    ref_xy = R64.bitmap_op(rb.XOR, x, y, True)
    assert xy.serialize_portable()[0] == ref_xy.to_portable()
    assert [c[2] for c in ref_xy.buckets[0][1].containers()] == [0, 0]  # two kept empty containers
    # the device result itself is the left operand (its portable bytes, card - 1 = 0xFFFF, do not read
    # back — the reference's own reader would take 65536 values there too)
    refs = [ref_xy, z_other_high, z_other_key, z_matched]
    for opname, op in OPS.items():
        for j in (1, 2, 3):
            for inplace in (False, True):
                got = ctx.pairwise64(rb.RB64_BITMAP, op, xy, s, [0], [j + 1], inplace=inplace).serialize_portable()[0]
                want = R64.bitmap_op(op, refs[0], refs[j], inplace)
                assert got == want.to_portable(), (opname, j, inplace)


def test_roaring64_mirror_after_empty_xor(ctx, oracle):
    """isEmpty is getLongCardinality() == 0 (Roaring64NavigableMap.java:1148, Roaring64Bitmap.java:837);
    toArray / select / clone read the device buckets, so the empty containers a Roaring64Bitmap xor keeps
    (or the empty buckets a Roaring64NavigableMap and leaves) read back correctly."""
    import roaringbitmap_amd as rb
    from oracle import rbref64 as R64
    same = np.concatenate([np.arange(0, 30000, 3, dtype=np.uint64), (1 << 16) + np.arange(100, 200, dtype=np.uint64)])
    extra = (3 << 32) + np.arange(7, dtype=np.uint64)
    for cls in (rb.Roaring64Bitmap, rb.Roaring64NavigableMap):
        x, y = cls.bitmapOf(np.concatenate([same, extra])), cls.bitmapOf(same)
        x.xor(y)
        assert not x.isEmpty()
        assert np.array_equal(x.toArray(), extra)
        assert x.select(3) == int(extra[3])
        with pytest.raises(ValueError):
            x.select(7)
        c = x.clone()
        assert c.serializePortable() == x.serializePortable()
        assert np.array_equal(c.toArray(), extra)
        x.andNot(cls.bitmapOf(extra))
        assert x.isEmpty() and x.getLongCardinality() == 0 and len(x.toArray()) == 0
    nav = rb.Roaring64NavigableMap.bitmapOf([1])
    nav.and_(rb.Roaring64NavigableMap.bitmapOf([2]))  # the emptied bucket stays in the map
    assert nav.isEmpty() and len(nav._set.highs(0)) == 1
    ref = R64.navigable_op(rb.AND, R64.Ref64.of([1]), R64.Ref64.of([2]))
    assert nav.serializePortable() == ref.to_portable()


@pytest.mark.parametrize("seed", [1, 2])
def test_roaring64_legacy_format_and_cardinality(ctx, oracle, seed):
    """Roaring64NavigableMap's default (legacy) format on the device: ingest and emit round-trip the
    oracle's bytes, signed and unsigned (parity unpinned: no reference fixture, see test_oracle64); an
    in-place op keeps x1's signedLongs and the legacy bytes equal the oracle's.  The 64-bit cardinality
    entry (Roaring64Bitmap.andCardinality, longlong/Roaring64Bitmap.java:562-592, and the same merge for
    or / xor / andNot) equals the materialised static results' cardinalities."""
    import roaringbitmap_amd as rb
    from oracle import rbref64 as R64
    _, refs = _pool(ctx, oracle, seed, n=8)
    for i, r in enumerate(refs):
        r.signed = i % 2 == 1
    blobs = [r.to_legacy() for r in refs]
    s = ctx.upload_legacy64(blobs)
    assert s.serialize_legacy() == blobs
    assert s.serialize_portable() == [r.to_portable() for r in refs]
    n = len(refs)
    ai = np.array([i for i in range(n) for j in range(n)], np.uint32)
    bi = np.array([j for i in range(n) for j in range(n)], np.uint32)
    for opname, op in OPS.items():
        got = ctx.pairwise64(rb.RB64_NAVIGABLE, op, s, s, ai, bi, inplace=True).serialize_legacy()
        for k in range(len(ai)):
            i, j = int(ai[k]), int(bi[k])
            assert got[k] == R64.navigable_op(op, refs[i], refs[j], same=i == j).to_legacy(), (opname, i, j)
        cards = ctx.pairwise64_cardinality(op, s, s, ai, bi)
        mat = ctx.pairwise64(rb.RB64_BITMAP, op, s, s, ai, bi).cardinalities()
        assert np.array_equal(cards, mat), opname
        if op == rb.AND:
            for k in range(0, len(ai), 7):
                assert int(cards[k]) == R64.and_cardinality(refs[ai[k]], refs[bi[k]])
    with pytest.raises(rb.FormatError):
        ctx.upload_legacy64([blobs[0][:-1]])


def test_roaring64_legacy_hand_built_streams(ctx, oracle):
    """deserializeLegacy (Roaring64NavigableMap.java:1295-1324) reads the flag with readBoolean
    (any non-zero byte is true) and puts each (high, bitmap) into a TreeMap: highs in any stream order are
    ordered by the map and a repeated high keeps the bitmap read last.  A hand-built stream with flag byte 7,
    highs 9, 2, 9, 5 reads back as the oracle's map (signed, highs 2 / 5 / 9, the second bitmap of 9)."""
    import struct

    from oracle import rbref as R
    from oracle import rbref64 as R64
    parts = [(9, [1, 2, 3]), (2, [7]), (9, [100, 200]), (5, list(range(70000, 90000)))]
    blob = bytes([7]) + struct.pack(">i", len(parts)) + b"".join(
        struct.pack(">I", h) + R.RefBitmap.of(np.array(v, np.uint32)).serialize() for h, v in parts)
    want = R64.Ref64.from_legacy(blob)
    assert want.signed and [h for h, _ in want.buckets] == [2, 5, 9]
    s = ctx.upload_legacy64([blob])
    assert s.signed_longs(0)
    assert list(s.highs(0)) == [2, 5, 9]
    assert s.serialize_legacy() == [want.to_legacy()]
    assert s.serialize_portable() == [want.to_portable()]
    assert np.array_equal(s.values(0), want.to_array())


def test_roaring64_navigable_mirror_legacy(ctx, oracle):
    """TestRoaring64NavigableMap.testSerialization_MultipleBuckets_Signed / _Unsigned (:741-773) through
    the mirror: serialize() is the legacy format, deserialize() restores the map and its value order."""
    import roaringbitmap_amd as rb
    vals = np.array([(-123) & (2**64 - 1), 123, 2**63 - 1], np.uint64)
    for signed, order in ((True, [-123, 123, 2**63 - 1]), (False, [123, 2**63 - 1, -123])):
        m = rb.Roaring64NavigableMap(rb.Roaring64NavigableMap.bitmapOf(vals)._set, signedLongs=signed)
        clone = rb.Roaring64NavigableMap.deserialize(m.serialize())
        assert clone.getLongCardinality() == 3
        assert [int(np.int64(np.uint64(clone.select(j)))) for j in range(3)] == order
        assert len(m.serialize()) == 1 + 4 + 3 * 4 + sum(
            len(x) - 12 for x in [rb.Roaring64NavigableMap.bitmapOf([v]).serializePortable() for v in vals])
    a = rb.Roaring64Bitmap.bitmapOf(vals)
    b = rb.Roaring64Bitmap.bitmapOf(np.array([123, 5], np.uint64))
    assert rb.Roaring64Bitmap.andCardinality(a, b) == 1


def test_roaring64_art_format(ctx, oracle):
    """Roaring64Bitmap.serialize / deserialize (HighLowContainer: ART + Containers) on the device: ingest
    and emit equal the oracle's canonical bytes for sets covering every node type, a stream with another
    container placement (null slots, permuted indices) reads back to the same set, and the static ops'
    results emit the oracle's bytes — an xor's kept-empty containers included (parity unpinned: no
    reference fixture, see test_oracle64.test_oracle64_art_format)."""
    import roaringbitmap_amd as rb
    from oracle import rbref64 as R64
    from test_oracle64 import _art_sets
    sets = _art_sets()
    blobs = [r.to_art() for r in sets]
    s = ctx.upload_art64(blobs)
    assert s.serialize_art() == blobs
    assert s.serialize_portable() == [r.to_portable() for r in sets]
    other = []
    for r in sets:
        n = sum(len(b.containers()) for _, b in r.buckets)
        other.append(r.to_art(slots=list(np.random.default_rng(n).permutation(n + 2)[:n]), cap=n + 2) if n else b"\x00")
    assert ctx.upload_art64(other).serialize_art() == blobs
    p, refs = _pool(ctx, oracle, 5, n=6)
    n = len(refs)
    ai = np.array([i for i in range(n) for j in range(n)], np.uint32)
    bi = np.array([j for i in range(n) for j in range(n)], np.uint32)
    for opname, op in OPS.items():
        got = ctx.pairwise64(rb.RB64_BITMAP, op, p, p, ai, bi).serialize_art()
        for k in range(len(ai)):
            want = R64.bitmap_op(op, refs[int(ai[k])], refs[int(bi[k])], False).to_art()
            assert got[k] == want, (opname, int(ai[k]), int(bi[k]))
    x = rb.Roaring64Bitmap.bitmapOf(np.array([1, 2, (7 << 40) | 3], np.uint64))
    y = rb.Roaring64Bitmap.deserialize(x.serialize())
    assert np.array_equal(y.toArray(), x.toArray())
    with pytest.raises(rb.FormatError):
        ctx.upload_art64([blobs[2][:-1]])


@pytest.mark.parametrize("seed", [1, 2, 3, 5])
def test_roaring64_kept_empty_container_types(ctx, oracle, seed):
    """Every container of a static Roaring64Bitmap.xor(x_i, x_j) — the kept-empty ones included — has the
    oracle's key, type, cardinality and run count in the device's bucket view (rbgpu_set64_bucket_set ->
    download), i.e. the kernel's type choice, apart from any writer: an empty Run xor Run is a Run, an
    empty Array / Bitmap xor an Array (RunContainer.java:2445-2482, 2326-2335; ArrayContainer.java:
    1311-1336; BitmapContainer.java:1381-1422; Roaring64Bitmap.java:421-460 puts with no isEmpty check).
    Seed 5 is GPUTEST_r04's failing pool."""
    import roaringbitmap_amd as rb
    from oracle import rbref64 as R64
    p, refs = _pool(ctx, oracle, seed, n=6)
    n = len(refs)
    ai = np.array([i for i in range(n) for j in range(n)], np.uint32)
    bi = np.array([j for i in range(n) for j in range(n)], np.uint32)
    res = ctx.pairwise64(rb.RB64_BITMAP, rb.XOR, p, p, ai, bi)
    kept_empty = {0: 0, 2: 0}
    for k in range(len(ai)):
        want = R64.bitmap_op(rb.XOR, refs[int(ai[k])], refs[int(bi[k])], False)
        assert [int(h) for h in res.highs(k)] == [h for h, _ in want.buckets], k
        if not want.buckets:
            continue
        h = res.bucket_set(k).download()
        got = [(int(h.key[c]), int(h.type[c]), int(h.card[c]), int(h.nruns[c])) for c in range(len(h.key))]
        exp = [c for _, b in want.buckets for c in b.containers()]
        assert got == exp, (int(ai[k]), int(bi[k]))
        for c in exp:
            if c[2] == 0:
                kept_empty[c[1]] = kept_empty.get(c[1], 0) + 1
    if seed == 5:  # the pool holds both kinds of kept-empty containers
        assert kept_empty[0] > 0 and kept_empty[2] > 0, kept_empty


def test_roaring64_art_round_trip_kept_empty(ctx, oracle):
    """Roaring64Bitmap.deserialize keeps the empty containers an xor left in the stream
    (art/Containers.java:276-303 reads every non-null slot), so deserialize -> serialize returns the same bytes,
    and a later op treats those containers like the ones the xor produced on the device."""
    import roaringbitmap_amd as rb
    from oracle import rbref64 as R64
    run = np.arange(100, 20000, dtype=np.uint64)
    arr = (np.uint64(1) << np.uint64(16)) + np.arange(0, 900, 3, dtype=np.uint64)
    other = (np.uint64(5) << np.uint64(32)) + np.arange(10, dtype=np.uint64)
    x, y = R64.Ref64.of(np.concatenate([run, arr, other])), R64.Ref64.of(np.concatenate([run, arr]))
    for r in (x, y):
        for _, b in r.buckets:
            b.run_optimize()
    xy = R64.bitmap_op(rb.XOR, x, y, False)
    art = xy.to_art()
    s = ctx.upload_art64([art, y.to_art()])
    assert s.serialize_art() == [art, y.to_art()]
    assert s.serialize_portable()[0] == xy.to_portable()
    assert np.array_equal(s.values(0), other)
    h = s.bucket_set(0).download()
    assert [(int(h.type[c]), int(h.card[c])) for c in range(len(h.key))] == [(2, 0), (0, 0), (2, 10)]
    dev = ctx.pairwise64(rb.RB64_BITMAP, rb.XOR, s, s, [0], [0]).serialize_art()[0]  # from the device result
    for op in (rb.AND, rb.OR, rb.XOR, rb.ANDNOT):
        got = ctx.pairwise64(rb.RB64_BITMAP, op, s, s, [0], [1]).serialize_art()[0]
        assert got == R64.bitmap_op(op, xy, y, False).to_art(), op
    assert dev == R64.bitmap_op(rb.XOR, xy, xy, False).to_art()


def test_roaring64_kept_empty_through_later_ops(ctx, oracle):
    """x.xor(y) keeps an empty container under its key (Roaring64Bitmap.java:468-495);
    a later in-place andNot / or with a bitmap lacking that high leaves x's unmatched key untouched
    (:599-628, 392-419), and the static forms clone it — the empty container stays in the bytes (ART
    stream, the oracle's canonical writer) while the values agree."""
    import roaringbitmap_amd as rb
    from oracle import rbref64 as R64
    H = np.uint64(5 << 32)
    xv, yv, zv = H | np.arange(3, dtype=np.uint64), H | np.arange(3, dtype=np.uint64), np.array([1 << 40], np.uint64)
    for op, name in ((rb.ANDNOT, "andNot"), (rb.OR, "or_")):
        x, y, z = (rb.Roaring64Bitmap.bitmapOf(v) for v in (xv, yv, zv))
        x.xor(y)
        ref = R64.bitmap_op(rb.XOR, R64.Ref64.of(xv), R64.Ref64.of(yv), True)
        assert x.serialize() == ref.to_art() and x.isEmpty()
        getattr(x, name)(z)
        ref_i = R64.bitmap_op(op, ref, R64.Ref64.of(zv), True)
        assert x.serialize() == ref_i.to_art(), name
        assert np.array_equal(x.toArray(), ref_i.to_array())

"""Parity of the MI355X pairwise path (librbgpu k_pairwise) with the oracle: identical
RoaringFormatSpec bytes for every result, identical cardinalities.  Every test runs twice: batches of
<= 4096 pairs through the two-launch small-batch path (k_pair_small), and with RBGPU_NO_SMALL_PAIRS=1
through the general pipeline (merge-path segments, light / heavy task kernels)."""
import numpy as np
import pytest

from datasets import (DATASETS, EXPECTED, fixture_bytes, load_realdata, ornot_fuzz_bitmaps, range_bitmap_bytes,
                      synthetic_bitmaps)

pytestmark = pytest.mark.gpu
OPS = {"AND": 0, "OR": 1, "XOR": 2, "ANDNOT": 3}


@pytest.fixture(autouse=True, params=["small", "general"])
def pair_path(request, monkeypatch):
    monkeypatch.setenv("RBGPU_NO_SMALL_PAIRS", "1" if request.param == "general" else "0")
    return request.param


def _ref_list(oracle, blobs):
    return [oracle.RefBitmap.deserialize(b) for b in blobs]


@pytest.mark.parametrize("name", DATASETS)
@pytest.mark.parametrize("run_optimize", [False, True])
def test_realdata_pairwise_bytes_and_golden(ctx, oracle, name, run_optimize):
    vals = load_realdata(name)
    s = ctx.upload_values(vals, run_optimize=run_optimize)
    refs = _ref_list(oracle, s.serialize())
    n = len(vals) - 1
    a_idx = np.arange(n, dtype=np.uint32)
    b_idx = a_idx + 1
    for opname, op in OPS.items():
        out = ctx.pairwise(op, s, s, a_idx, b_idx)
        got = out.serialize()
        for k in range(n):
            assert got[k] == oracle.op(op, refs[k], refs[k + 1]).serialize(), (opname, k)
        assert int(out.cardinalities().sum()) == EXPECTED[name][opname]
        cards = ctx.pairwise_cardinality(op, s, s, a_idx, b_idx)
        assert int(cards.sum()) == EXPECTED[name][opname]


@pytest.mark.parametrize("seed", [1, 2, 3])
@pytest.mark.parametrize("opname", list(OPS))
def test_synthetic_all_type_pairs(ctx, oracle, seed, opname):
    op = OPS[opname]
    bms = synthetic_bitmaps(80, seed=seed)
    for ro in (False, True):
        s = ctx.upload_values(bms, run_optimize=ro)
        refs = _ref_list(oracle, s.serialize())
        rng = np.random.default_rng(seed + 100)
        a_idx = rng.integers(0, len(bms), size=300).astype(np.uint32)
        b_idx = rng.integers(0, len(bms), size=300).astype(np.uint32)
        out = ctx.pairwise(op, s, s, a_idx, b_idx)
        got = out.serialize()
        cards = ctx.pairwise_cardinality(op, s, s, a_idx, b_idx)
        for i in range(len(a_idx)):
            ref = oracle.op(op, refs[a_idx[i]], refs[b_idx[i]])
            assert got[i] == ref.serialize(), (opname, ro, i)
            assert int(cards[i]) == oracle.op_cardinality(op, refs[a_idx[i]], refs[b_idx[i]])


def test_two_sets_and_identity_pairs(ctx, oracle):
    a_vals = synthetic_bitmaps(50, seed=21)
    b_vals = synthetic_bitmaps(50, seed=22)
    a = ctx.upload_values(a_vals, run_optimize=True)
    b = ctx.upload_values(b_vals, run_optimize=False)
    ra, rbs = _ref_list(oracle, a.serialize()), _ref_list(oracle, b.serialize())
    for op in OPS.values():
        got = ctx.pairwise(op, a, b).serialize()
        assert got == [oracle.op(op, ra[i], rbs[i]).serialize() for i in range(50)]


def _array_pair_bitmaps(rng):
    """Bitmaps of Array containers only, sized around the small-batch merge path's bounds (ca + cb <= 4088
    takes the merge, above it the register path): equal, disjoint, interleaved, nested and random arrays
    on shared keys, so ties fall on and off the merge's 64 lane boundaries."""
    def arr(key, lows):
        return (np.uint32(key) << np.uint32(16)) | np.asarray(sorted(set(int(x) for x in lows)), np.uint32)

    def rnd(n, lo=0, hi=65536):
        return rng.choice(np.arange(lo, hi), size=n, replace=False)

    base = rnd(4000)
    sizes = [(1, 1), (1, 4000), (4000, 88), (4000, 89), (4096, 1), (2000, 2000), (3000, 1088), (63, 65), (640, 640)]
    left, right = [], []
    for k, (na, nb) in enumerate(sizes):
        a = rnd(na)
        shared = a[: min(na, nb) // 2]
        b = np.concatenate([shared, rnd(nb)])[:nb]
        left.append(arr(k, a))
        right.append(arr(k, b))
    # equal arrays (XOR empty, AND = A), disjoint evens / odds, nested (B inside A), one value apart
    left.append(arr(20, base[:1500]))
    right.append(arr(20, base[:1500]))
    left.append(arr(21, np.arange(0, 4000, 2)))
    right.append(arr(21, np.arange(1, 4000, 2)))
    left.append(arr(22, base[:3000]))
    right.append(arr(22, base[1000:1500]))
    left.append(arr(23, np.arange(100, 2100)))
    right.append(arr(23, np.arange(101, 2101)))
    # one side of <= 64 values (closed-form placement) and just above it: all / none / some of it in the
    # other side, below / above every value of the other side, the extreme values 0 and 65535
    big = np.sort(rnd(3000, 1000, 60000))
    for k, small in enumerate((big[::47][:64], rnd(64, 0, 1000), np.concatenate([[0, 65535], big[5:40:7], rnd(20, 60001, 65535)]),
                               big[::46][:65], np.array([65535]), np.array([0, 999]))):
        left.append(arr(24 + k, big))
        right.append(arr(24 + k, small))
        left.append(arr(40 + k, small))
        right.append(arr(40 + k, big))
    a_bms, b_bms = [], []
    for i in range(len(left)):  # one bitmap per case, and one holding every case's key
        a_bms.append(left[i])
        b_bms.append(right[i])
    a_bms.append(np.sort(np.concatenate(left)))
    b_bms.append(np.sort(np.concatenate(right)))
    return a_bms, b_bms


def test_array_pairs_merge_path(ctx, oracle):
    """Array x Array keys of the small-batch kernel (merge path) against the oracle, bytes and
    cardinalities, for all four ops and both operand orders."""
    rng = np.random.default_rng(77)
    a_bms, b_bms = _array_pair_bitmaps(rng)
    a = ctx.upload_values(a_bms, run_optimize=False)
    b = ctx.upload_values(b_bms, run_optimize=False)
    ra, rbs = _ref_list(oracle, a.serialize()), _ref_list(oracle, b.serialize())
    for op in OPS.values():
        for x, y, rx, ry in ((a, b, ra, rbs), (b, a, rbs, ra)):
            got = ctx.pairwise(op, x, y).serialize()
            cards = ctx.pairwise_cardinality(op, x, y)
            for i in range(len(a_bms)):
                ref = oracle.op(op, rx[i], ry[i])
                assert got[i] == ref.serialize(), (op, i)
                assert int(cards[i]) == ref.cardinality(), (op, i)


def test_fixtures_through_the_device(ctx, oracle):
    w, wo = fixture_bytes("bitmapwithruns.bin"), fixture_bytes("bitmapwithoutruns.bin")
    s = ctx.upload_serialized([w, wo])
    assert s.serialize() == [w, wo]
    assert list(s.cardinalities()) == [200100, 200100]
    refs = _ref_list(oracle, [w, wo])
    for op in OPS.values():
        got = ctx.pairwise(op, s, s, [0, 1, 0], [1, 0, 0]).serialize()
        assert got == [oracle.op(op, refs[i], refs[j]).serialize() for i, j in ((0, 1), (1, 0), (0, 0))]


def test_empty_bitmaps_and_empty_batch(ctx, oracle):
    bms = [np.zeros(0, np.uint32), np.array([1, 2, 3], np.uint32), np.zeros(0, np.uint32)]
    s = ctx.upload_values(bms)
    refs = _ref_list(oracle, s.serialize())
    for op in OPS.values():
        got = ctx.pairwise(op, s, s, [0, 0, 1, 2], [0, 1, 0, 2]).serialize()
        assert got == [oracle.op(op, refs[i], refs[j]).serialize() for i, j in ((0, 0), (0, 1), (1, 0), (2, 2))]
        empty = ctx.pairwise(op, s, s, np.zeros(0, np.uint32), np.zeros(0, np.uint32))
        assert len(empty) == 0


def test_bad_inputs_raise(ctx):
    import roaringbitmap_amd as rb
    for i in range(1, 8):
        with pytest.raises(IOError):
            ctx.upload_serialized([fixture_bytes(f"crashproneinput{i}.bin")])
    s = ctx.upload_values([np.array([1], np.uint32)])
    with pytest.raises(ValueError):
        ctx.pairwise(rb.AND, s, s, [5], [0])
    # non-canonical run list (two touching runs) is rejected (RB_EINVAL)
    soa = rb.soa_from_values([np.array([1, 2, 3], np.uint32)], run_optimize=True)
    soa.type[0] = rb.RUN
    soa.nruns[0] = 2
    soa.payload[:8] = np.array([1, 0, 2, 1], np.uint16).view(np.uint8)
    soa.card[0] = 3
    with pytest.raises(ValueError):
        ctx.upload_soa(soa)


def test_generated_filter_posting_sample_parity(ctx, oracle):
    """Device-generated config-2 data: a downloaded sample must match the oracle byte for byte."""
    import roaringbitmap_amd as rb
    a, b = ctx.generate(rb.WL_FILTER_POSTING, 3000, seed=42)
    assert len(a) == 3000 and len(b) == 3000
    out = ctx.pairwise(rb.AND, a, b)
    ra = _ref_list(oracle, a.serialize(0, 400))
    rbs = _ref_list(oracle, b.serialize(0, 400))
    got = out.serialize(0, 400)
    for i in range(400):
        assert got[i] == oracle.op(rb.AND, ra[i], rbs[i]).serialize()
    # generated containers are canonical and runOptimize-stable
    h = a.download(0, 400)
    for i in range(h.n_containers):
        t, c, r = int(h.type[i]), int(h.card[i]), int(h.nruns[i])
        if t == rb.ARRAY:
            assert 1 <= c <= 4096
        elif t == rb.BITMAP:
            assert c > 4096
        else:
            assert 2 + 4 * r < min(8192, 2 * c)


def test_large_pairs_merge_path_segments(ctx, oracle):
    """Pairs of bitmaps with thousands of keys: key alignment is cut into merge-path segments of
    256 merged keys; matched keys straddling a cut must stay together and every op must still
    give the oracle's bytes (RoaringBitmap.and/or/xor/andNot key loops)."""
    rng = np.random.default_rng(77)
    bms = []
    for n_keys, space in ((3000, 5000), (2500, 5000), (700, 1400), (65536, 65536), (1, 65536), (0, 10)):
        keys = np.sort(rng.choice(space, size=n_keys, replace=False)).astype(np.uint32)
        vals = [np.unique(rng.integers(0, 65536, size=int(rng.integers(1, 40)))).astype(np.uint32) | (k << 16)
                for k in keys]
        bms.append(np.concatenate(vals) if vals else np.zeros(0, np.uint32))
    s = ctx.upload_values(bms, run_optimize=True)
    refs = _ref_list(oracle, s.serialize())
    a_idx = np.array([0, 1, 0, 2, 3, 3, 4, 5, 0, 3], np.uint32)
    b_idx = np.array([1, 0, 2, 1, 3, 0, 3, 0, 5, 4], np.uint32)
    for opname, op in OPS.items():
        got = ctx.pairwise(op, s, s, a_idx, b_idx).serialize()
        cards = ctx.pairwise_cardinality(op, s, s, a_idx, b_idx)
        for i in range(len(a_idx)):
            ref = oracle.op(op, refs[a_idx[i]], refs[b_idx[i]])
            assert got[i] == ref.serialize(), (opname, i)
            assert int(cards[i]) == ref.cardinality(), (opname, i)


def _run_values(rng, nruns, lo=0, hi=65536, full=False):
    """Sorted values of `nruns` random non-adjacent runs inside [lo, hi) (one container)."""
    if full:
        return np.arange(lo, hi, dtype=np.uint32)
    cuts = np.sort(rng.choice(np.arange(lo, hi + 1), size=2 * nruns, replace=False))
    starts, ends = cuts[0::2], cuts[1::2]  # [start, end) with end < next start: gaps >= 1
    return np.concatenate([np.arange(s, e, dtype=np.uint32) for s, e in zip(starts, ends)])


@pytest.mark.parametrize("seed", [5, 6])
def test_run_and_run_interval_path(ctx, oracle, seed):
    """Run AND Run takes the interval-intersection path when EFF says Run and both lists fit the
    wave's scratch, else the register bitmap: every run count / overlap shape against the oracle
    (RunContainer.and(RunContainer), RunContainer.java:381-456)."""
    rng = np.random.default_rng(seed)
    bms = []
    for r in (1, 2, 3, 7, 64, 100, 511, 1000, 1023, 1024, 1500, 2000, 2047):
        bms.append(_run_values(rng, r))
    bms.append(_run_values(rng, 0, full=True))                          # one run over the whole key
    bms.append(np.arange(65000, 65536, dtype=np.uint32))                # run ending at 65535
    bms.append(np.arange(0, 300, dtype=np.uint32))                      # run starting at 0
    bms.append(np.concatenate([np.arange(0, 10), np.arange(65530, 65536)]).astype(np.uint32))
    bms.append(_run_values(rng, 20, 30000, 31000))                     # narrow: small intersections
    bms.append(_run_values(rng, 900, 0, 8000))                          # short runs: Array/Bitmap results
    s = ctx.upload_values(bms, run_optimize=True)
    refs = _ref_list(oracle, s.serialize())
    n = len(bms)
    a_idx = np.repeat(np.arange(n), n).astype(np.uint32)
    b_idx = np.tile(np.arange(n), n).astype(np.uint32)
    out = ctx.pairwise(OPS["AND"], s, s, a_idx, b_idx)
    got = out.serialize()
    cards = ctx.pairwise_cardinality(OPS["AND"], s, s, a_idx, b_idx)
    for i in range(len(a_idx)):
        ref = oracle.op(OPS["AND"], refs[a_idx[i]], refs[b_idx[i]])
        assert got[i] == ref.serialize(), (int(a_idx[i]), int(b_idx[i]))
        assert int(cards[i]) == ref.cardinality(), (int(a_idx[i]), int(b_idx[i]))


def test_identity_segments_large_batch(ctx, oracle):
    """> 4096 index-free pairs of few-key bitmaps: one merge-path segment per pair (identity
    seg_begin, no count kernel) and the fused multi-array scan; every op against the oracle."""
    base_a = synthetic_bitmaps(50, seed=31)
    base_b = synthetic_bitmaps(50, seed=32)
    a_vals = [base_a[i % 50] for i in range(5000)]
    b_vals = [base_b[(7 * i) % 50] for i in range(5000)]
    a = ctx.upload_values(a_vals, run_optimize=True)
    b = ctx.upload_values(b_vals, run_optimize=True)
    ra = _ref_list(oracle, a.serialize()[:50])
    rbs = _ref_list(oracle, b.serialize()[:50])
    for opname, op in OPS.items():
        got = ctx.pairwise(op, a, b).serialize()
        cards = ctx.pairwise_cardinality(op, a, b)
        assert len(got) == 5000
        for i in range(0, 5000, 7):
            ref = oracle.op(op, ra[i % 50], rbs[i % 50])  # b_vals[i] == b_vals[i % 50]
            assert got[i] == ref.serialize(), (opname, i)
            assert int(cards[i]) == ref.cardinality(), (opname, i)


@pytest.mark.parametrize("opname", list(OPS))
def test_concurrent_task_phase_parity(ctx, oracle, opname):
    """>= 65536 tasks: the light and heavy task kernels run concurrently and the light tasks come
    from the shared chunk queue (two light launches).  Samples across the whole batch must match
    the oracle byte for byte; materialised and cardinality-only results must agree."""
    import roaringbitmap_amd as rb
    op = OPS[opname]
    n = 40000
    a, b = ctx.generate(rb.WL_FILTER_POSTING, n, seed=11)
    out = ctx.pairwise(op, a, b)
    assert any("||" in k["name"] for k in ctx.stats()["kernels"])  # the concurrent phase ran
    cards = ctx.pairwise_cardinality(op, a, b)
    assert np.array_equal(out.cardinalities().astype(np.uint64), cards[:n].astype(np.uint64))
    for first in range(0, n, 4000):
        cnt = 60
        ra = _ref_list(oracle, a.serialize(first, cnt))
        rbs = _ref_list(oracle, b.serialize(first, cnt))
        got = out.serialize(first, cnt)
        for i in range(cnt):
            assert got[i] == oracle.op(op, ra[i], rbs[i]).serialize(), (opname, first + i)


def test_ornot_fuzz_fixture_through_the_device(ctx, oracle):
    # testdata/ornot-fuzz-failure.json (TestRoaringBitmapOrNot.java:379-425): l (144 Bitmap / 33 Run
    # / 4 Array containers) and r (293 Array / 80 Run / 1 Bitmap), disjoint keys, plus the 65k-key
    # range [0, limit) of that test; every op over every ordered pair, then the test's expected side
    # l | ([0, limit) \ r) composed on the device.
    lb, rbytes = ornot_fuzz_bitmaps()
    l = oracle.RefBitmap.deserialize(lb)
    limit = int(l.to_array()[-1]) + 1
    blobs = [lb, rbytes, range_bitmap_bytes(limit)]
    s = ctx.upload_serialized(blobs)
    assert s.serialize() == blobs
    refs = _ref_list(oracle, blobs)
    a_idx = np.repeat(np.arange(3, dtype=np.uint32), 3)
    b_idx = np.tile(np.arange(3, dtype=np.uint32), 3)
    for opname, op in OPS.items():
        got = ctx.pairwise(op, s, s, a_idx, b_idx).serialize()
        cards = ctx.pairwise_cardinality(op, s, s, a_idx, b_idx)
        for i in range(len(a_idx)):
            ref = oracle.op(op, refs[a_idx[i]], refs[b_idx[i]])
            assert got[i] == ref.serialize(), (opname, int(a_idx[i]), int(b_idx[i]))
            assert int(cards[i]) == ref.cardinality(), (opname, int(a_idx[i]), int(b_idx[i]))
    diff = ctx.pairwise(OPS["ANDNOT"], s, s, np.array([2], np.uint32), np.array([1], np.uint32))
    got = ctx.pairwise(OPS["OR"], s, diff, np.array([0], np.uint32), np.array([0], np.uint32))
    want = oracle.op(OPS["OR"], refs[0], oracle.op(OPS["ANDNOT"], refs[2], refs[1]))
    assert got.serialize() == [want.serialize()]
    ra = refs[1].to_array()
    assert int(got.cardinalities()[0]) == limit - int((ra < limit).sum())


def test_small_batch_kernel_timing_switch(ctx, oracle, pair_path, monkeypatch):
    """RBGPU_SMALL_KERNEL_TIMES=1 (the bench's per-kernel census breakdown) only adds timing events
    around the small-batch launch: the same bytes, and the kernel's time in the call's stats (one launch:
    its last block compacts the slots)."""
    if pair_path != "small":
        pytest.skip("small-batch path only")
    bms = synthetic_bitmaps(40, seed=5)
    s = ctx.upload_values(bms, run_optimize=True)
    refs = _ref_list(oracle, s.serialize())
    a_idx = np.arange(39, dtype=np.uint32)
    b_idx = a_idx + 1
    for flag in ("0", "1"):
        monkeypatch.setenv("RBGPU_SMALL_KERNEL_TIMES", flag)
        for opname, op in OPS.items():
            got = ctx.pairwise(op, s, s, a_idx, b_idx).serialize()
            for k in range(len(a_idx)):
                assert got[k] == oracle.op(op, refs[k], refs[k + 1]).serialize(), (flag, opname, k)
            names = [k["name"] for k in ctx.stats()["kernels"]]
            if flag == "1":
                assert names == ["k_pair_small"], names
            else:
                assert not names, names

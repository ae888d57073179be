"""The CPU oracle against the reference's own known answers (no GPU needed)."""
import numpy as np
import pytest

from datasets import DATASETS, EXPECTED, fixture_bytes, load_realdata, ornot_fuzz_bitmaps, range_bitmap_bytes

OPS = ["AND", "OR", "XOR", "ANDNOT"]


@pytest.mark.parametrize("name", DATASETS)
@pytest.mark.parametrize("run_optimize", [False, True])
def test_realdata_golden_cardinalities(oracle, name, run_optimize):
    # RealDataBenchmark{And,Or,Xor,AndNot}Test: sum over consecutive pairs (k, k+1);
    # RealDataBenchmarkWide{OrNaive,AndNaive}Test: wide aggregate over all bitmaps.
    R = oracle
    bms = [R.RefBitmap.of(v) for v in load_realdata(name)]
    if run_optimize:  # the ROARING_WITH_RUN variant (BitmapFactory: bitmapOf + runOptimize)
        for b in bms:
            b.run_optimize()
    for opname in OPS:
        op = getattr(R, opname)
        total = sum(R.op(op, bms[k], bms[k + 1]).cardinality() for k in range(len(bms) - 1))
        assert total == EXPECTED[name][opname]
        total_c = sum(R.op_cardinality(op, bms[k], bms[k + 1]) for k in range(len(bms) - 1))
        assert total_c == EXPECTED[name][opname]
    assert R.wide(R.FAST_OR, bms).cardinality() == EXPECTED[name]["WIDE_OR"]
    assert R.wide(R.PAR_OR, bms).cardinality() == EXPECTED[name]["WIDE_OR"]
    assert R.wide(R.FAST_AND, bms).cardinality() == EXPECTED[name]["WIDE_AND"]
    assert R.wide_cardinality(R.OR, bms) == EXPECTED[name]["WIDE_OR"]


def test_fixture_round_trip_and_run_optimize_kat(oracle):
    # TestAdversarialInputs.testInputGoodFile1/2 (TestAdversarialInputs.java:32-48)
    R = oracle
    with_runs, without_runs = fixture_bytes("bitmapwithruns.bin"), fixture_bytes("bitmapwithoutruns.bin")
    a, b = R.RefBitmap.deserialize(with_runs), R.RefBitmap.deserialize(without_runs)
    assert a.cardinality() == 200100 and b.cardinality() == 200100
    assert a.serialize() == with_runs and b.serialize() == without_runs
    assert [c[1] for c in a.containers()] == [0, 0, 1, 1, 1, 1, 1, 0, 2, 2, 2]
    b.run_optimize()
    assert b.serialize() == with_runs  # runOptimize(withoutruns) reproduces withruns byte for byte


def test_ornot_fuzz_fixture_mixed_types(oracle):
    # testdata/ornot-fuzz-failure.json as TestRoaringBitmapOrNot.testBigOrNot(Static) reads it
    # (TestRoaringBitmapOrNot.java:379-425): the expected side of that test, l | ([0, limit) \ r),
    # composed from the oracle's OR / ANDNOT over Array/Bitmap/Run containers.
    R = oracle
    lb, rbytes = ornot_fuzz_bitmaps()
    l, r = R.RefBitmap.deserialize(lb), R.RefBitmap.deserialize(rbytes)
    assert l.serialize() == lb and r.serialize() == rbytes
    assert sorted(t for _, t, _, _ in l.containers()).count(2) == 33  # 33 Run / 144 Bitmap / 4 Array
    assert [sum(t == k for _, t, _, _ in r.containers()) for k in (0, 1, 2)] == [293, 1, 80]
    assert not {c[0] for c in l.containers()} & {c[0] for c in r.containers()}  # disjoint keys
    limit = int(l.to_array()[-1]) + 1
    rng_bm = R.RefBitmap.deserialize(range_bitmap_bytes(limit))
    assert rng_bm.cardinality() == limit
    expected = R.op(R.OR, l, R.op(R.ANDNOT, rng_bm, r))
    # l lies inside [0, limit) and shares no key with r, so the result is exactly [0, limit) \ r
    ra = r.to_array()
    assert expected.cardinality() == limit - int((ra < limit).sum())
    assert R.op_cardinality(R.AND, expected, r) == 0
    assert R.op_cardinality(R.ANDNOT, expected, rng_bm) == 0
    assert R.op_cardinality(R.AND, l, r) == 0
    assert R.op(R.XOR, l, r).serialize() == R.op(R.OR, l, r).serialize()
    assert R.op(R.ANDNOT, l, r).serialize() == lb  # unmatched left containers are cloned as-is


@pytest.mark.parametrize("i", range(1, 8))
def test_crashprone_inputs_rejected(oracle, i):
    # TestAdversarialInputs.testInputBadFile8 (TestAdversarialInputs.java:18-21, 50-62)
    with pytest.raises(IOError):
        oracle.RefBitmap.deserialize(fixture_bytes(f"crashproneinput{i}.bin"))


def _one(oracle, values, run_optimize):
    b = oracle.RefBitmap.of(np.asarray(values, np.uint32))
    if run_optimize:
        b.run_optimize()
    return b


def test_type_pins_full_or_is_run(oracle):
    # TestRunContainer.orFullToRunContainer{,2,3} (TestRunContainer.java:2634-2662)
    R = oracle
    cases = [
        (_one(R, range(0, 1 << 15), True), _one(R, range(1 << 15, 1 << 16), False)),   # Run | Bitmap
        (_one(R, range(1024 - 200, 1 << 16), True), _one(R, range(0, 1024), False)),   # Run | Array
        (_one(R, range(0, 1 << 15), True), _one(R, range((1 << 15) - 200, 1 << 16), True)),  # Run | Run
    ]
    for x, y in cases:
        assert [c[1] for c in x.containers()][0] == R.RUN
        r = R.op(R.OR, x, y)
        assert r.containers() == [(0, R.RUN, 65536, 1)]


def test_type_pins_lazy_or_full(oracle):
    # TestRunContainer.testLazyORFull (TestRunContainer.java:3219-3228): naive_or repairs to a full Run
    R = oracle
    x = _one(R, range(0, 1 << 15), True)
    y = _one(R, range(3210, 1 << 16), False)
    assert R.wide(R.FAST_OR, [x, y]).containers() == [(0, R.RUN, 65536, 1)]


def test_in_place_vs_static_or_full(oracle):
    # BitmapContainer.ior(ArrayContainer) never converts a full bitmap (BitmapContainer.java:749-766)
    R = oracle
    x = _one(R, range(0, 65535), False)  # Bitmap, one value short of full
    y = _one(R, [65535], False)
    assert R.op(R.OR, x, y).containers()[0][1] == R.RUN
    z = x.clone()
    R.op_inplace(R.OR, z, y)
    assert z.containers()[0][1] == R.BITMAP


def test_bsi_known_answers(oracle):
    """The oracle's restatement of Roaring64BitmapSliceIndex.compare reproduces the reference's own
    known answers (bsi/src/test/java/org/roaringbitmap/bsi/R64BSITest.java: testGT/GE/LT/LE/RANGE/
    NEQ/EQ/ValueZero/Sum-style foundSet, and RBBsiTest.java's 32-bit twins)."""
    import numpy as np
    R = oracle
    cols = np.arange(1, 100)
    sl, ebm, mn, mx = R.bsi_build(cols, cols)

    def q(op, a, b=0, f=None, s=None):
        s = s or (sl, ebm, mn, mx)
        return list(R.bsi_compare(s[0], s[1], op, a, b, f, s[2], s[3]).to_array())
    assert q(R.BSI_GT, 50) == list(range(51, 100)) and q(R.BSI_GT, 0) == list(range(1, 100)) and q(R.BSI_GT, 99) == []
    assert q(R.BSI_GE, 50) == list(range(50, 100)) and q(R.BSI_GE, 1) == list(range(1, 100)) and q(R.BSI_GE, 100) == []
    assert q(R.BSI_LT, 50) == list(range(1, 50)) and q(R.BSI_LT, 2**31 - 1) == list(range(1, 100)) and q(R.BSI_LT, 1) == []
    assert q(R.BSI_LE, 50) == list(range(1, 51)) and q(R.BSI_LE, 2**31 - 1) == list(range(1, 100)) and q(R.BSI_LE, 0) == []
    assert q(R.BSI_RANGE, 10, 20) == list(range(10, 21)) and q(R.BSI_RANGE, 1, 200) == list(range(1, 100))
    assert q(R.BSI_RANGE, 1000, 2000) == []
    assert q(R.BSI_GE, 50, 0, R.RefBitmap.of(np.array([51, 52, 53], np.uint32))) == [51, 52, 53]
    neq = R.bsi_build([1, 2, 3], [99, 1, 50])
    assert q(R.BSI_NEQ, 99, s=neq) == [2, 3] and q(R.BSI_NEQ, 100, s=neq) == [1, 2, 3]
    same = R.bsi_build([1, 2, 3], [99, 99, 99])
    assert q(R.BSI_NEQ, 99, s=same) == [] and q(R.BSI_NEQ, 1, s=same) == [1, 2, 3]
    zero = R.bsi_build([0, 1, 2], [0, 0, 1])
    assert q(R.BSI_EQ, 0, s=zero) == [0, 1] and q(R.BSI_EQ, 1, s=zero) == [2]
    eq = R.bsi_build(list(range(1, 100)), [1 if x <= 50 else x for x in range(1, 100)])
    assert len(q(R.BSI_EQ, 1, s=eq)) == 50


def test_bsi_cpp_twin_matches_restatement(oracle):
    """rbref_bsi_compare (C++, the BSI CPU baseline's engine) gives the Python restatement's bytes — itself pinned
    by R64BSITest's known answers above — for every operation, with and without a foundSet, across the min/max
    shortcut's edges; rbref_bsi_compare_keys' total over per-key indexes is the same at 1 and 4 threads."""
    R = oracle
    rng = np.random.default_rng(21)
    for trial in range(4):
        n = int(rng.integers(50, 40000))
        cols = rng.integers(0, 1 << 18, n)
        vals = rng.integers(0, 1 << int(rng.integers(3, 40)), n, dtype=np.uint64)
        sl, ebm, mn, mx = R.bsi_build(cols, vals)
        found = R.RefBitmap.of(np.unique(rng.integers(0, 1 << 18, 3000)).astype(np.uint32))
        for op in range(7):
            for a, b in ((mn, mx), (mn - 1 if mn else 0, mx + 1), (int(vals[0]), int(vals[-1])),
                         (int(rng.integers(mn, mx + 1)), int(rng.integers(mn, mx + 1))), (mx + 1, mx + 5)):
                lo, hi = min(a, b), max(a, b)
                for f in (None, found):
                    want = R.bsi_compare(sl, ebm, op, lo, hi, f, mn, mx).serialize()
                    assert R.bsi_compare_cpp(sl, ebm, op, lo, hi, f, mn, mx).serialize() == want, (trial, op, lo, hi)
    per_key = []
    for k in range(6):
        cols = rng.integers(0, 65536, 5000)
        vals = rng.integers(0, 1 << 20, 5000, dtype=np.uint64)
        sl, ebm, _, _ = R.bsi_build(cols, vals)
        sl = sl + [R.RefBitmap.of(np.zeros(0, np.uint32))] * (20 - len(sl))  # one slice count for every key
        per_key.append((sl, ebm))
    want = sum(R.bsi_compare(sl, eb, R.BSI_RANGE, 1000, 600000, None, 0, (1 << 20) - 1).cardinality()
               for sl, eb in per_key)
    for th in (1, 4):
        assert R.bsi_compare_keys(per_key, R.BSI_RANGE, 1000, 600000, 0, (1 << 20) - 1, th) == want


@pytest.mark.parametrize("sem", ["FAST_OR", "FAST_AND", "WORKSHY_AND", "FAST_XOR", "PAR_OR", "PAR_XOR"])
def test_key_parallel_restatement_matches(oracle, sem):
    """rbref_wide_mt (the all-cores CPU baseline) gives the single-threaded oracle's bytes for every
    key-independent semantics, on real data and on mixed synthetic bitmaps."""
    from datasets import synthetic_bitmaps
    R = oracle
    sets = [[R.RefBitmap.of(v) for v in load_realdata("census1881_srt")[:60]],
            [R.RefBitmap.of(v) for v in synthetic_bitmaps(40, seed=4, max_keys=6, key_space=6)]]
    for bms in sets:
        for r in bms[::2]:
            r.run_optimize()
        for n in (3, 11, len(bms)):
            want = R.wide(getattr(R, sem), bms[:n]).serialize()
            for threads in (1, 4):
                assert R.wide_mt(getattr(R, sem), bms[:n], threads).serialize() == want, (sem, n, threads)


def test_horizontal_and_priorityqueue_known_answers(oracle):
    """TestFastAggregation.java:22-69 (horizontal_or, horizontal_or2, priorityqueue_or,
    priorityqueue_or2): the union of {0,1,2}, {0,5,6}, {1<<16, 2<<16}; TestRoaringBitmap.java:3190-3320:
    horizontal_* / priorityqueue_* equal RoaringBitmap.or / xor (content)."""
    R = oracle
    rb1, rb2, rb3 = R.RefBitmap.of([0, 1, 2]), R.RefBitmap.of([0, 5, 6]), R.RefBitmap.of([1 << 16, 2 << 16])
    for sem in (R.HORIZONTAL_OR, R.PQ_OR):
        assert list(R.wide(sem, [rb1, rb2, rb3]).to_array()) == [0, 1, 2, 5, 6, 1 << 16, 2 << 16]
    rng = np.random.default_rng(7)
    for trial in range(6):
        bms = []
        for i in range(int(rng.integers(1, 30))):
            v = np.unique(rng.integers(0, 6 * 65536, int(rng.integers(1, 20000)))).astype(np.uint32)
            if i % 4 == 0:
                a = int(rng.integers(0, 6 * 65536 - 70000))
                v = np.union1d(v, np.arange(a, a + 70000, dtype=np.uint32))
            b = R.RefBitmap.of(v)
            if (i + trial) % 3 == 0:
                b.run_optimize()
            bms.append(b)
        u = R.wide(R.FAST_OR, bms).to_array()
        x = R.wide(R.FAST_XOR, bms).to_array()
        for sem in (R.HORIZONTAL_OR, R.PQ_OR):
            assert np.array_equal(R.wide(sem, bms).to_array(), u)
        for sem in (R.HORIZONTAL_XOR, R.PQ_XOR):
            assert np.array_equal(R.wide(sem, bms).to_array(), x)


def test_java_priority_queue_tie_order(oracle):
    """horizontal_or of bitmaps whose key-0 containers tie on cardinality: the result is the union
    whatever the order, and its container type follows the restated java.util.PriorityQueue order
    (deterministic: the same inputs in the same order give the same bytes)."""
    R = oracle
    bms = []
    for i in range(9):
        v = np.arange(100 * i, 100 * i + 50, dtype=np.uint32) if i % 2 else np.arange(0, 5000, 100, dtype=np.uint32)
        b = R.RefBitmap.of(v)
        if i % 3 == 0:
            b.run_optimize()
        bms.append(b)
    a = R.wide(R.HORIZONTAL_OR, bms).serialize()
    assert a == R.wide(R.HORIZONTAL_OR, bms).serialize()
    assert np.array_equal(R.RefBitmap.deserialize(a).to_array(), R.wide(R.FAST_OR, bms).to_array())


def test_oracle_sanitizers_clean():
    """The oracle under AddressSanitizer + UBSan (oracle/san_check.cpp via `make -C oracle san`):
    random bitmaps of every container type through each pairwise op, every wide semantics and
    the codec, including truncated / bit-flipped buffers (TestAdversarialInputs.java:18-62); the
    first sanitizer report aborts the run."""
    import os
    import shutil
    import subprocess

    if shutil.which(os.environ.get("CXX", "g++")) is None:
        pytest.skip("no host C++ compiler")
    root = os.path.join(os.path.dirname(__file__), "..", "oracle")
    subprocess.run(["make", "-s", "-C", root, "san_check"], check=True, timeout=600)
    r = subprocess.run([os.path.join(root, "san_check"), "25", "7"], capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "0 failures" in r.stdout


def test_buffer_reference_vectors_on_oracle(oracle):
    """buffer/TestFastAggregation.java:47-100 on the oracle's BufferFastAggregation restatement."""
    R = oracle
    a1 = [39173, 39174]
    a2 = [39173, 39174, 39175, 39176, 39177, 39178, 39179]
    p1 = [1232, 3324, 123, 43243, 1322, 7897, 8767]
    d1, d2, d4 = R.RefBitmap.of(p1), R.RefBitmap.of(a2), R.RefBitmap.of([])
    want3 = sorted(p1 + a2)
    assert R.wide(R.NAIVE_AND, [R.RefBitmap.of(a1), d2]).to_array().tolist() == a1
    for sem in (R.BUFFER_PQ_OR, R.BUFFER_PQ_OR_ITER):
        assert R.wide(sem, [d1, d2]).to_array().tolist() == want3
        assert R.wide(sem, [d1]).to_array().tolist() == sorted(p1)
        assert R.wide(sem, [d1, d4]).to_array().tolist() == sorted(p1)
        assert R.wide(sem, []).cardinality() == 0
    assert R.wide(R.BUFFER_PQ_XOR, [d1, d2]).to_array().tolist() == want3
    import pytest as _pytest
    for bad in ([d1], []):
        with _pytest.raises(ValueError):
            R.wide(R.BUFFER_PQ_XOR, bad)


def test_buffer_naive_or_chain_has_no_16_switch(oracle):
    """naive_or(MutableRoaringBitmap...) folds answer.lazyor(b) (buffer/BufferFastAggregation.java:711-717):
    the lazyIOR chain of ParallelAggregation.or for any count.  Below 16 containers per key both give the
    same bytes; at 20 Run containers ParallelAggregation.or starts from a lazy Bitmap (LR -> Bitmap) while
    the chain stays a Run (RunContainer.ior(Run) -> toEfficientContainer)."""
    R = oracle
    bms = []
    for k in range(20):
        b = R.RefBitmap.of(np.arange(2000 * k, 2000 * k + 501, dtype=np.uint32))
        b.run_optimize()
        bms.append(b)
    for n in (2, 7, 15):
        assert R.wide(R.BUFFER_NAIVE_OR, bms[:n]).serialize() == R.wide(R.PAR_OR, bms[:n]).serialize()
    chain, par = R.wide(R.BUFFER_NAIVE_OR, bms), R.wide(R.PAR_OR, bms)
    assert np.array_equal(chain.to_array(), par.to_array())
    assert chain.containers()[0][1] == R.RUN and par.containers()[0][1] == R.BITMAP
    # one bitmap: its containers cloned then repaired (a Run through toEfficientContainer)
    assert R.wide(R.BUFFER_NAIVE_OR, bms[:1]).serialize() == R.wide(R.PAR_OR, bms[:1]).serialize()


def test_buffer_pq_or_single_is_a_copy(oracle):
    """BufferFastAggregation.priorityqueue_or of one bitmap returns toMutableRoaringBitmap() (no repair),
    FastAggregation.priorityqueue_or repairs it: an inefficient Run stays a Run only in the buffer form."""
    R = oracle
    from type_pins import RUN, oracle_bitmap
    x = oracle_bitmap(R, RUN, np.arange(0, 6000, 2, dtype=np.uint32))  # 3000 one-value runs
    assert R.wide(R.BUFFER_PQ_OR, [x]).containers()[0][1] == R.RUN
    assert R.wide(R.BUFFER_PQ_OR_ITER, [x]).containers()[0][1] == R.RUN
    assert R.wide(R.PQ_OR, [x]).containers()[0][1] == R.ARRAY

"""The Python mirror of the reference's Java surface (roaringbitmap_amd/roaring.py) on the device:
RoaringBitmap static and in-place ops, cardinalities and runOptimize, FastAggregation,
ParallelAggregation and BufferFastAggregation, each against the oracle on census1881 bitmaps, plus the
reference's own buffer/TestFastAggregation.java vectors (content equalities and the
IllegalArgumentException of priorityqueue_xor)."""
import numpy as np
import pytest

from datasets import load_realdata

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def census(oracle):
    from roaringbitmap_amd import RoaringBitmap
    vals = load_realdata("census1881")[:24]
    bms = [RoaringBitmap.bitmapOf(v) for v in vals]
    refs = [oracle.RefBitmap.of(v) for v in vals]
    return bms, refs


def test_roaringbitmap_static_and_inplace(oracle, census):
    from roaringbitmap_amd import RoaringBitmap
    bms, refs = census
    statics = {"and_": oracle.AND, "or_": oracle.OR, "xor": oracle.XOR, "andNot": oracle.ANDNOT}
    cards = {"and_": "andCardinality", "or_": "orCardinality", "xor": "xorCardinality", "andNot": "andNotCardinality"}
    for i in range(len(bms) - 1):
        for name, op in statics.items():
            got = getattr(RoaringBitmap, name)(bms[i], bms[i + 1])
            want = oracle.op(op, refs[i], refs[i + 1])
            assert got.serialize() == want.serialize(), (name, i)
            assert getattr(RoaringBitmap, cards[name])(bms[i], bms[i + 1]) == want.cardinality()
            x, xr = bms[i].clone(), refs[i].clone()
            assert getattr(x, name)(bms[i + 1]) is None          # void, like the Java instance method
            oracle.op_inplace(op, xr, refs[i + 1])
            assert x.serialize() == xr.serialize(), ("in place", name, i)
            assert bms[i + 1].serialize() == refs[i + 1].serialize()  # the argument is unchanged
    # x.op(x): the reference's x2 == this branches
    x = bms[3].clone()
    x.and_(x)
    assert x.serialize() == refs[3].serialize()
    x.xor(x)
    assert x.isEmpty()


def test_roaringbitmap_run_optimize_and_sizes(oracle, census):
    from roaringbitmap_amd import RoaringBitmap
    bms, refs = census
    for b, r in zip(bms[:10], refs[:10]):
        x, xr = b.clone(), r.clone()
        assert x.runOptimize() == xr.run_optimize()
        assert x.serialize() == xr.serialize()
        assert x.serializedSizeInBytes() == len(xr.serialize())
        assert x.getCardinality() == xr.cardinality()
    assert RoaringBitmap.or_(bms[0], bms[1]).serialize() == oracle.op(oracle.OR, refs[0], refs[1]).serialize()


def test_fast_parallel_aggregation(oracle, census):
    from roaringbitmap_amd import FastAggregation, ParallelAggregation
    bms, refs = census
    cases = [("and_", oracle.FAST_AND), ("or_", oracle.FAST_OR), ("xor", oracle.FAST_XOR),
             ("naive_and", oracle.NAIVE_AND), ("naive_or", oracle.FAST_OR), ("naive_xor", oracle.FAST_XOR),
             ("horizontal_or", oracle.HORIZONTAL_OR), ("horizontal_xor", oracle.HORIZONTAL_XOR),
             ("priorityqueue_or", oracle.PQ_OR), ("priorityqueue_xor", oracle.PQ_XOR)]
    for lo, n in ((0, 3), (4, 12), (0, 24)):
        sub, rsub = bms[lo:lo + n], refs[lo:lo + n]
        for name, sem in cases:
            assert getattr(FastAggregation, name)(*sub).serialize() == oracle.wide(sem, rsub).serialize(), (name, n)
        buf = np.ones(1024, np.int64)
        assert FastAggregation.workShyAnd(buf, *sub).serialize() == oracle.wide(oracle.WORKSHY_AND, rsub).serialize()
        assert FastAggregation.workAndMemoryShyAnd(buf, *sub).serialize() == \
            oracle.wide(oracle.WORKSHY_AND, rsub).serialize()
        assert FastAggregation.and_(buf, *sub).serialize() == oracle.wide(oracle.FAST_AND, rsub).serialize()
        assert not buf.any()  # Arrays.fill(aggregationBuffer, 0L)
        assert FastAggregation.and_iterator(iter(sub)).serialize() == \
            oracle.wide(oracle.NAIVE_AND_ITER, rsub).serialize()
        assert ParallelAggregation.or_(*sub).serialize() == oracle.wide(oracle.PAR_OR, rsub).serialize()
        assert ParallelAggregation.xor(*sub).serialize() == oracle.wide(oracle.PAR_XOR, rsub).serialize()
        assert FastAggregation.andCardinality(*sub) == oracle.wide(oracle.WORKSHY_AND, rsub).cardinality()
        assert FastAggregation.orCardinality(*sub) == oracle.wide(oracle.FAST_OR, rsub).cardinality()
    with pytest.raises(ValueError):  # buffer should have at least 1024 elements (FastAggregation.java:53-55)
        FastAggregation.and_(np.zeros(10, np.int64), *bms[:12])
    with pytest.raises(ValueError):
        FastAggregation.workAndMemoryShyAnd(np.zeros(10, np.int64), *bms[:2])
    # a bitmap passed twice is the same object: naive_and skips the smallest by identity
    dup = [bms[2], bms[5], bms[2]]
    assert FastAggregation.naive_and(*dup).serialize() == \
        oracle.wide(oracle.NAIVE_AND, [refs[2], refs[5], refs[2]]).serialize()


def test_buffer_fast_aggregation(oracle, census):
    from roaringbitmap_amd import BufferFastAggregation as B
    bms, refs = census
    for lo, n in ((0, 2), (3, 9), (0, 24)):
        sub, rsub = bms[lo:lo + n], refs[lo:lo + n]
        w = lambda sem: oracle.wide(sem, rsub).serialize()  # noqa: E731
        assert B.and_(*sub).serialize() == w(oracle.FAST_AND)
        assert B.and_iterator(iter(sub)).serialize() == w(oracle.WORKSHY_AND)
        assert B.and_mutable(*sub).serialize() == w(oracle.WORKSHY_AND)
        assert B.naive_and_mutable(*sub).serialize() == w(oracle.NAIVE_AND_ITER)
        assert B.or_(*sub).serialize() == w(oracle.FAST_OR)
        assert B.or_mutable(*sub).serialize() == w(oracle.BUFFER_NAIVE_OR)
        assert B.xor(*sub).serialize() == w(oracle.FAST_XOR)
        assert B.priorityqueue_or(*sub).serialize() == w(oracle.BUFFER_PQ_OR)
        assert B.priorityqueue_or_iterator(iter(sub)).serialize() == w(oracle.BUFFER_PQ_OR_ITER)
        assert B.priorityqueue_xor(*sub).serialize() == w(oracle.BUFFER_PQ_XOR)
    with pytest.raises(ValueError):
        B.priorityqueue_xor(bms[0])


def test_buffer_reference_vectors():
    """buffer/TestFastAggregation.java:47-100: naive_and, priorityqueue_or (varargs and Iterator, with an
    empty and a single input), priorityqueue_xor's IllegalArgumentException."""
    from roaringbitmap_amd import BufferFastAggregation as B
    from roaringbitmap_amd import RoaringBitmap
    a1 = [39173, 39174]
    a2 = [39173, 39174, 39175, 39176, 39177, 39178, 39179]
    d1, d2 = RoaringBitmap.bitmapOf(a1), RoaringBitmap.bitmapOf(a2)
    assert B.naive_and(d1, d2).toArray().tolist() == a1
    assert B.naive_and(RoaringBitmap.bitmapOf([])).isEmpty()
    p1 = [1232, 3324, 123, 43243, 1322, 7897, 8767]
    d1, d2, d4 = RoaringBitmap.bitmapOf(p1), RoaringBitmap.bitmapOf(a2), RoaringBitmap.bitmapOf([])
    want3 = sorted(p1 + a2)
    assert B.priorityqueue_or(d1, d2).toArray().tolist() == want3
    assert B.priorityqueue_or(d1).toArray().tolist() == sorted(p1)
    assert B.priorityqueue_or(d1, d4).toArray().tolist() == sorted(p1)
    assert B.priorityqueue_or_iterator(iter([d1, d2])).toArray().tolist() == want3
    assert B.priorityqueue_or_iterator(iter([])).isEmpty()
    assert B.priorityqueue_or_iterator(iter([d1])).toArray().tolist() == sorted(p1)
    assert B.priorityqueue_xor(d1, d2).toArray().tolist() == want3
    with pytest.raises(ValueError):
        B.priorityqueue_xor(d1)


def test_buffer_parallel_aggregation(oracle, census):
    """BufferParallelAggregation.or / xor (buffer/BufferParallelAggregation.java:166-192) fold each key
    like ParallelAggregation (clone + lazyIOR below 16 containers, a lazy Bitmap from 16; clone + ixor
    with no removal): the RB_PAR_OR / RB_PAR_XOR results, on census bitmaps and on a run-optimised mix of
    Array / Bitmap / Run containers (the lazyIOR chain's states)."""
    from datasets import synthetic_bitmaps
    from roaringbitmap_amd import BufferParallelAggregation as BP
    from roaringbitmap_amd import RoaringBitmap
    bms, refs = census
    mixed_vals = synthetic_bitmaps(40, seed=11)
    mixed = [RoaringBitmap.bitmapOf(v) for v in mixed_vals]
    for b in mixed[::2]:
        b.runOptimize()
    mixed_refs = [oracle.RefBitmap.deserialize(b.serialize()) for b in mixed]
    for pool, rpool in ((bms, refs), (mixed, mixed_refs)):
        for lo, n in ((0, 2), (1, 9), (0, 17), (0, len(pool))):
            sub, rsub = pool[lo:lo + n], rpool[lo:lo + n]
            assert BP.or_(*sub).serialize() == oracle.wide(oracle.PAR_OR, rsub).serialize(), n
            assert BP.xor(*sub).serialize() == oracle.wide(oracle.PAR_XOR, rsub).serialize(), n

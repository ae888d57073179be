"""In-place instance ops x1.and/or/xor/andNot(x2) (rbgpu_pairwise_inplace) and runOptimize
(rbgpu_set_run_optimize) on the device, byte-exact against the oracle's restatement of
RoaringBitmap.and(x2) :1270-1296, or(x2) :2481-2523, xor(x2) :3296-3348, andNot(x2) :1346-1382 and
RoaringBitmap.runOptimize :2764-2775."""
import os

import numpy as np
import pytest

from datasets import DATASETS, load_realdata, synthetic_bitmaps

pytestmark = pytest.mark.gpu
OPS = {"AND": 0, "OR": 1, "XOR": 2, "ANDNOT": 3}


@pytest.fixture(params=["small", "general"])
def path(request, monkeypatch):
    """Both pairwise paths: the small-batch kernels and the general pipeline."""
    if request.param == "general":
        monkeypatch.setenv("RBGPU_NO_SMALL_PAIRS", "1")
    return request.param


def _inplace_ref(oracle, refs, op, i, j, same):
    x = refs[i].clone()
    oracle.op_inplace(op, x, x if same else refs[j])
    return x.serialize()


@pytest.mark.parametrize("name", DATASETS[:3])
def test_inplace_realdata(ctx, oracle, path, name):
    vals = load_realdata(name)[:80]
    for ro in (False, True):
        s = ctx.upload_values(vals, run_optimize=ro)
        refs = [oracle.RefBitmap.deserialize(b) for b in s.serialize()]
        n = len(refs)
        ai = np.concatenate([np.arange(n - 1), np.arange(0, n, 7)]).astype(np.uint32)
        bi = np.concatenate([np.arange(1, n), np.arange(0, n, 7)]).astype(np.uint32)  # then x.op(x) pairs
        for opname, op in OPS.items():
            got = ctx.pairwise_inplace(op, s, s, ai, bi).serialize()
            for k in range(len(ai)):
                want = _inplace_ref(oracle, refs, op, ai[k], bi[k], ai[k] == bi[k])
                assert got[k] == want, (name, ro, opname, k, ai[k], bi[k])


def test_inplace_two_sets_and_identity_is_by_object(ctx, oracle, path):
    """With two sets, equal indices are different objects: the container algebra runs (not the
    `x2 == this` branches), even when both hold the same bytes."""
    bms = synthetic_bitmaps(40, seed=21, max_keys=8, key_space=10)
    a = ctx.upload_values(bms, run_optimize=True)
    b = ctx.upload_values(bms, run_optimize=True)
    refs = [oracle.RefBitmap.deserialize(x) for x in a.serialize()]
    idx = np.arange(40, dtype=np.uint32)
    for opname, op in OPS.items():
        got = ctx.pairwise_inplace(op, a, b, idx, idx).serialize()
        for k in range(40):
            assert got[k] == _inplace_ref(oracle, refs, op, k, k, False), (opname, k)


def test_inplace_bitmap_ior_array_stays_bitmap(ctx, oracle, path):
    """BitmapContainer.ior(ArrayContainer) (BitmapContainer.java:749-766) returns this even when the
    union fills the container: x1.or(x2) keeps a full Bitmap where the static or() gives a full Run."""
    import roaringbitmap_amd as rb
    from type_pins import ARRAY, BITMAP, one_container_soa, oracle_bitmap
    full_minus = np.setdiff1d(np.arange(65536), np.arange(1000, 1700)).astype(np.uint32)
    missing = np.arange(1000, 1700, dtype=np.uint32)
    conts = [(BITMAP, full_minus), (ARRAY, missing)]
    s = ctx.upload_soa(one_container_soa(conts))
    got_i = ctx.pairwise_inplace(rb.OR, s, s, [0], [1]).download()
    got_s = ctx.pairwise(rb.OR, s, s, [0], [1]).download()
    assert int(got_i.type[0]) == BITMAP and int(got_i.card[0]) == 65536
    assert int(got_s.type[0]) == rb.RUN
    ref = oracle_bitmap(oracle, *conts[0])
    oracle.op_inplace(rb.OR, ref, oracle_bitmap(oracle, *conts[1]))
    assert ctx.pairwise_inplace(rb.OR, s, s, [0], [1]).serialize()[0] == ref.serialize()
    # the other operand order is ArrayContainer.ior(Bitmap) = x.or(this): a full Run
    assert int(ctx.pairwise_inplace(rb.OR, s, s, [1], [0]).download().type[0]) == rb.RUN


def test_inplace_self_keeps_inefficient_runs(ctx, oracle, path):
    """x.and(x) / x.or(x) return x as it is (`x2 == this`), where the static and(x, x) would re-type an
    inefficient Run container (EFF); x.xor(x) / x.andNot(x) clear x."""
    import roaringbitmap_amd as rb
    from type_pins import RUN, one_container_soa
    v = np.arange(0, 6000, 2, dtype=np.uint32)  # 3000 one-value runs: 12002 B as a Run, 6000 B as an Array
    s = ctx.upload_soa(one_container_soa([(RUN, v)]))
    for op in (rb.AND, rb.OR):
        h = ctx.pairwise_inplace(op, s, s, [0], [0]).download()
        assert int(h.type[0]) == RUN and int(h.nruns[0]) == 3000
        assert int(ctx.pairwise(op, s, s, [0], [0]).download().type[0]) == rb.ARRAY
    for op in (rb.XOR, rb.ANDNOT):
        assert ctx.pairwise_inplace(op, s, s, [0], [0]).n_containers == 0


def test_inplace_large_batch_general_path(ctx, oracle):
    """More pairs than the small-batch path takes (kSmallPairs = 4096), identity pairs mixed in."""
    bms = synthetic_bitmaps(300, seed=17, max_keys=6, key_space=8)
    s = ctx.upload_values(bms, run_optimize=True)
    refs = [oracle.RefBitmap.deserialize(x) for x in s.serialize()]
    rng = np.random.default_rng(5)
    ai = rng.integers(0, 300, 6000).astype(np.uint32)
    bi = rng.integers(0, 300, 6000).astype(np.uint32)
    bi[::5] = ai[::5]
    for opname, op in OPS.items():
        got = ctx.pairwise_inplace(op, s, s, ai, bi).serialize()
        for k in range(0, 6000, 13):
            assert got[k] == _inplace_ref(oracle, refs, op, ai[k], bi[k], ai[k] == bi[k]), (opname, k)


@pytest.mark.parametrize("name", DATASETS)
def test_run_optimize_realdata(ctx, oracle, name):
    vals = load_realdata(name)
    s = ctx.upload_values(vals, run_optimize=False)
    out, flags = s.run_optimize()
    got = out.serialize()
    for i, b in enumerate(s.serialize()):
        ref = oracle.RefBitmap.deserialize(b)
        assert bool(flags[i]) == ref.run_optimize(), (name, i)
        assert got[i] == ref.serialize(), (name, i)
    # idempotent: an optimized set stays as it is
    again, _ = out.run_optimize()
    assert again.serialize() == got


def test_run_optimize_run_inputs(ctx, oracle):
    """Run containers through toEfficientContainer (RunContainer.java:2326-2335), including lists far
    over 8 KiB (32767 one-value runs) and inefficient ones that become Arrays."""
    from type_pins import RUN, one_container_soa, oracle_bitmap
    sets = [np.arange(0, 65536, 2), np.arange(0, 65534, 2), np.arange(10, 3000, 3), np.arange(5, 50000),
            np.concatenate([np.arange(0, 100), np.arange(200, 40000, 2)])]
    conts = [(RUN, v.astype(np.uint32)) for v in sets]
    s = ctx.upload_soa(one_container_soa(conts))
    out, flags = s.run_optimize()
    got = out.serialize()
    for i, (t, v) in enumerate(conts):
        ref = oracle_bitmap(oracle, t, v)
        assert bool(flags[i]) == ref.run_optimize()
        assert got[i] == ref.serialize(), i

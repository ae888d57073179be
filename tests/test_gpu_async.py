"""rbgpu_pairwise_async (include/rbgpu.h; SURVEY §8b threading row): batches enqueued back to back return
before their results are complete, and every result is byte-identical to the synchronous call's (itself
oracle-pinned in test_gpu_pairwise / test_gpu_configs).  Covers: several pending results at once, a pending
result freed without a wait, a pending result as the next call's input, a caller's stream, and the
small-batch path (completes before the return)."""
import numpy as np
import pytest

from datasets import synthetic_bitmaps

pytestmark = pytest.mark.gpu
OPS = {"AND": 0, "OR": 1, "XOR": 2, "ANDNOT": 3}


@pytest.fixture(scope="module")
def pairs(ctx):
    import roaringbitmap_amd as rb
    a, b = ctx.generate(rb.WL_FILTER_POSTING, 70_000, seed=9)  # > 4096 pairs: the general pipeline
    yield a, b
    a.close()
    b.close()


def test_async_results_equal_sync(ctx, pairs):
    a, b = pairs
    want = {op: ctx.pairwise(op, a, b).serialize(0, 4000) for op in OPS.values()}
    pending = [(op, ctx.pairwise_async(op, a, b)) for op in OPS.values() for _ in range(2)]
    for op, r in pending:  # serialize settles the pending result first
        assert r.serialize(0, 4000) == want[op], op
    for _, r in pending:
        r.close()


def test_async_free_pending_and_chain(ctx, pairs, oracle):
    import roaringbitmap_amd as rb
    a, b = pairs
    r = ctx.pairwise_async(rb.OR, a, b)
    r.close()  # freed while its kernels may still run: the free waits for them
    x = ctx.pairwise_async(rb.AND, a, b)
    y = ctx.pairwise_async(rb.XOR, x, b)  # a pending result as an input
    want = ctx.pairwise(rb.XOR, ctx.pairwise(rb.AND, a, b), b).serialize(0, 3000)
    assert y.wait().serialize(0, 3000) == want
    assert int(x.wait().n_containers) == int(ctx.pairwise(rb.AND, a, b).n_containers)


def test_async_caller_stream_and_small_batch(ctx, pairs, oracle):
    import torch

    import roaringbitmap_amd as rb
    a, b = pairs
    s = torch.cuda.Stream(device=ctx.device)
    r = ctx.pairwise_async(rb.ANDNOT, a, b, stream=s.cuda_stream)
    s.synchronize()  # the caller's stream waits for the result
    assert r.serialize(0, 2000) == ctx.pairwise(rb.ANDNOT, a, b).serialize(0, 2000)
    bms = synthetic_bitmaps(30, seed=3)
    small = ctx.upload_values(bms, run_optimize=True)
    refs = [oracle.RefBitmap.deserialize(x) for x in small.serialize()]
    ai = np.arange(29, dtype=np.uint32)
    got = ctx.pairwise_async(rb.AND, small, small, ai, ai + 1).serialize()
    for i in range(29):
        assert got[i] == oracle.op(rb.AND, refs[i], refs[i + 1]).serialize()

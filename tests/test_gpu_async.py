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


def test_async_input_freed_before_wait(ctx, pairs):
    """an input freed while an asynchronous call still reads it.  The free waits for the
    context's pending work before its blocks return to the pool, so sets allocated right after (their
    blocks recycled, written by an upload and an empty result) do not overwrite what the pending kernels
    read: the result equals the synchronous one."""
    import roaringbitmap_amd as rb
    a, b = pairs
    a2 = ctx.pairwise(rb.OR, a, a)   # fresh sets with a's / b's values
    b2 = ctx.pairwise(rb.OR, b, b)
    want = {op: _digest(ctx.pairwise(op, a2, b2)) for op in (rb.OR, rb.XOR)}
    r1 = ctx.pairwise_async(rb.OR, a2, b2)
    r2 = ctx.pairwise_async(rb.XOR, a2, b2)
    a2.close()
    b2.close()
    junk = [ctx.pairwise(rb.AND, a, a), ctx.upload_values([np.arange(0, 70000, 7, dtype=np.uint32)] * 8),
            ctx.pairwise(rb.AND, a, b, np.zeros(0, np.uint32), np.zeros(0, np.uint32))]
    assert _digest(r1.wait()) == want[rb.OR]
    assert _digest(r2.wait()) == want[rb.XOR]
    for x in junk + [r1, r2]:
        x.close()


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


def _hip():
    import ctypes
    for name in ("libamdhip64.so", "/opt/rocm/lib/libamdhip64.so"):
        try:
            h = ctypes.CDLL(name)
        except OSError:
            continue
        h.hipMemcpyAsync.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t, ctypes.c_int, ctypes.c_void_p]
        h.hipMemcpyAsync.restype = ctypes.c_int
        return h
    raise RuntimeError("libamdhip64 not found")


def test_async_small_batch_caller_stream_consumer(ctx, oracle):
    """a <= 4096-pair batch returns on its last block's sequence word, before the kernel's end
    is signalled; the caller's stream must still see the complete result.  The consumer is device work on the
    caller's torch stream only (copies out of the result's HBM addresses from rbgpu_set_device_view, then torch
    kernels over them), queued right behind the call and read with nothing but that stream's own
    synchronisation; every container's metadata and payload equals the oracle's result."""
    import torch

    import roaringbitmap_amd as rb
    from roaringbitmap_amd.engine import HostSoA
    hip = _hip()
    bms = synthetic_bitmaps(64, seed=11)
    small = ctx.upload_values(bms, run_optimize=True)
    refs = [oracle.RefBitmap.deserialize(x) for x in small.serialize()]
    ai = np.arange(63, dtype=np.uint32)
    dev = torch.device("cuda", ctx.device)
    s = torch.cuda.Stream(device=dev)
    for rep, op in enumerate((rb.OR, rb.XOR, rb.AND, rb.ANDNOT, rb.OR)):
        with torch.cuda.stream(s):  # earlier work on the caller's stream: the call runs after it
            busy = torch.ones(1 << 22, device=dev).cumsum(0)
        r = ctx.pairwise_async(op, small, small, ai, ai + 1, stream=s.cuda_stream)
        v = r.device_view()
        nc = v["n_containers"]
        assert nc is not None  # the small path knows its count at the return
        with torch.cuda.stream(s):
            out = {}
            for f, dt, n in (("begin", torch.int64, 64), ("key", torch.int16, nc), ("type", torch.uint8, nc),
                             ("card", torch.int32, nc), ("nruns", torch.int16, nc), ("offset", torch.int64, nc),
                             ("payload", torch.uint8, int(v["payload_bytes"]))):
                t = torch.empty(max(n, 1), dtype=dt, device=dev)
                nbytes = n * t.element_size()
                if nbytes:
                    assert hip.hipMemcpyAsync(t.data_ptr(), v[f], nbytes, 3, s.cuda_stream) == 0
                out[f] = t[:n]
            # a torch kernel over the payload on the same stream (reads what the copies brought over)
            chk = out["payload"].to(torch.int64).sum()
            host = {f: t.to("cpu", non_blocking=False) for f, t in out.items()}
        assert int(chk.item()) == int(host["payload"].to(torch.int64).sum())
        h = HostSoA(begin=host["begin"].numpy().view(np.uint64)[:64].copy(),
                    key=host["key"].numpy().view(np.uint16), type=host["type"].numpy(),
                    card=host["card"].numpy().view(np.uint32), nruns=host["nruns"].numpy().view(np.uint16),
                    offset=host["offset"].numpy().view(np.uint64), payload=host["payload"].numpy())
        want = [oracle.op(op, refs[i], refs[i + 1]).serialize() for i in range(63)]
        got = ctx.upload_soa(h).serialize()
        assert got == want, (rep, op)
        del busy
        r.close()


def _digest(s):
    """Per-bitmap cardinalities and serialized sizes, container type counts, and the bytes of three
    1000-bitmap windows (head, middle, tail: the tail's tasks run last in the task kernels)."""
    n = len(s)
    wins = [s.serialize(lo, min(1000, n - lo)) for lo in (0, n // 2, max(0, n - 1000))]
    return (s.cardinalities().tobytes(), s.serialized_sizes().tobytes(), s.type_stats(), int(s.n_containers), wins)


def test_async_back_to_back(ctx, pairs):
    """Eight calls in flight with alternating ops, a synchronous call and an indexed asynchronous call in
    between, each equal to the synchronous result (the calls share the context's workspaces in stream
    order)."""
    import roaringbitmap_amd as rb
    a, b = pairs
    ops = [rb.AND, rb.OR, rb.XOR, rb.ANDNOT, rb.OR, rb.AND, rb.ANDNOT, rb.XOR]
    want = {}
    for op in set(ops):
        w = ctx.pairwise(op, a, b)
        want[op] = _digest(w)
        w.close()
    pend = [ctx.pairwise_async(op, a, b) for op in ops[:4]]
    mid = ctx.pairwise(rb.XOR, a, b)  # synchronous, behind four pending calls
    idx = np.arange(len(a), dtype=np.uint32)
    pend += [ctx.pairwise_async(op, a, b, idx, idx) for op in ops[4:5]]  # indexed: the non-pipelined path
    pend += [ctx.pairwise_async(op, a, b) for op in ops[5:]]
    assert _digest(mid) == want[rb.XOR]
    mid.close()
    for op, r in zip(ops, pend):
        assert _digest(r) == want[op], op
        r.close()


def test_async_release_order(ctx, pairs):
    """The bench's pattern: each step's result freed one step later (its free waits for it), 12 steps."""
    import roaringbitmap_amd as rb
    a, b = pairs
    w = ctx.pairwise(rb.AND, a, b)
    want = _digest(w)
    w.close()
    prev, got = None, []
    for i in range(12):
        r = ctx.pairwise_async(rb.AND, a, b)
        if prev is not None:
            if i % 4 == 0:
                got.append(_digest(prev))
            prev.close()
        prev = r
    got.append(_digest(prev.wait()))
    prev.close()
    assert all(g == want for g in got)

"""The library's multi-GPU exchange (include/rbgpu.h, multi-GPU section) on one MI355X: an RCCL
communicator of one rank, the shard summary all-gather, the device-side gather + header assembly
of the serialized result, the BSI shard path and the cardinality all-reduce.  World sizes > 1 need
one GPU per rank; their assembly logic is covered on the CPU (tests/test_sharding.py,
rbgpu_shard_assemble_host runs the same code as the gather kernel)."""
import numpy as np
import pytest

from datasets import load_realdata, synthetic_bitmaps

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def comm(ctx):
    from roaringbitmap_amd.engine import Comm
    c = Comm(ctx, Comm.unique_id(), 1, 0)
    yield c
    c.close()


def test_comm_wide_sharded_gather(ctx, oracle, comm):
    import roaringbitmap_amd as rb
    vals = load_realdata("census1881_srt")[:40] + synthetic_bitmaps(30, seed=3, max_keys=12, key_space=40)
    s = ctx.upload_values(vals, run_optimize=True)
    refs = [oracle.RefBitmap.deserialize(x) for x in s.serialize()]
    for sem in (rb.FAST_OR, rb.FAST_XOR, rb.WORKSHY_AND, rb.PAR_OR, rb.NAIVE_AND):
        want = ctx.wide(sem, s)
        want_bytes = want.serialize()[0]
        if sem in (rb.NAIVE_AND, rb.FAST_XOR):  # the shard path pinned to the oracle directly
            assert want_bytes == oracle.wide(sem, refs).serialize()
        local, summ = comm.wide_sharded(sem, s, (0, 65536))
        assert summ["serialized_size"] == len(want_bytes)
        assert summ["cardinality"] == int(want.cardinalities()[0])
        assert summ["container_offset"] == 0 and summ["local_serialized"] == len(want_bytes)
        assert comm.gather_serialized(local, summ) == want_bytes
        if sem == rb.NAIVE_AND:  # its fold order needs a whole partition of the keys (the counts' sum)
            continue
        # a sub-range shard at world size 1 is the whole result of that key range
        local2, summ2 = comm.wide_sharded(sem, s, (3, 17))
        part = ctx.wide(sem, s, key_range=(3, 17)).serialize()[0]
        assert comm.gather_serialized(local2, summ2) == part
        assert summ2["serialized_size"] == len(part)


def test_comm_bsi_sharded_and_allreduce(ctx, oracle, comm):
    import roaringbitmap_amd as rb
    d = ctx.generate_bsi(16, 3 * 65536 + 99, seed=5)
    for kr in ((0, 65536), (1, 3)):
        local, summ = comm.bsi_compare_sharded(rb.BSI_RANGE, d, 1000, 40000, 0, (1 << 16) - 1, kr)
        want = ctx.bsi_compare(rb.BSI_RANGE, d, 1000, 40000, 0, (1 << 16) - 1, key_range=kr).serialize()[0]
        assert comm.gather_serialized(local, summ) == want
    v = comm.allreduce_sum([1, 2, 3, 2**40])
    assert list(v) == [1, 2, 3, 2**40]


def test_range_counts_partition_sum_gives_whole_order(ctx):
    """the sharded naive_and fold order comes from the per-range counts summed over the
    ranks (rbgpu_wide_sharded's all-reduce); over every partition the sums must equal the whole-range
    counts, so every shard folds the order the unsharded call folds (FastAggregation.java:328-346)."""
    from roaringbitmap_amd.sharding import partition_keys
    vals = load_realdata("census1881_srt")[:30] + synthetic_bitmaps(20, seed=11, max_keys=30, key_space=200)
    s = ctx.upload_values(vals, run_optimize=True)
    whole = s.range_counts()
    kb = s.key_bytes()
    for nparts in (2, 3, 5, 8):
        parts = partition_keys(kb, nparts)
        tot = sum(s.range_counts(None, p) for p in parts)
        assert np.array_equal(tot, whole), nparts
        mem = list(range(len(s)))
        sm = int(np.argmin(tot))
        assert [sm] + [m for m in mem if m != sm] == [int(np.argmin(whole))] + \
            [m for m in mem if m != int(np.argmin(whole))]


def test_comm_errors_are_collective(ctx, comm):
    """A bad argument on one rank fails the call on that rank without a dangling collective (world 1:
    the call returns instead of waiting); the communicator stays usable afterwards."""
    import ctypes as C

    import roaringbitmap_amd as rb
    from roaringbitmap_amd import _lib as L
    s = ctx.upload_values(synthetic_bitmaps(6, seed=2, max_keys=5, key_space=10), run_optimize=True)
    local, summ = comm.wide_sharded(rb.FAST_OR, s, (0, 65536))
    ss = L.RbShardSummary(**summ)
    rc = L.lib().rbgpu_shard_gather_serialized(comm.h, local.h, C.byref(ss), 0, None, 0)
    assert rc == L.RB_EINVAL
    assert comm.gather_serialized(local, summ) == ctx.wide(rb.FAST_OR, s).serialize()[0]
    # priorityqueue_or is a whole-result call: allowed at world size 1 over the whole key range
    pl, ps = comm.wide_sharded(rb.PQ_OR, s, (0, 65536))
    assert comm.gather_serialized(pl, ps) == ctx.wide(rb.PQ_OR, s).serialize()[0]

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
    for sem in (rb.FAST_OR, rb.FAST_XOR, rb.WORKSHY_AND, rb.PAR_OR, rb.NAIVE_AND):
        want = ctx.wide(sem, s)
        want_bytes = want.serialize()[0]
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

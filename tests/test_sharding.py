"""Key-range sharding of the wide aggregations, on the CPU: the byte-balanced key
partition, the RoaringFormatSpec writer over key-ordered parts, and the 2-rank gloo exchange
(summary all_gather + container gather) — the shard results themselves come from the oracle here,
the MI355X shards are covered by tests/test_gpu_wide.py."""
import os
import socket

import numpy as np
import pytest
import torch.multiprocessing as mp

from datasets import fixture_bytes, load_realdata, synthetic_bitmaps
from roaringbitmap_amd import _lib as L
from roaringbitmap_amd.engine import HostSoA, assemble_host, host_summary, soa_from_serialized
from roaringbitmap_amd.sharding import (ShardedWide, header_size, pair_bytes, partition_keys, partition_pairs,
                                        serialize_parts)

SEMS = {"FAST_OR": L.FAST_OR, "WORKSHY_AND": L.WORKSHY_AND, "FAST_XOR": L.FAST_XOR, "PAR_OR": L.PAR_OR,
        "PAR_XOR": L.PAR_XOR, "NAIVE_AND": L.NAIVE_AND, "HORIZONTAL_OR": L.HORIZONTAL_OR,
        "HORIZONTAL_XOR": L.HORIZONTAL_XOR}


def _subset(h: HostSoA, lo: int, hi: int) -> HostSoA:
    """Containers of bitmap 0 with keys in [lo, hi), as a one-bitmap host SoA."""
    sel = np.nonzero((h.key >= lo) & (h.key < hi))[0]
    return HostSoA(np.array([0, len(sel)], np.uint64), h.key[sel].copy(), h.type[sel].copy(), h.card[sel].copy(),
                   h.nruns[sel].copy(), h.offset[sel].copy(), h.payload)


def test_partition_keys_balanced():
    rng = np.random.default_rng(3)
    kb = np.zeros(65536, np.uint64)
    kb[rng.integers(0, 65536, 5000)] = rng.integers(1, 9000, 5000)
    for n in (1, 2, 3, 8):
        parts = partition_keys(kb, n)
        assert parts[0][0] == 0 and parts[-1][1] == 65536
        assert all(parts[i][1] == parts[i + 1][0] for i in range(n - 1))
        share = kb.sum() / n
        for lo, hi in parts:
            assert int(kb[lo:hi].sum()) <= share + int(kb.max())
    # a single heavy key: the other ranges may be empty, nothing is lost
    kb = np.zeros(65536, np.uint64)
    kb[7] = 100
    parts = partition_keys(kb, 4)
    assert sum(int(kb[lo:hi].sum()) for lo, hi in parts) == 100


def test_writer_matches_reference_fixtures():
    # testdata/bitmapwithruns.bin / bitmapwithoutruns.bin (TestAdversarialInputs.java:32-48)
    for name in ("bitmapwithruns.bin", "bitmapwithoutruns.bin"):
        data = fixture_bytes(name)
        h = soa_from_serialized([data])
        assert serialize_parts([h]) == data
        # split at every container boundary region, including shards of < 4 containers with Runs
        # (no offset table: the assembly walks their payloads) and empty shards
        nk = len(h.key)
        for cuts in ([0, nk], [0, 1, nk], [0, 2, 3, nk], [0, 0, nk // 2, nk, nk], [0, nk - 3, nk - 1, nk]):
            parts = [_subset(h, int(h.key[a]) if a < nk else 65536, int(h.key[b]) if b < nk else 65536)
                     for a, b in zip(cuts[:-1], cuts[1:])]
            assert assemble_host([serialize_parts([p]) for p in parts]) == data, cuts


def test_assemble_host_edges():
    empty = serialize_parts([HostSoA(np.zeros(2, np.uint64), np.zeros(0, np.uint16), np.zeros(0, np.uint8),
                                     np.zeros(0, np.uint32), np.zeros(0, np.uint16), np.zeros(0, np.uint64),
                                     np.zeros(16, np.uint8))])
    assert assemble_host([empty, empty]) == empty
    assert assemble_host([]) == empty
    with pytest.raises(L.FormatError):
        assemble_host([b"\x01\x02\x03\x04\x05\x06\x07\x08"])


@pytest.mark.parametrize("run_optimize", [False, True])
def test_split_and_reassemble(oracle, run_optimize):
    bms = synthetic_bitmaps(40, seed=11, max_keys=8, key_space=12)
    for v in bms:
        r = oracle.RefBitmap.of(v)
        if run_optimize:
            r.run_optimize()
        data = r.serialize()
        h = soa_from_serialized([data])
        for n in (2, 3, 5):
            kb = np.zeros(65536, np.uint64)
            np.add.at(kb, h.key.astype(np.int64), 1)
            parts = [_subset(h, lo, hi) for lo, hi in partition_keys(kb, n)]
            assert serialize_parts(parts) == data
            # the library's gather assembly (rbgpu_shard_assemble_host, the code the root GPU runs)
            # from each shard's standalone bytes
            assert assemble_host([serialize_parts([p]) for p in parts]) == data
            s = host_summary(h)
            assert len(data) == header_size(s["n_containers"], s["n_run_containers"] > 0) + s["payload_bytes"]


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _rank_main(rank, world, port, q):
    import torch.distributed as dist

    from oracle import rbref as R
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        vals = load_realdata("census1881_srt")[:64] + synthetic_bitmaps(24, seed=5, max_keys=10, key_space=40)
        full = [R.RefBitmap.of(v) for v in vals]
        for r in full[::3]:
            r.run_optimize()
        hs = soa_from_serialized([r.serialize() for r in full])
        kb = np.zeros(65536, np.uint64)
        np.add.at(kb, hs.key.astype(np.int64), 1)
        parts = partition_keys(kb, world)
        lo, hi = parts[rank]
        sw = ShardedWide(dist, rank, world)
        out = {}
        for name, sem in SEMS.items():
            # this rank's key range of every input, in member order
            shard_in = []
            for i, r in enumerate(full):
                v = r.to_array()
                key = v >> 16
                sub = R.RefBitmap.of(v[(key >= lo) & (key < hi)])
                if i % 3 == 0:
                    sub.run_optimize()
                shard_in.append(sub)
            if name == "NAIVE_AND":  # the fold order from the all-reduced range counts
                order = sw.naive_and_order([len(x.containers()) for x in shard_in], list(range(len(shard_in))))
                local = soa_from_serialized([R.wide(R.NAIVE_AND_ITER, [shard_in[i] for i in order]).serialize()])
            else:
                local = soa_from_serialized([R.wide(sem, shard_in).serialize()])
            res = sw.finish(local, (lo, hi), host_summary(local))
            data = sw.gather_serialized(res)
            if rank == 0:
                want = R.wide(sem, full)
                out[name] = (data == want.serialize(), res.cardinality == want.cardinality(),
                             res.serialized_size == len(want.serialize()))
        if rank == 0:
            q.put(out)
    finally:
        dist.destroy_process_group()


def _spawn(target, world=2):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=target, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    out = q.get(timeout=240)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    return out


def test_gloo_two_rank_sharded_wide():
    for name, ok in _spawn(_rank_main).items():
        assert all(ok), (name, ok)


def test_partition_pairs_balanced():
    rng = np.random.default_rng(9)
    pb = rng.integers(0, 20000, 3001).astype(np.uint64)
    for n in (1, 2, 3, 8):
        parts = partition_pairs(pb, n)
        assert parts[0][0] == 0 and parts[-1][1] == len(pb)
        assert all(parts[i][1] == parts[i + 1][0] for i in range(n - 1))
        for lo, hi in parts:
            assert int(pb[lo:hi].sum()) <= pb.sum() / n + int(pb.max())
    assert partition_pairs(np.zeros(0, np.uint64), 3) == [(0, 0)] * 3
    assert list(pair_bytes(np.array([5, 7]), np.array([1, 2, 3]), np.array([1, 0]), np.array([2, 2]))) == [10, 8]


def _restrict(R, r, lo, hi):
    """The containers of oracle bitmap r with high keys in [lo, hi) (bitmapOf-built, as r is)."""
    v = r.to_array()
    k = v >> 16
    return R.RefBitmap.of(v[(k >= lo) & (k < hi)])


def _bsi_case(R, seed=4):
    """A BSI over ~6 high keys of rows (bitmapOf-built slices, BitmapSliceIndex.setValue order)."""
    rng = np.random.default_rng(seed)
    cols = np.unique(rng.integers(0, 6 * 65536, 40000)).astype(np.uint64)
    vals = rng.integers(0, 1 << 20, len(cols)).astype(np.uint64)
    slices, ebm, vmin, vmax = R.bsi_build(cols, vals)
    found = R.RefBitmap.of(cols[rng.random(len(cols)) < 0.6].astype(np.uint32))
    return slices, ebm, vmin, vmax, found


BSI_QUERIES = [  # (op, start, end, with foundSet)
    ("RANGE", 1 << 18, 3 << 18, False), ("GE", 12345, 0, True), ("LT", 99999, 0, False), ("EQ", None, 0, False),
    ("NEQ", None, 0, True), ("GT", 0, 0, False),  # GT 0 with min 0: the O'Neil path
    ("LE", 1 << 40, 0, True),  # LE above max: the min/max shortcut (all of ebM AND foundSet)
]


def _rank_bsi(rank, world, port, q):
    import torch.distributed as dist

    from oracle import rbref as R
    from roaringbitmap_amd.sharding import ShardedBsi
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        slices, ebm, vmin, vmax, found = _bsi_case(R)
        kb = np.zeros(65536, np.uint64)
        h = soa_from_serialized([ebm.serialize()])
        np.add.at(kb, h.key.astype(np.int64), 1)
        lo, hi = partition_keys(kb, world)[rank]
        # this rank's shard of the index: slices + ebM (+ foundSet) restricted to its key range
        s_sl = [_restrict(R, s, lo, hi) for s in slices]
        s_eb, s_fd = _restrict(R, ebm, lo, hi), _restrict(R, found, lo, hi)
        sw = ShardedBsi(dist, rank, world)
        out = {}
        for name, start, end, use_found in BSI_QUERIES:
            op_ = getattr(R, "BSI_" + name)
            if start is None:  # EQ the minimum value, NEQ 0
                start = 0 if name == "NEQ" else int(vmin)
            local = R.bsi_compare(s_sl, s_eb, op_, start, end, s_fd if use_found else None, vmin, vmax)
            hl = soa_from_serialized([local.serialize()])
            res = sw.finish(hl, (lo, hi), host_summary(hl))
            data = sw.gather_serialized(res)
            if rank == 0:
                want = R.bsi_compare(slices, ebm, op_, start, end, found if use_found else None, vmin, vmax)
                out[name] = (data == want.serialize(), res.cardinality == want.cardinality(),
                             res.serialized_size == len(want.serialize()))
        if rank == 0:
            q.put(out)
    finally:
        dist.destroy_process_group()


def test_gloo_two_rank_sharded_bsi():
    for name, ok in _spawn(_rank_bsi).items():
        assert all(ok), (name, ok)


def _rank_pairs(rank, world, port, q):
    import torch.distributed as dist

    from oracle import rbref as R
    from roaringbitmap_amd.sharding import ShardedPairwise
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        vals = load_realdata("census1881_srt")[:60] + synthetic_bitmaps(20, seed=8, max_keys=6, key_space=16)
        bms = [R.RefBitmap.of(v) for v in vals]
        for r in bms[1::4]:
            r.run_optimize()
        sizes = np.array([len(r.serialize()) for r in bms], np.uint64)
        rng = np.random.default_rng(1)
        ai = rng.integers(0, len(bms), 150).astype(np.uint32)
        bi = rng.integers(0, len(bms), 150).astype(np.uint32)
        sp = ShardedPairwise(dist, rank, world)
        lo, hi = sp.split(pair_bytes(sizes, sizes, ai, bi))
        out = {}
        for name, opc in (("AND", L.AND), ("OR", L.OR), ("XOR", L.XOR), ("ANDNOT", L.ANDNOT)):
            local = [R.op(opc, bms[a], bms[b]) for a, b in zip(ai[lo:hi], bi[lo:hi])]
            res = sp.finish([r.serialize() for r in local], (lo, hi), sum(r.cardinality() for r in local),
                            sum(len(r.containers()) for r in local), 0)
            got = sp.gather_serialized(res)
            if rank == 0:
                want = [R.op(opc, bms[a], bms[b]) for a, b in zip(ai, bi)]
                out[name] = (got == [w.serialize() for w in want],
                             res.cardinality == sum(w.cardinality() for w in want),
                             res.n_containers == sum(len(w.containers()) for w in want))
        if rank == 0:
            q.put(out)
    finally:
        dist.destroy_process_group()


def test_gloo_two_rank_sharded_pairwise():
    for name, ok in _spawn(_rank_pairs).items():
        assert all(ok), (name, ok)


def _rank_pq_refused(rank, world, port, q):
    import torch.distributed as dist

    from roaringbitmap_amd.sharding import ShardedWide
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        # every byte on key 65535: partition_keys gives rank 0 the whole range, rank 1 an empty one
        kb = np.zeros(65536, np.uint64)
        kb[65535] = 100
        key_range = partition_keys(kb, world)[rank]
        sw = ShardedWide(dist, rank, world)
        raised = {}
        for sem in (L.PQ_OR, L.PQ_XOR):
            try:
                sw.aggregate(None, sem, [object()], key_range)  # refused before touching ctx / dset
                raised[sem] = False
            except ValueError:
                raised[sem] = True
        dist.barrier()  # both ranks reach here: no rank waits in a collective
        g = sw._all_gather_i64([int(all(raised.values()))])
        if rank == 0:
            q.put({"raised": bool(g[:, 0].all()), "ranges": partition_keys(kb, world)})
    finally:
        dist.destroy_process_group()


def test_gloo_two_rank_pq_refused_on_every_rank():
    """priorityqueue_or / _xor are refused alike on every rank (no rank left waiting)."""
    out = _spawn(_rank_pq_refused)
    assert out["raised"]
    assert out["ranges"] == [(0, 65536), (65536, 65536)]


# ---- the library's own exchange code (comm.hip) over a host transport: rbgpu_comm_init_host with a gloo
# group, so the sequencing a multi-GPU run takes through RCCL (summaries, failure agreement, naive_and's
# global order, the shard gather, the header assembly) runs here with 2 and 3 ranks
def _rank_host_comm(rank, world, port, q):
    import torch.distributed as dist

    from oracle import rbref as R
    from roaringbitmap_amd.engine import HostComm, HostTransport
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    out = {}
    comm = None
    try:
        comm = HostComm(HostTransport(dist))
        vals = load_realdata("census1881_srt")[:48] + synthetic_bitmaps(24, seed=5, max_keys=10, key_space=40)
        full = [R.RefBitmap.of(v) for v in vals]
        for r in full[::3]:
            r.run_optimize()
        hs = soa_from_serialized([r.serialize() for r in full])
        kb = np.zeros(65536, np.uint64)
        np.add.at(kb, hs.key.astype(np.int64), 1)
        lo, hi = partition_keys(kb, world)[rank]
        shard_in = []
        for i, r in enumerate(full):
            v = r.to_array()
            sub = R.RefBitmap.of(v[((v >> 16) >= lo) & ((v >> 16) < hi)])
            if i % 3 == 0:
                sub.run_optimize()
            shard_in.append(sub)
        members = list(range(len(shard_in)))
        for name, sem in SEMS.items():
            if name == "NAIVE_AND":  # the global fold order from the all-reduced range counts, in C
                order = comm.naive_and_order(members, [len(x.containers()) for x in shard_in])
                local = R.wide(R.NAIVE_AND_ITER, [shard_in[i] for i in order]).serialize()
            else:
                local = R.wide(sem, shard_in).serialize()
            summ = comm.summarize_serialized(local)
            data = comm.gather_host(local, summ)
            if rank == 0:
                want = R.wide(sem, full)
                out[name] = (data == want.serialize(), summ["cardinality"] == want.cardinality(),
                             summ["serialized_size"] == len(want.serialize()))
        # a Run-marker byte straddling a rank boundary, and shards of < 4 containers with Runs (no
        # offset table): 20 keys alternating Run / Array, cut at containers 3 and 11 (2 ranks: at 5)
        one = np.concatenate([(k << 16) + (np.arange(100, 3000) if k % 2 else np.arange(0, 4000, 7))
                              for k in range(20)]).astype(np.uint32)
        ref = R.RefBitmap.of(one)
        ref.run_optimize()
        cuts = {2: [0, 5, 20], 3: [0, 3, 11, 20]}[world]
        v = ref.to_array()
        sub = R.RefBitmap.of(v[((v >> 16) >= cuts[rank]) & ((v >> 16) < cuts[rank + 1])])
        sub.run_optimize()
        summ = comm.summarize_serialized(sub.serialize())
        data = comm.gather_host(sub.serialize(), summ)
        if rank == 0:
            out["straddle"] = (data == ref.serialize(), summ["cardinality"] == ref.cardinality(),
                               summ["n_run_containers"] == 10)
        # one rank fails its argument checks: every rank fails the call together (no rank hangs)
        bad = rank == world - 1
        errs = []
        try:
            comm.summarize_serialized(None if bad else sub.serialize())
        except L.RbError as e:
            errs.append(type(e).__name__)
        try:  # the root's destination is too small: it fails, the others are told
            comm.gather_host(sub.serialize(), summ, root=0, cap=8 if rank == 0 else None)
        except L.RbError as e:
            errs.append(type(e).__name__)
        try:
            comm.naive_and_order(members, [1] * len(members), failed=bad)
        except L.RbError as e:
            errs.append(type(e).__name__)
        out[f"errors{rank}"] = errs
        sums = comm.allreduce_sum([rank + 1, 2**40])
        out[f"sum{rank}"] = list(sums) == [world * (world + 1) // 2, world * 2**40]
        if rank == 0:
            for r in range(1, world):  # every rank's error list at the root
                t = torch_obj_recv(dist, r)
                out.update(t)
            q.put(out)
        else:
            torch_obj_send(dist, {f"errors{rank}": errs, f"sum{rank}": out[f"sum{rank}"]})
    finally:
        if comm is not None:
            comm.close()
        dist.destroy_process_group()


def torch_obj_send(dist, obj):
    import json

    import torch
    b = json.dumps(obj).encode()
    dist.send(torch.tensor([len(b)], dtype=torch.int64), dst=0)
    dist.send(torch.frombuffer(bytearray(b), dtype=torch.uint8), dst=0)


def torch_obj_recv(dist, src):
    import json

    import torch
    n = torch.zeros(1, dtype=torch.int64)
    dist.recv(n, src=src)
    t = torch.zeros(int(n[0]), dtype=torch.uint8)
    dist.recv(t, src=src)
    return json.loads(bytes(t.numpy().tobytes()).decode())


@pytest.mark.parametrize("world", [2, 3])
def test_gloo_host_transport_exchange_in_c(world):
    out = _spawn(_rank_host_comm, world=world)
    for name in SEMS:
        assert all(out[name]), (name, out[name])
    assert all(out["straddle"]), out["straddle"]
    for r in range(world):
        assert out[f"sum{r}"], r
        errs = out[f"errors{r}"]
        # summarize (the last rank's null shard), gather (the root's small destination), naive_and order
        assert len(errs) == 3, (r, errs)


def _rank_host_comm_subgroup(rank, world, port, q):
    """a HostTransport over a non-default group maps the library's group-relative peers to the
    global ranks torch.distributed's send / recv take.  World 3, the group {1, 2}: global rank 1 is the
    group's root, so a gather with group-relative peers sent as global ones would reach rank 0 / hang."""
    import torch.distributed as dist

    from oracle import rbref as R
    from roaringbitmap_amd.engine import HostComm, HostTransport
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    comm = None
    try:
        grp = dist.new_group([1, 2])
        if rank == 0:
            q.put(torch_obj_recv(dist, 1))
            return
        comm = HostComm(HostTransport(dist, grp))
        one = np.concatenate([(k << 16) + (np.arange(100, 3000) if k % 2 else np.arange(0, 4000, 7))
                              for k in range(12)]).astype(np.uint32)
        ref = R.RefBitmap.of(one)
        ref.run_optimize()
        v = ref.to_array()
        lo, hi = (0, 5) if comm.rank == 0 else (5, 12)
        sub = R.RefBitmap.of(v[((v >> 16) >= lo) & ((v >> 16) < hi)])
        sub.run_optimize()
        summ = comm.summarize_serialized(sub.serialize())
        data = comm.gather_host(sub.serialize(), summ)
        if comm.rank == 0:
            torch_obj_send(dist, {"rank": rank, "group_rank": comm.rank, "world": comm.nranks,
                                  "ok": data == ref.serialize(), "card": summ["cardinality"] == ref.cardinality()})
    finally:
        if comm is not None:
            comm.close()
        dist.destroy_process_group()


def test_gloo_host_transport_subgroup():
    out = _spawn(_rank_host_comm_subgroup, world=3)
    assert out == {"rank": 1, "group_rank": 0, "world": 2, "ok": True, "card": True}

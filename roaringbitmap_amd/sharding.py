"""Key-range sharding of the wide aggregations across GPUs, one process per GPU.

Every high-16-bit key of FastAggregation / ParallelAggregation is independent and keeps its
member order inside a shard, so a contiguous key range per rank reproduces the single-GPU result
exactly (order-dependent semantics such as naive_xor included).  The data path has no
collective: each rank aggregates its own key range (rbgpu_wide_keys).  RCCL (torch.distributed
backend "nccl"; "gloo" on the CPU tests) carries only the exchange the result needs:

  1. all_gather of each rank's shard summary (cardinality, container count, Run-container count,
     payload bytes) -> the global cardinality (the reference's getCardinality) and everything a
     RoaringFormatSpec header over the concatenated shards needs (RoaringArray.java:851-940:
     container count, has-Run flag and per-container offsets, which depend on every earlier
     rank's payload bytes);
  2. on request, a gather of the shard containers to one rank, which writes the global bytes.

partition_keys() balances ranges by bytes (rbgpu_set_key_bytes), not by key count.
"""
from __future__ import annotations

import struct
from dataclasses import dataclass
from typing import List, Optional, Sequence, Tuple

import numpy as np

from . import _lib as L
from .engine import HostSoA

SERIAL_COOKIE_NO_RUNCONTAINER = 12346  # RoaringArray.java:43
SERIAL_COOKIE = 12347                  # RoaringArray.java:42
NO_OFFSET_THRESHOLD = 4                # RoaringArray.java:44


def _balanced_ranges(weights: np.ndarray, nparts: int) -> List[Tuple[int, int]]:
    """Contiguous [lo, hi) ranges covering [0, len(weights)) with near-equal weight totals.

    Range r ends at the first item where the running total reaches r/nparts of the whole, so every
    range holds at most one item's weight more than its share.  Ranges may be empty when a few items
    hold all the weight."""
    w = np.asarray(weights, dtype=np.float64)
    n = len(w)
    if nparts < 1:
        raise ValueError("nparts must be >= 1")
    csum = np.cumsum(w) if n else np.zeros(1)
    total = csum[-1]
    bounds = [0]
    for r in range(1, nparts):
        if total <= 0:
            b = (n * r) // nparts
        else:
            b = int(np.searchsorted(csum, total * r / nparts, side="left")) + 1
        bounds.append(min(max(b, bounds[-1]), n))
    bounds.append(n)
    return [(bounds[i], bounds[i + 1]) for i in range(nparts)]


def partition_keys(key_bytes: np.ndarray, nparts: int) -> List[Tuple[int, int]]:
    """Contiguous [lo, hi) high-key ranges covering [0, 65536) with near-equal byte totals."""
    kb = np.asarray(key_bytes)
    if kb.shape != (65536,):
        raise ValueError("key_bytes must have 65536 entries")
    return _balanced_ranges(kb, nparts)


def pair_bytes(a_bytes: np.ndarray, b_bytes: np.ndarray, a_idx: np.ndarray, b_idx: np.ndarray) -> np.ndarray:
    """Input payload bytes of each pair of a batch (the work a pair costs the HBM-bound kernels):
    a_bytes / b_bytes are per-bitmap payload bytes of the two sets (DeviceSet.summaries())."""
    return np.asarray(a_bytes, np.uint64)[np.asarray(a_idx, np.int64)] + \
        np.asarray(b_bytes, np.uint64)[np.asarray(b_idx, np.int64)]


def partition_pairs(bytes_per_pair: np.ndarray, nparts: int) -> List[Tuple[int, int]]:
    """Contiguous [lo, hi) ranges of one caller batch with near-equal input bytes: a rank computes
    its range of the pairs (results stay in batch order across ranks)."""
    return _balanced_ranges(bytes_per_pair, nparts)


def _payload_size(t: int, c: int, r: int) -> int:
    return 8192 if t == L.BITMAP else (2 * c if t == L.ARRAY else 2 + 4 * r)


def header_size(n: int, has_run: bool) -> int:
    """RoaringArray.headerSize (RoaringArray.java:781-790)."""
    if has_run:
        return 4 + (n + 7) // 8 + 4 * n + (4 * n if n >= NO_OFFSET_THRESHOLD else 0)
    return 8 + 8 * n


def serialize_parts(parts: Sequence[HostSoA], bitmap: int = 0) -> bytes:
    """RoaringFormatSpec bytes of one bitmap whose containers are spread over key-ordered parts
    (bitmap `bitmap` of each part): RoaringArray.serialize, RoaringArray.java:851-940."""
    keys, types, cards, runs, payloads = [], [], [], [], []
    last = -1
    for h in parts:
        for i in range(int(h.begin[bitmap]), int(h.begin[bitmap + 1])):
            k = int(h.key[i])
            if k <= last:
                raise ValueError("parts are not in increasing key order")
            last = k
            t, c, r = int(h.type[i]), int(h.card[i]), int(h.nruns[i])
            keys.append(k)
            types.append(t)
            cards.append(c)
            runs.append(r)
            p = h.container_payload(i)
            payloads.append(struct.pack("<H", r) + p.tobytes() if t == L.RUN else p.tobytes())
    n = len(keys)
    has_run = any(t == L.RUN for t in types)
    out = bytearray()
    if has_run:
        out += struct.pack("<I", SERIAL_COOKIE | ((n - 1) << 16))
        flags = bytearray((n + 7) // 8)
        for i, t in enumerate(types):
            if t == L.RUN:
                flags[i >> 3] |= 1 << (i & 7)
        out += flags
    else:
        out += struct.pack("<II", SERIAL_COOKIE_NO_RUNCONTAINER, n)
    for k, c in zip(keys, cards):
        out += struct.pack("<HH", k, c - 1)
    if not has_run or n >= NO_OFFSET_THRESHOLD:
        pos = header_size(n, has_run)
        for t, c, r in zip(types, cards, runs):
            out += struct.pack("<I", pos)
            pos += _payload_size(t, c, r)
    for p in payloads:
        out += p
    return bytes(out)


@dataclass
class ShardResult:
    """One rank's share of a sharded wide aggregation plus the global facts about the result."""
    local: object                 # DeviceSet (one bitmap: this rank's key range), or a HostSoA
    key_range: Tuple[int, int]
    cardinality: int              # of the whole result (all ranks)
    n_containers: int
    n_run_containers: int
    payload_bytes: int
    serialized_size: int          # RoaringBitmap.serializedSizeInBytes of the whole result
    payload_offset: int           # where this rank's first container payload starts in those bytes


def _gather_blobs(dist, rank: int, world: int, device, blobs: Sequence[bytes], dst: int) -> Optional[List[List[bytes]]]:
    """Every rank's byte strings on rank `dst` (None elsewhere), as tensors: an all_gather of the
    (count, bytes) sizes, then two tensor gathers (the lengths, the concatenated bytes), each padded
    to the largest rank's — no pickling."""
    import torch
    lens = np.array([len(b) for b in blobs], np.int64)
    sz = torch.tensor([len(blobs), int(lens.sum())], dtype=torch.int64, device=device)
    szs = [torch.zeros_like(sz) for _ in range(world)]
    dist.all_gather(szs, sz)
    g = torch.stack(szs).cpu().numpy()
    maxn, maxb = max(int(g[:, 0].max()), 1), max(int(g[:, 1].max()), 1)
    tl = torch.zeros(maxn, dtype=torch.int64, device=device)
    tl[:len(blobs)] = torch.from_numpy(lens).to(device)
    tb = torch.zeros(maxb, dtype=torch.uint8, device=device)
    if int(lens.sum()):
        tb[:int(lens.sum())] = torch.frombuffer(bytearray(b"".join(blobs)), dtype=torch.uint8).to(device)
    gl = [torch.empty_like(tl) for _ in range(world)] if rank == dst else None
    gb = [torch.empty_like(tb) for _ in range(world)] if rank == dst else None
    dist.gather(tl, gl, dst=dst)
    dist.gather(tb, gb, dst=dst)
    if rank != dst:
        return None
    out = []
    for r in range(world):
        ln = gl[r].cpu().numpy()[:int(g[r, 0])]
        data = gb[r].cpu().numpy().tobytes()
        offs = np.concatenate([[0], np.cumsum(ln)])
        out.append([data[int(offs[i]):int(offs[i + 1])] for i in range(len(ln))])
    return out


class ShardedWide:
    """Key-range-sharded FastAggregation / ParallelAggregation over torch.distributed.

    `compute(sem, key_range)` may be replaced (tests drive the collective logic on CPU with gloo);
    by default it is Context.wide(sem, dset, members, key_range) on this rank's MI355X."""

    def __init__(self, dist, rank: int, world: int, device=None):
        self.dist, self.rank, self.world = dist, rank, world
        self.device = device  # torch device for collective tensors (cuda for nccl, cpu for gloo)

    def _all_gather_i64(self, vals: Sequence[int]) -> np.ndarray:
        import torch
        t = torch.tensor(list(vals), dtype=torch.int64, device=self.device)
        out = [torch.zeros_like(t) for _ in range(self.world)]
        self.dist.all_gather(out, t)
        return torch.stack(out).cpu().numpy()

    def finish(self, local, key_range: Tuple[int, int], summary: dict) -> ShardResult:
        """Exchange step: all_gather of the shard summaries -> global metadata."""
        g = self._all_gather_i64([summary["cardinality"], summary["n_containers"], summary["n_run_containers"],
                                  summary["payload_bytes"]])
        n = int(g[:, 1].sum())
        has_run = bool(g[:, 2].sum() > 0)
        hdr = header_size(n, has_run) if n else header_size(0, False)
        before = int(g[:self.rank, 3].sum())
        return ShardResult(local, key_range, int(g[:, 0].sum()), n, int(g[:, 2].sum()), int(g[:, 3].sum()),
                           hdr + int(g[:, 3].sum()), hdr + before)

    def naive_and_order(self, counts: Sequence[int], members: Sequence[int]) -> List[int]:
        """FastAggregation.naive_and(varargs)'s fold order (FastAggregation.java:328-346): the bitmap
        with the fewest containers (first on ties), then the others in order, skipping it by
        identity.  Container counts are global, so this rank's key-range counts are summed over the
        ranks (an all_reduce) — every shard then folds the same order as the unsharded call."""
        import torch
        t = torch.tensor([int(c) for c in counts], dtype=torch.int64, device=self.device)
        self.dist.all_reduce(t)
        tot = t.cpu().numpy()
        if len(members) == 0:
            return []
        sm = members[int(np.argmin(tot))]  # argmin: the first minimal one
        return [sm] + [m for m in members if m != sm]

    def check_semantics(self, sem: int) -> None:
        """priorityqueue_or / _xor merge in the order of intermediate result sizes, which are global:
        a key-range shard cannot follow it.  Every rank raises alike (the arguments agree), before any
        collective, as rbgpu_wide_sharded refuses them."""
        if self.world > 1 and sem in L.PQ_SEMS:
            raise ValueError("priorityqueue_or / priorityqueue_xor cannot be key-range sharded")

    def aggregate(self, ctx, sem: int, dset, key_range: Tuple[int, int], members=None) -> ShardResult:
        self.check_semantics(sem)
        mem = list(range(len(dset))) if members is None else [int(m) for m in members]
        if sem == L.NAIVE_AND or (sem == L.FAST_AND and len(mem) <= 10):
            order = self.naive_and_order(dset.range_counts(mem, key_range), mem)
            local = ctx.wide(L.NAIVE_AND_ITER, dset, order, key_range=key_range)
        else:
            local = ctx.wide(sem, dset, members, key_range=key_range)
        return self.finish(local, key_range, local.summaries()[0])

    def gather_serialized(self, res: ShardResult, dst: int = 0) -> Optional[bytes]:
        """Global RoaringFormatSpec bytes on rank `dst` (None elsewhere): each shard serialized on its
        rank, the bytes gathered as tensors, the header of the concatenation assembled by the
        library (rbgpu_shard_assemble_host)."""
        from .engine import assemble_host
        mine = serialize_parts([res.local]) if isinstance(res.local, HostSoA) else res.local.serialize()[0]
        parts = _gather_blobs(self.dist, self.rank, self.world, self.device, [mine], dst)
        if parts is None:
            return None
        return assemble_host([p[0] for p in parts])


class ShardedBsi(ShardedWide):
    """Key-range-sharded Roaring64BitmapSliceIndex.compare.

    The O'Neil comparison is key-local: every 2^16-row chunk (high key) of the answer depends only
    on the slices' and ebM's containers of that key, the way the reference already splits the work
    (BitSliceIndexBase.java:99-166 partitions the foundSet by high key for its thread pool).  Rank r
    holds the slices and ebM of its key range (rbgpu_generate_bsi_keys, or any BSI set: keys outside
    the range are ignored) and computes that range of the answer (rbgpu_bsi_compare_keys); the
    exchange is ShardedWide's: an all_gather of the shard summaries (global cardinality = the
    reference's getCardinality of the answer, serialized size) and, on request, the gather of the
    shards to one rank."""

    def compare(self, ctx, op: int, bsi, start: int, end: int, min_value: int, max_value: int,
                key_range: Tuple[int, int], found=None) -> ShardResult:
        local = ctx.bsi_compare(op, bsi, start, end, min_value, max_value, found, key_range=key_range)
        return self.finish(local, key_range, local.summaries()[0])


@dataclass
class PairShardResult:
    """One rank's share of a pair-sharded batch plus the global facts about the results."""
    local: object                 # DeviceSet of this rank's results (pairs [lo, hi) in order), or HostSoA
    pair_range: Tuple[int, int]
    cardinality: int              # sum of every result's cardinality over all ranks
    n_containers: int
    payload_bytes: int


class ShardedPairwise:
    """One caller batch of (a[i], b[i]) pairs split across ranks by input bytes (partition_pairs).

    Pairs are independent (RoaringBitmap.and/or/xor/andNot of two bitmaps), so the data path has no
    collective; the exchange is one all_reduce of (result cardinality, containers, payload bytes) —
    the batch's total cardinality, which the reference's callers get by summing
    getCardinality / andCardinality — and, on request, the gather of the serialized results to one
    rank in batch order."""

    def __init__(self, dist, rank: int, world: int, device=None):
        self.dist, self.rank, self.world = dist, rank, world
        self.device = device

    def split(self, bytes_per_pair: np.ndarray) -> Tuple[int, int]:
        return partition_pairs(bytes_per_pair, self.world)[self.rank]

    def finish(self, local, pair_range: Tuple[int, int], cardinality: int, n_containers: int,
               payload_bytes: int) -> PairShardResult:
        import torch
        t = torch.tensor([cardinality, n_containers, payload_bytes], dtype=torch.int64, device=self.device)
        self.dist.all_reduce(t)
        g = t.cpu().tolist()
        return PairShardResult(local, pair_range, int(g[0]), int(g[1]), int(g[2]))

    def run(self, ctx, op: int, a, b, a_idx: np.ndarray, b_idx: np.ndarray, bytes_per_pair=None) -> PairShardResult:
        """This rank's pairs of the batch on its MI355X (rbgpu_pairwise) + the exchange."""
        if bytes_per_pair is None:
            pa = np.array([s["payload_bytes"] for s in a.summaries()], np.uint64)
            pb = pa if b is a else np.array([s["payload_bytes"] for s in b.summaries()], np.uint64)
            bytes_per_pair = pair_bytes(pa, pb, a_idx, b_idx)
        lo, hi = self.split(bytes_per_pair)
        ai = np.ascontiguousarray(a_idx[lo:hi], np.uint32)
        bi = np.ascontiguousarray(b_idx[lo:hi], np.uint32)
        local = ctx.pairwise(op, a, b, ai, bi)
        st = ctx.stats()
        # output_bytes counts 16 B of metadata per result container beside the payloads
        return self.finish(local, (lo, hi), st["result_cardinality"], st["result_containers"],
                           st["output_bytes"] - 16 * st["result_containers"])

    def gather_serialized(self, res: PairShardResult, dst: int = 0) -> Optional[List[bytes]]:
        """Every result's RoaringFormatSpec bytes, in batch order, on rank `dst` (None elsewhere)."""
        mine = res.local.serialize() if hasattr(res.local, "serialize") else list(res.local)
        parts = _gather_blobs(self.dist, self.rank, self.world, self.device, mine, dst)
        if parts is None:
            return None
        return [x for p in parts for x in p]

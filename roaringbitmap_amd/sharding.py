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


def partition_keys(key_bytes: np.ndarray, nparts: int) -> List[Tuple[int, int]]:
    """Contiguous [lo, hi) ranges covering [0, 65536) with near-equal byte totals.

    Range r ends at the first key where the running byte total reaches r/nparts of the whole, so
    every range holds at most one key's bytes more than its share.  Ranges may be empty when a few
    keys hold all the bytes."""
    kb = np.asarray(key_bytes, dtype=np.float64)
    if kb.shape != (65536,):
        raise ValueError("key_bytes must have 65536 entries")
    if nparts < 1:
        raise ValueError("nparts must be >= 1")
    csum = np.cumsum(kb)
    total = csum[-1]
    bounds = [0]
    for r in range(1, nparts):
        if total <= 0:
            b = (65536 * r) // nparts
        else:
            b = int(np.searchsorted(csum, total * r / nparts, side="left")) + 1
        bounds.append(min(max(b, bounds[-1]), 65536))
    bounds.append(65536)
    return [(bounds[i], bounds[i + 1]) for i in range(nparts)]


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

    def aggregate(self, ctx, sem: int, dset, key_range: Tuple[int, int], members=None) -> ShardResult:
        local = ctx.wide(sem, dset, members, key_range=key_range)
        return self.finish(local, key_range, local.summaries()[0])

    def gather_serialized(self, res: ShardResult, dst: int = 0) -> Optional[bytes]:
        """Global RoaringFormatSpec bytes on rank `dst` (None elsewhere)."""
        h = res.local if isinstance(res.local, HostSoA) else res.local.download()
        parts: List[Optional[HostSoA]] = [None] * self.world if self.rank == dst else None
        self.dist.gather_object(h, parts, dst=dst)
        if self.rank != dst:
            return None
        return serialize_parts(parts)

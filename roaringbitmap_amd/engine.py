"""Device-resident engine objects over the C ABI: Context (one HIP stream + workspaces on
one MI355X) and DeviceSet (a batch of bitmaps in SoA form in HBM).

Host SoA helpers build canonical containers from values the way the reference does
(RoaringBitmap.bitmapOf: ArrayContainer up to 4096 values, BitmapContainer beyond,
RoaringBitmap.java:498-570; runOptimize rules ArrayContainer.java:1085-1099,
BitmapContainer.java:1227-1246).
"""
from __future__ import annotations

import ctypes as C
from dataclasses import dataclass, field
from typing import List, Optional, Sequence, Tuple

import numpy as np

from . import _lib as L


@dataclass
class HostSoA:
    """A batch of bitmaps on the host, same layout as rb_soa."""
    begin: np.ndarray                       # uint64 [nb+1]
    key: np.ndarray                         # uint16 [nc]
    type: np.ndarray                        # uint8  [nc]
    card: np.ndarray                        # uint32 [nc]
    nruns: np.ndarray                       # uint16 [nc]
    offset: np.ndarray                      # uint64 [nc]
    payload: np.ndarray = field(repr=False)  # uint8

    @property
    def n_bitmaps(self) -> int:
        return len(self.begin) - 1

    @property
    def n_containers(self) -> int:
        return len(self.key)

    def container_payload(self, i: int) -> np.ndarray:
        t, c, r = int(self.type[i]), int(self.card[i]), int(self.nruns[i])
        n = 8192 if t == L.BITMAP else (2 * c if t == L.ARRAY else 4 * r)
        o = int(self.offset[i])
        return self.payload[o:o + n]

    def values(self, b: int) -> np.ndarray:
        """All uint32 values of bitmap b (ascending)."""
        out = []
        for i in range(int(self.begin[b]), int(self.begin[b + 1])):
            hi = np.uint32(int(self.key[i]) << 16)
            p = self.container_payload(i)
            t = int(self.type[i])
            if t == L.ARRAY:
                low = p.view(np.uint16).astype(np.uint32)
            elif t == L.BITMAP:
                bits = np.unpackbits(p, bitorder="little")
                low = np.nonzero(bits)[0].astype(np.uint32)
            else:
                rl = p.view(np.uint16).reshape(-1, 2).astype(np.uint32)
                low = np.concatenate([np.arange(s, s + l + 1, dtype=np.uint32) for s, l in rl]) if len(rl) else \
                    np.zeros(0, np.uint32)
            out.append(low | hi)
        return np.concatenate(out) if out else np.zeros(0, np.uint32)

    def as_rb_soa(self) -> L.RbSoa:
        s = L.RbSoa()
        s.n_bitmaps = self.n_bitmaps
        s.n_containers = self.n_containers
        s.payload_bytes = len(self.payload)
        for name in ("begin", "key", "type", "card", "nruns", "offset", "payload"):
            arr = getattr(self, name)
            assert arr.flags["C_CONTIGUOUS"]
            setattr(s, name, arr.ctypes.data if arr.size else None)
        return s


def _runs_of_sorted(low: np.ndarray):
    if len(low) == 0:
        return np.zeros((0, 2), np.uint16)
    brk = np.nonzero(np.diff(low.astype(np.int64)) != 1)[0]
    starts = np.concatenate([[0], brk + 1])
    ends = np.concatenate([brk, [len(low) - 1]])
    s = low[starts].astype(np.uint32)
    e = low[ends].astype(np.uint32)
    return np.stack([s, e - s], axis=1).astype(np.uint16)


def soa_from_values(bitmaps: Sequence[np.ndarray], run_optimize: bool = False) -> HostSoA:
    """Canonical containers of each value list (bitmapOf semantics, optional runOptimize)."""
    begin = [0]
    key, typ, card, nruns, offset = [], [], [], [], []
    chunks = []
    pos = 0
    for vals in bitmaps:
        v = np.unique(np.asarray(vals, dtype=np.uint32))
        hi = (v >> 16).astype(np.uint16)
        lo = (v & 0xFFFF).astype(np.uint16)
        cuts = np.nonzero(np.diff(hi.astype(np.int64)))[0] + 1
        for part_hi, part_lo in zip(np.split(hi, cuts), np.split(lo, cuts)):
            if len(part_lo) == 0:
                continue
            c = len(part_lo)
            runs = _runs_of_sorted(part_lo)
            r = len(runs)
            t = L.ARRAY if c <= 4096 else L.BITMAP
            if run_optimize:
                if t == L.ARRAY and 2 * c > 2 + 4 * r:
                    t = L.RUN
                elif t == L.BITMAP and 8192 > 2 + 4 * r:
                    t = L.RUN
            if t == L.ARRAY:
                data = part_lo.tobytes()
            elif t == L.BITMAP:
                bits = np.zeros(65536, np.uint8)
                bits[part_lo] = 1
                data = np.packbits(bits, bitorder="little").tobytes()
            else:
                data = runs.tobytes()
            key.append(int(part_hi[0]))
            typ.append(t)
            card.append(c)
            nruns.append(r if t == L.RUN else 0)
            offset.append(pos)
            pad = (-len(data)) % 16
            chunks.append(data + b"\0" * pad)
            pos += len(data) + pad
        begin.append(len(key))
    payload = np.frombuffer(b"".join(chunks) or b"\0" * 16, dtype=np.uint8).copy()
    return HostSoA(np.array(begin, np.uint64), np.array(key, np.uint16), np.array(typ, np.uint8),
                   np.array(card, np.uint32), np.array(nruns, np.uint16), np.array(offset, np.uint64), payload)


def soa_from_serialized(blobs: Sequence[bytes]) -> HostSoA:
    """Host SoA of RoaringFormatSpec bitmaps, container types as stored (the layout that
    RoaringArray.deserialize reads, RoaringArray.java:276-348).  A host-side helper for splitting
    and re-assembling shards; device uploads go through rbgpu_set_from_serialized, which also
    validates."""
    import struct
    begin, key, typ, card, nruns, offset, chunks = [0], [], [], [], [], [], []
    pos = 0
    for data in blobs:
        cookie = struct.unpack_from("<I", data, 0)[0]
        if (cookie & 0xFFFF) == 12347:
            n = (cookie >> 16) + 1
            flags = data[4:4 + (n + 7) // 8]
            p = 4 + (n + 7) // 8
            is_run = [bool(flags[i >> 3] >> (i & 7) & 1) for i in range(n)]
            has_offsets = n >= 4
        elif cookie == 12346:
            n = struct.unpack_from("<I", data, 4)[0]
            p = 8
            is_run = [False] * n
            has_offsets = True
        else:
            raise L.FormatError(L.RB_EFORMAT, "bad cookie")
        desc = np.frombuffer(data, np.uint16, 2 * n, p).reshape(-1, 2)
        p += 4 * n + (4 * n if has_offsets else 0)
        for i in range(n):
            c = int(desc[i, 1]) + 1
            if is_run[i]:
                r = struct.unpack_from("<H", data, p)[0]
                raw, t, p = data[p + 2:p + 2 + 4 * r], L.RUN, p + 2 + 4 * r
            elif c > 4096:
                raw, t, r, p = data[p:p + 8192], L.BITMAP, 0, p + 8192
            else:
                raw, t, r, p = data[p:p + 2 * c], L.ARRAY, 0, p + 2 * c
            key.append(int(desc[i, 0]))
            typ.append(t)
            card.append(c)
            nruns.append(r)
            offset.append(pos)
            pad = (-len(raw)) % 16
            chunks.append(bytes(raw) + b"\0" * pad)
            pos += len(raw) + pad
        begin.append(len(key))
    payload = np.frombuffer(b"".join(chunks) or b"\0" * 16, dtype=np.uint8).copy()
    return HostSoA(np.array(begin, np.uint64), np.array(key, np.uint16), np.array(typ, np.uint8),
                   np.array(card, np.uint32), np.array(nruns, np.uint16), np.array(offset, np.uint64), payload)


def host_summary(h: HostSoA, b: int = 0) -> dict:
    """rb_bitmap_summary of bitmap b of a host SoA (cf. DeviceSet.summaries)."""
    lo, hi = int(h.begin[b]), int(h.begin[b + 1])
    t, c, r = h.type[lo:hi].astype(np.int64), h.card[lo:hi].astype(np.int64), h.nruns[lo:hi].astype(np.int64)
    pay = np.where(t == L.BITMAP, 8192, np.where(t == L.ARRAY, 2 * c, 2 + 4 * r))
    return {"cardinality": int(c.sum()), "n_containers": hi - lo, "n_run_containers": int((t == L.RUN).sum()),
            "payload_bytes": int(pay.sum())}


class DeviceSet:
    """A batch of bitmaps resident in HBM (rbgpu_set*).  Freed on close() / GC."""

    def __init__(self, ctx: "Context", handle: int):
        self.ctx = ctx
        self.h = C.c_void_p(handle)

    def close(self):
        if self.h and self.h.value:
            L.lib().rbgpu_set_free(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def __len__(self) -> int:
        return int(L.lib().rbgpu_set_bitmap_count(self.h))

    @property
    def n_containers(self) -> int:
        return int(L.lib().rbgpu_set_container_count(self.h))

    @property
    def payload_capacity(self) -> int:
        """rbgpu_set_payload_capacity: bytes of the HBM payload arena (16-B padded payloads)."""
        return int(L.lib().rbgpu_set_payload_capacity(self.h))

    def run_optimize(self):
        """RoaringBitmap.runOptimize of every bitmap on the device (rbgpu_set_run_optimize): the new set
        and, per bitmap, runOptimize's return value (it holds a Run container)."""
        out = C.c_void_p()
        flags = np.zeros(max(len(self), 1), np.uint8)
        L.check(L.lib().rbgpu_set_run_optimize(self.h, C.byref(out), flags.ctypes.data))
        return DeviceSet(self.ctx, out.value), flags[:len(self)].astype(bool)

    def cardinalities(self) -> np.ndarray:
        out = np.zeros(len(self), np.uint64)
        L.check(L.lib().rbgpu_set_cardinalities(self.h, out.ctypes.data_as(L._U64P)))
        return out

    def serialized_sizes(self) -> np.ndarray:
        out = np.zeros(len(self), np.uint64)
        L.check(L.lib().rbgpu_set_serialized_sizes(self.h, out.ctypes.data_as(L._U64P)))
        return out

    def summaries(self, first: int = 0, count: Optional[int] = None) -> List[dict]:
        """Per-bitmap cardinality / container counts / payload bytes (rbgpu_set_summaries)."""
        count = len(self) - first if count is None else count
        arr = (L.RbBitmapSummary * max(count, 1))()
        L.check(L.lib().rbgpu_set_summaries(self.h, first, count, arr))
        return [{k: int(getattr(arr[i], k)) for k, _ in L.RbBitmapSummary._fields_} for i in range(count)]

    def type_stats(self) -> dict:
        """Container mix (rbgpu_set_type_stats): counts and serialized payload bytes per type."""
        out = np.zeros(6, np.uint64)
        L.check(L.lib().rbgpu_set_type_stats(self.h, out.ctypes.data_as(L._U64P)))
        return {"array": int(out[0]), "bitmap": int(out[1]), "run": int(out[2]),
                "array_bytes": int(out[3]), "bitmap_bytes": int(out[4]), "run_bytes": int(out[5])}

    def key_bytes(self) -> np.ndarray:
        """Algorithmic bytes per high key (rbgpu_set_key_bytes), shape [65536]."""
        out = np.zeros(65536, np.uint64)
        L.check(L.lib().rbgpu_set_key_bytes(self.h, out.ctypes.data_as(L._U64P)))
        return out

    def range_counts(self, members=None, key_range: Tuple[int, int] = (0, 65536)) -> np.ndarray:
        """Containers of each member with high key in key_range (rbgpu_set_range_counts)."""
        m = None if members is None else np.ascontiguousarray(members, dtype=np.uint32)
        n = len(self) if m is None else len(m)
        out = np.zeros(n, np.uint64)
        L.check(L.lib().rbgpu_set_range_counts(self.h, None if m is None else m.ctypes.data_as(L._U32P), n,
                                               int(key_range[0]), int(key_range[1]), out.ctypes.data_as(L._U64P)))
        return out

    def serialize(self, first: int = 0, count: Optional[int] = None) -> List[bytes]:
        count = len(self) - first if count is None else count
        if count == 0:
            return []
        sizes = self.serialized_sizes()[first:first + count]
        total = int(sizes.sum())
        buf = C.create_string_buffer(max(total, 1))
        offs = np.zeros(count + 1, np.uint64)
        L.check(L.lib().rbgpu_set_serialize(self.h, first, count, buf, total, offs.ctypes.data_as(L._U64P)))
        raw = buf.raw
        return [raw[int(offs[i]):int(offs[i + 1])] for i in range(count)]

    def serialize_device(self, dst_ptr: int, cap: int, first: int = 0, count: Optional[int] = None) -> np.ndarray:
        """RoaringFormatSpec bytes of bitmaps [first, first+count) written by the GPU into device memory
        at dst_ptr (rbgpu_set_serialize_device); returns the count+1 byte offsets."""
        count = len(self) - first if count is None else count
        offs = np.zeros(count + 1, np.uint64)
        L.check(L.lib().rbgpu_set_serialize_device(self.h, first, count, C.c_void_p(dst_ptr), cap,
                                                    offs.ctypes.data_as(L._U64P)))
        return offs

    def device_view(self) -> dict:
        """rbgpu_set_device_view: device addresses of the SoA (never blocks; n_containers is None while an
        asynchronous result is pending)."""
        v = L.RbDeviceView()
        L.check(L.lib().rbgpu_set_device_view(self.h, C.byref(v)))
        d = {f: getattr(v, f) or 0 for f, _ in L.RbDeviceView._fields_}
        if d["n_containers"] == L.UNKNOWN_COUNT:
            d["n_containers"] = None
        return d

    def wait(self) -> "DeviceSet":
        """rbgpu_set_wait: an asynchronous result complete (no-op otherwise)."""
        L.check(L.lib().rbgpu_set_wait(self.h))
        return self

    def setup_stats(self) -> dict:
        """rbgpu_set_setup_stats: device ms and algorithmic bytes of the derived per-set metadata so far."""
        ms, b = C.c_double(), C.c_uint64()
        L.check(L.lib().rbgpu_set_setup_stats(self.h, C.byref(ms), C.byref(b)))
        return {"ms": round(ms.value, 4), "bytes": int(b.value)}

    def setup_parts(self) -> dict:
        """rbgpu_set_setup_parts: {item: {ms, bytes}} for the dense check, mrec, krec and the BSI key tables
        built so far."""
        ms, b = (C.c_double * 4)(), np.zeros(4, np.uint64)
        L.check(L.lib().rbgpu_set_setup_parts(self.h, ms, b.ctypes.data_as(L._U64P)))
        return {k: {"ms": round(ms[i], 4), "bytes": int(b[i])}
                for i, k in enumerate(("dense_check", "mrec", "krec", "bsi_tables"))}

    def download(self, first: int = 0, count: Optional[int] = None) -> HostSoA:
        count = len(self) - first if count is None else count
        q = L.RbSoa()
        L.check(L.lib().rbgpu_set_download(self.h, first, count, C.byref(q)))
        nc, nbytes = int(q.n_containers), int(q.payload_bytes)
        h = HostSoA(np.zeros(count + 1, np.uint64), np.zeros(nc, np.uint16), np.zeros(nc, np.uint8),
                    np.zeros(nc, np.uint32), np.zeros(nc, np.uint16), np.zeros(nc, np.uint64),
                    np.zeros(max(nbytes, 16), np.uint8))
        s = h.as_rb_soa()
        s.n_containers, s.payload_bytes = max(nc, 0), len(h.payload)
        if nc == 0:  # still need a non-null key pointer to mean "fill"
            h.begin[:] = 0
            return h
        L.check(L.lib().rbgpu_set_download(self.h, first, count, C.byref(s)))
        return h


def _idx(arr):
    if arr is None:
        return None, None
    a = np.ascontiguousarray(np.asarray(arr, dtype=np.uint32))
    return a, a.ctypes.data_as(L._U32P)


def _idx_addr(arr):
    """(array, address) of a u32 index array — the address as a plain int for void* parameters (the
    ctypes pointer object costs ~2 us per call; small-batch calls take tens of microseconds)."""
    if arr is None:
        return None, None
    a = arr if (type(arr) is np.ndarray and arr.dtype == np.uint32 and arr.flags.c_contiguous) else \
        np.ascontiguousarray(arr, dtype=np.uint32)
    return a, a.__array_interface__["data"][0]


def stats_dict(s: "L.RbStats") -> dict:
    """rb_stats as a dict: the scalar fields, main_kernel, and one entry per timed kernel span."""
    out = {k: getattr(s, k) for k, _ in s._fields_ if not k.startswith("kernel_")}
    out["main_kernel"] = s.main_kernel.decode()
    out["kernels"] = [{"name": s.kernel_name[i].value.decode(), "ms": s.kernel_ms[i],
                       "bytes": int(s.kernel_bytes[i]), "items": int(s.kernel_items[i])}
                      for i in range(s.n_kernels)]
    return out


class Context:
    """One MI355X: a HIP stream, workspaces and an allocation cache (rbgpu_ctx*)."""

    def __init__(self, device: int = 0):
        h = C.c_void_p()
        L.check(L.lib().rbgpu_open(device, C.byref(h)))
        self.h = h
        self.device = device

    def close(self):
        if self.h and self.h.value:
            L.lib().rbgpu_close(self.h)
            self.h = None

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.close()

    @staticmethod
    def device_count() -> int:
        return int(L.lib().rbgpu_device_count())

    def synchronize(self):
        L.check(L.lib().rbgpu_synchronize(self.h))

    def stats(self) -> dict:
        return stats_dict(self.stats_raw())

    def stats_raw(self) -> "L.RbStats":
        """The last call's rb_stats as the ctypes struct (rbgpu_get_stats), for loops that convert it
        later (`stats_dict`) rather than build a dict per call."""
        s = L.RbStats()
        L.check(L.lib().rbgpu_get_stats(self.h, C.byref(s)))
        return s

    # ---- sets
    def upload_serialized(self, blobs: Sequence[bytes]) -> DeviceSet:
        n = len(blobs)
        arr = (C.c_char_p * max(n, 1))(*blobs)
        lens = np.array([len(b) for b in blobs] or [0], np.uint64)
        out = C.c_void_p()
        L.check(L.lib().rbgpu_set_from_serialized(self.h, arr, lens.ctypes.data_as(L._U64P), n, C.byref(out)))
        return DeviceSet(self, out.value)

    def upload_serialized_device(self, src_ptr: int, offsets: np.ndarray) -> DeviceSet:
        """Bitmaps already serialized in device memory at src_ptr, bitmap i at [offsets[i], offsets[i+1])
        (rbgpu_set_from_serialized_device): parsed and validated on the GPU."""
        offs = np.ascontiguousarray(offsets, np.uint64)
        out = C.c_void_p()
        L.check(L.lib().rbgpu_set_from_serialized_device(self.h, C.c_void_p(src_ptr), offs.ctypes.data_as(L._U64P),
                                                          len(offs) - 1, C.byref(out)))
        return DeviceSet(self, out.value)

    def upload_soa(self, soa: HostSoA) -> DeviceSet:
        s = soa.as_rb_soa()
        out = C.c_void_p()
        L.check(L.lib().rbgpu_set_from_soa(self.h, C.byref(s), C.byref(out)))
        return DeviceSet(self, out.value)

    def upload_values(self, bitmaps: Sequence[np.ndarray], run_optimize: bool = False) -> DeviceSet:
        return self.upload_soa(soa_from_values(bitmaps, run_optimize))

    def generate_keys(self, workload: int, n: int, key_lo: int, key_hi: int, seed: int = 42) -> DeviceSet:
        """The [key_lo, key_hi) shard of a wide synthetic workload (rbgpu_generate_keys)."""
        a = C.c_void_p()
        L.check(L.lib().rbgpu_generate_keys(self.h, workload, n, seed, key_lo, key_hi, C.byref(a)))
        return DeviceSet(self, a.value)

    def generate(self, workload: int, n: int, seed: int = 42):
        a, b = C.c_void_p(), C.c_void_p()
        L.check(L.lib().rbgpu_generate(self.h, workload, n, seed, C.byref(a), C.byref(b)))
        return DeviceSet(self, a.value), (DeviceSet(self, b.value) if b.value else None)

    # ---- algebra
    def pairwise(self, op: int, a: DeviceSet, b: DeviceSet, a_idx=None, b_idx=None, npairs=None) -> DeviceSet:
        ai, ap = _idx_addr(a_idx)
        bi, bp = _idx_addr(b_idx)
        n = npairs if npairs is not None else (len(ai) if ai is not None else min(len(a), len(b)))
        out = C.c_void_p()
        L.check(L.lib().rbgpu_pairwise(self.h, op, a.h, b.h, ap, bp, n, C.byref(out)))
        return DeviceSet(self, out.value)

    # ---- 64-bit bitmaps (longlong/)
    def upload_portable64(self, blobs: Sequence[bytes]) -> "DeviceSet64":
        """Roaring64NavigableMap.deserializePortable per blob (rbgpu_set64_from_portable)."""
        n = len(blobs)
        arr = (C.c_char_p * max(n, 1))(*blobs)
        lens = np.array([len(b) for b in blobs] or [0], np.uint64)
        out = C.c_void_p()
        L.check(L.lib().rbgpu_set64_from_portable(self.h, arr, lens.ctypes.data_as(L._U64P), n, C.byref(out)))
        return DeviceSet64(self, out.value)

    def upload_legacy64(self, blobs: Sequence[bytes]) -> "DeviceSet64":
        """Roaring64NavigableMap.deserializeLegacy per blob (rbgpu_set64_from_legacy): the signedLongs
        flag travels with each bitmap."""
        n = len(blobs)
        arr = (C.c_char_p * max(n, 1))(*blobs)
        lens = np.array([len(b) for b in blobs] or [0], np.uint64)
        out = C.c_void_p()
        L.check(L.lib().rbgpu_set64_from_legacy(self.h, arr, lens.ctypes.data_as(L._U64P), n, C.byref(out)))
        return DeviceSet64(self, out.value)

    def upload_art64(self, blobs: Sequence[bytes]) -> "DeviceSet64":
        """Roaring64Bitmap.deserialize per blob (rbgpu_set64_from_art: the ART + Containers stream)."""
        n = len(blobs)
        arr = (C.c_char_p * max(n, 1))(*blobs)
        lens = np.array([len(b) for b in blobs] or [0], np.uint64)
        out = C.c_void_p()
        L.check(L.lib().rbgpu_set64_from_art(self.h, arr, lens.ctypes.data_as(L._U64P), n, C.byref(out)))
        return DeviceSet64(self, out.value)

    def pairwise64_cardinality(self, op: int, a: "DeviceSet64", b: "DeviceSet64", a_idx=None, b_idx=None,
                               npairs=None) -> np.ndarray:
        """rbgpu_pairwise64_cardinality: the static op's getLongCardinality per pair (Roaring64Bitmap.
        andCardinality for AND) without materialising the results."""
        ai, ap = _idx_addr(a_idx)
        bi, bp = _idx_addr(b_idx)
        n = npairs if npairs is not None else (len(ai) if ai is not None else min(len(a), len(b)))
        out = np.zeros(max(n, 1), np.uint64)
        L.check(L.lib().rbgpu_pairwise64_cardinality(self.h, op, a.h, b.h, ap, bp, n, out.ctypes.data_as(L._U64P)))
        return out[:n]

    def upload_values64(self, bitmaps: Sequence[np.ndarray]) -> "DeviceSet64":
        """bitmapOf(long...) per value list: buckets by the high 32 bits (rbgpu_set64_from_buckets)."""
        lows, highs, begin = [], [], [0]
        for vals in bitmaps:
            v = np.unique(np.asarray(vals, dtype=np.uint64))
            hi = (v >> np.uint64(32)).astype(np.uint32)
            for h in np.unique(hi):
                highs.append(int(h))
                lows.append((v[hi == h] & np.uint64(0xFFFFFFFF)).astype(np.uint32))
            begin.append(len(highs))
        bset = self.upload_values(lows) if lows else self.upload_values([])
        hs = np.array(highs or [0], np.uint32)
        bg = np.array(begin, np.uint64)
        out = C.c_void_p()
        L.check(L.lib().rbgpu_set64_from_buckets(bset.h, hs.ctypes.data_as(L._U32P), bg.ctypes.data_as(L._U64P),
                                                 len(bitmaps), C.byref(out)))
        return DeviceSet64(self, out.value)

    def pairwise64(self, flavor: int, op: int, a: "DeviceSet64", b: "DeviceSet64", a_idx=None, b_idx=None,
                   npairs=None, inplace: bool = False) -> "DeviceSet64":
        """rbgpu_pairwise64: Roaring64Bitmap (flavor RB64_BITMAP) static or in-place ops,
        Roaring64NavigableMap (RB64_NAVIGABLE) in-place ops, over a batch of pairs."""
        ai, ap = _idx_addr(a_idx)
        bi, bp = _idx_addr(b_idx)
        n = npairs if npairs is not None else (len(ai) if ai is not None else min(len(a), len(b)))
        out = C.c_void_p()
        L.check(L.lib().rbgpu_pairwise64(self.h, flavor, op, 1 if inplace else 0, a.h, b.h, ap, bp, n, C.byref(out)))
        return DeviceSet64(self, out.value)

    def pairwise_async(self, op: int, a: DeviceSet, b: DeviceSet, a_idx=None, b_idx=None, npairs=None,
                       stream: int = 0) -> DeviceSet:
        """rbgpu_pairwise_async: returns once the work is enqueued (stream: a hipStream_t address, 0 = the
        context's own); the result settles on first use or DeviceSet.wait()."""
        ai, ap = _idx_addr(a_idx)
        bi, bp = _idx_addr(b_idx)
        n = npairs if npairs is not None else (len(ai) if ai is not None else min(len(a), len(b)))
        out = C.c_void_p()
        L.check(L.lib().rbgpu_pairwise_async(self.h, op, a.h, b.h, ap, bp, n, C.c_void_p(stream or None),
                                             C.byref(out)))
        return DeviceSet(self, out.value)

    def pairwise_inplace(self, op: int, a: DeviceSet, b: DeviceSet, a_idx=None, b_idx=None,
                         npairs=None) -> DeviceSet:
        """result[i] = a[a_idx[i]] after the in-place a[a_idx[i]].op(b[b_idx[i]]) (rbgpu_pairwise_inplace:
        RoaringBitmap.and/or/xor/andNot(x2)); the inputs stay unchanged."""
        ai, ap = _idx_addr(a_idx)
        bi, bp = _idx_addr(b_idx)
        n = npairs if npairs is not None else (len(ai) if ai is not None else min(len(a), len(b)))
        out = C.c_void_p()
        L.check(L.lib().rbgpu_pairwise_inplace(self.h, op, a.h, b.h, ap, bp, n, C.byref(out)))
        return DeviceSet(self, out.value)

    def pairwise_cardinality(self, op: int, a: DeviceSet, b: DeviceSet, a_idx=None, b_idx=None,
                             npairs=None) -> np.ndarray:
        ai, ap = _idx_addr(a_idx)
        bi, bp = _idx_addr(b_idx)
        n = npairs if npairs is not None else (len(ai) if ai is not None else min(len(a), len(b)))
        out = np.zeros(max(n, 1), np.uint64)
        L.check(L.lib().rbgpu_pairwise_cardinality(self.h, op, a.h, b.h, ap, bp, n, out.ctypes.data_as(L._U64P)))
        return out[:n]

    def wide(self, sem: int, s: DeviceSet, members=None, key_range=None) -> DeviceSet:
        """FastAggregation / ParallelAggregation over members of s; key_range=(lo, hi) computes only
        that key-range shard (rbgpu_wide_keys)."""
        mi, mp = _idx(members)
        n = len(mi) if mi is not None else len(s)
        out = C.c_void_p()
        if key_range is None:
            L.check(L.lib().rbgpu_wide(self.h, sem, s.h, mp, n, C.byref(out)))
        else:
            lo, hi = key_range
            L.check(L.lib().rbgpu_wide_keys(self.h, sem, s.h, mp, n, int(lo), int(hi), C.byref(out)))
        return DeviceSet(self, out.value)

    def bsi_compare(self, op: int, bsi: DeviceSet, start: int, end: int, min_value: int, max_value: int,
                    found: Optional[DeviceSet] = None, key_range=None) -> DeviceSet:
        """Roaring64BitmapSliceIndex.compare over a device BSI (slices then ebM), rbgpu_bsi_compare;
        key_range=(lo, hi) computes only that key-range shard of the answer (rbgpu_bsi_compare_keys)."""
        out = C.c_void_p()
        lo, hi = key_range if key_range is not None else (0, 65536)
        L.check(L.lib().rbgpu_bsi_compare_keys(self.h, bsi.h, op, start & (2**64 - 1), end & (2**64 - 1),
                                               min_value & (2**64 - 1), max_value & (2**64 - 1),
                                               found.h if found is not None else None, int(lo), int(hi),
                                               C.byref(out)))
        return DeviceSet(self, out.value)

    def generate_bsi(self, nslices: int, nrows: int, seed: int = 42, key_range=None) -> DeviceSet:
        """The synthetic BSI of SURVEY §8d config 5, or its [lo, hi) key-range shard."""
        a = C.c_void_p()
        if key_range is None:
            L.check(L.lib().rbgpu_generate_bsi(self.h, nslices, nrows, seed, C.byref(a)))
        else:
            L.check(L.lib().rbgpu_generate_bsi_keys(self.h, nslices, nrows, seed, int(key_range[0]),
                                                    int(key_range[1]), C.byref(a)))
        return DeviceSet(self, a.value)

    def extract(self, s: DeviceSet, first: int, count: int = 1) -> DeviceSet:
        out = C.c_void_p()
        L.check(L.lib().rbgpu_set_extract(s.h, first, count, C.byref(out)))
        return DeviceSet(self, out.value)

    def wide_cardinality(self, op: int, s: DeviceSet, members=None) -> int:
        mi, mp = _idx(members)
        n = len(mi) if mi is not None else len(s)
        out = C.c_uint64()
        L.check(L.lib().rbgpu_wide_cardinality(self.h, op, s.h, mp, n, C.byref(out)))
        return int(out.value)


def _summary(s: L.RbShardSummary) -> dict:
    return {k: int(getattr(s, k)) for k, _ in L.RbShardSummary._fields_}


class Comm:
    """The library's RCCL communicator (rbgpu_comm): one rank per GPU; the shard exchange of the
    key-range-sharded aggregations runs inside librbgpu (include/rbgpu.h, multi-GPU section)."""

    @staticmethod
    def unique_id() -> bytes:
        buf = C.create_string_buffer(L.COMM_ID_BYTES)
        L.check(L.lib().rbgpu_comm_unique_id(buf))
        return buf.raw

    def __init__(self, ctx: "Context", uid: bytes, nranks: int, rank: int):
        if len(uid) != L.COMM_ID_BYTES:
            raise ValueError("communicator id must be 128 bytes")
        h = C.c_void_p()
        L.check(L.lib().rbgpu_comm_init(ctx.h, C.create_string_buffer(uid, L.COMM_ID_BYTES), nranks, rank,
                                        C.byref(h)))
        self.h, self.ctx, self.nranks, self.rank = h, ctx, nranks, rank

    def close(self):
        if self.h and self.h.value:
            L.lib().rbgpu_comm_destroy(self.h)
            self.h = None

    def allreduce_sum(self, values) -> np.ndarray:
        v = np.ascontiguousarray(np.asarray(values, dtype=np.uint64)).copy()
        L.check(L.lib().rbgpu_comm_allreduce_sum(self.h, v.ctypes.data_as(L._U64P), len(v)))
        return v

    def summarize(self, local: DeviceSet) -> dict:
        s = L.RbShardSummary()
        L.check(L.lib().rbgpu_shard_summarize(self.h, local.h, C.byref(s)))
        return _summary(s)

    def wide_sharded(self, sem: int, s: DeviceSet, key_range, members=None):
        mi, mp = _idx(members)
        n = len(mi) if mi is not None else len(s)
        out, summ = C.c_void_p(), L.RbShardSummary()
        L.check(L.lib().rbgpu_wide_sharded(self.h, sem, s.h, mp, n, int(key_range[0]), int(key_range[1]),
                                           C.byref(out), C.byref(summ)))
        return DeviceSet(self.ctx, out.value), _summary(summ)

    def bsi_compare_sharded(self, op: int, bsi: DeviceSet, start: int, end: int, min_value: int, max_value: int,
                            key_range, found: Optional[DeviceSet] = None):
        out, summ = C.c_void_p(), L.RbShardSummary()
        m = 2**64 - 1
        L.check(L.lib().rbgpu_bsi_compare_sharded(self.h, bsi.h, op, start & m, end & m, min_value & m, max_value & m,
                                                  found.h if found is not None else None, int(key_range[0]),
                                                  int(key_range[1]), C.byref(out), C.byref(summ)))
        return DeviceSet(self.ctx, out.value), _summary(summ)

    def gather_serialized(self, local: DeviceSet, summary: dict, root: int = 0) -> Optional[bytes]:
        """The whole result's RoaringFormatSpec bytes on `root` (None elsewhere), assembled on the
        root's GPU (rbgpu_shard_gather_serialized); the device buffer is a torch uint8 tensor."""
        import torch
        s = L.RbShardSummary(**summary)
        n = int(summary["serialized_size"]) if self.rank == root else 0
        buf = torch.empty(max(n, 16), dtype=torch.uint8, device=torch.device("cuda", self.ctx.device))
        L.check(L.lib().rbgpu_shard_gather_serialized(self.h, local.h, C.byref(s), root, C.c_void_p(buf.data_ptr()),
                                                      buf.numel()))
        if self.rank != root:
            return None
        return bytes(buf[:n].cpu().numpy().tobytes())


class HostTransport:
    """rb_host_transport over a torch.distributed process group (gloo on the CPU): the library's exchange
    code (summaries, failure agreement, naive_and's order, the shard gather, the header assembly) runs
    unchanged over it.  Keep the object alive as long as the communicator."""

    def __init__(self, dist, group=None):
        import torch
        self.dist, self.group = dist, group
        self.rank, self.world = dist.get_rank(group), dist.get_world_size(group)
        # the library numbers peers within the group; torch.distributed's send / recv take global ranks
        glob = (lambda p: p) if group is None else (lambda p: dist.get_global_rank(group, p))

        def all_gather(_user, send, recv, nbytes):
            try:
                n = int(nbytes)
                mine = torch.frombuffer(bytearray(C.string_at(send, n)), dtype=torch.uint8) if n else \
                    torch.zeros(0, dtype=torch.uint8)
                outs = [torch.zeros(n, dtype=torch.uint8) for _ in range(self.world)]
                dist.all_gather(outs, mine, group=group)
                if n:
                    C.memmove(recv, bytes(torch.cat(outs).numpy().tobytes()), n * self.world)
                return 0
            except Exception:  # noqa: BLE001 — a failure is reported to the library, not raised through C
                return 1

        def all_reduce(_user, values, n):
            try:
                v = np.ctypeslib.as_array(values, shape=(int(n),))
                t = torch.from_numpy(v.astype(np.int64))
                dist.all_reduce(t, group=group)
                v[:] = t.numpy().astype(np.uint64)
                return 0
            except Exception:  # noqa: BLE001
                return 1

        def send(_user, buf, nbytes, peer):
            try:
                dist.send(torch.frombuffer(bytearray(C.string_at(buf, int(nbytes))), dtype=torch.uint8), dst=glob(int(peer)),
                          group=group)
                return 0
            except Exception:  # noqa: BLE001
                return 1

        def recv(_user, buf, nbytes, peer):
            try:
                t = torch.zeros(int(nbytes), dtype=torch.uint8)
                dist.recv(t, src=glob(int(peer)), group=group)
                C.memmove(buf, bytes(t.numpy().tobytes()), int(nbytes))
                return 0
            except Exception:  # noqa: BLE001
                return 1

        self._cb = (L.HT_ALL_GATHER(all_gather), L.HT_ALL_REDUCE(all_reduce), L.HT_SEND(send), L.HT_RECV(recv))
        self.struct = L.RbHostTransport(None, self.world, self.rank, *self._cb)


class HostComm:
    """A communicator over a HostTransport (rbgpu_comm_init_host).  Without a device context only the
    byte-level exchange applies: a shard given as its serialized bytes (the CPU tests run the oracle's
    shards through the library's own exchange code this way)."""

    def __init__(self, transport: HostTransport, ctx: Optional["Context"] = None):
        h = C.c_void_p()
        L.check(L.lib().rbgpu_comm_init_host(ctx.h if ctx is not None else None, C.byref(transport.struct),
                                             C.byref(h)))
        self.h, self.t, self.ctx = h, transport, ctx
        self.rank, self.nranks = transport.rank, transport.world

    def close(self):
        if self.h and self.h.value:
            L.lib().rbgpu_comm_destroy(self.h)
            self.h = None

    def allreduce_sum(self, values) -> np.ndarray:
        v = np.ascontiguousarray(np.asarray(values, dtype=np.uint64)).copy()
        L.check(L.lib().rbgpu_comm_allreduce_sum(self.h, v.ctypes.data_as(L._U64P), len(v)))
        return v

    def summarize_serialized(self, shard: Optional[bytes]) -> dict:
        s = L.RbShardSummary()
        L.check(L.lib().rbgpu_shard_summarize_serialized(self.h, shard, len(shard) if shard else 0, C.byref(s)))
        return _summary(s)

    def gather_host(self, shard: Optional[bytes], summary: dict, root: int = 0, cap: Optional[int] = None):
        """The whole result's bytes on `root` (None elsewhere), through rbgpu_shard_gather_host."""
        s = L.RbShardSummary(**summary)
        n = int(summary["serialized_size"]) if self.rank == root else 0
        cap = n if cap is None else cap
        buf = C.create_string_buffer(max(cap, 1))
        L.check(L.lib().rbgpu_shard_gather_host(self.h, shard, len(shard) if shard else 0, C.byref(s), root, buf,
                                                cap))
        return buf.raw[:n] if self.rank == root else None

    def naive_and_order(self, members, local_counts, failed: bool = False) -> List[int]:
        m = np.ascontiguousarray(np.asarray(members, dtype=np.uint32))
        c = np.ascontiguousarray(np.asarray(local_counts, dtype=np.uint64))
        out = np.zeros(max(len(m), 1), np.uint32)
        k = C.c_uint32()
        L.check(L.lib().rbgpu_comm_naive_and_order(self.h, m.ctypes.data_as(L._U32P), c.ctypes.data_as(L._U64P),
                                                   len(m), 1 if failed else 0, out.ctypes.data_as(L._U32P),
                                                   C.byref(k)))
        return out[:k.value].tolist()


class DeviceSet64:
    """A batch of 64-bit bitmaps (rbgpu_set64*): buckets (high 32 bits, 32-bit bitmap) in HBM."""

    def __init__(self, ctx: "Context", handle: int):
        self.ctx = ctx
        self.h = C.c_void_p(handle)

    def close(self):
        if self.h and self.h.value:
            L.lib().rbgpu_set64_free(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def __len__(self) -> int:
        return int(L.lib().rbgpu_set64_bitmap_count(self.h))

    def cardinalities(self) -> np.ndarray:
        out = np.zeros(max(len(self), 1), np.uint64)
        L.check(L.lib().rbgpu_set64_cardinalities(self.h, out.ctypes.data_as(L._U64P)))
        return out[:len(self)]

    def highs(self, i: int) -> np.ndarray:
        cnt = C.c_uint64()
        L.check(L.lib().rbgpu_set64_buckets(self.h, i, None, 0, C.byref(cnt)))
        out = np.zeros(max(cnt.value, 1), np.uint32)
        L.check(L.lib().rbgpu_set64_buckets(self.h, i, out.ctypes.data_as(L._U32P), cnt.value, C.byref(cnt)))
        return out[:cnt.value]

    def bucket_set(self, i: int) -> "DeviceSet":
        """rbgpu_set64_bucket_set: bitmap i's buckets as a 32-bit set (bitmap k = bucket k), empty
        containers a Roaring64Bitmap keeps included."""
        out = C.c_void_p()
        L.check(L.lib().rbgpu_set64_bucket_set(self.h, i, C.byref(out)))
        return DeviceSet(self.ctx, out.value)

    def extract(self, first: int, count: int) -> "DeviceSet64":
        """rbgpu_set64_extract: a copy of bitmaps [first, first+count)."""
        out = C.c_void_p()
        L.check(L.lib().rbgpu_set64_extract(self.h, first, count, C.byref(out)))
        return DeviceSet64(self.ctx, out.value)

    def signed_longs(self, i: int) -> bool:
        v = C.c_int()
        L.check(L.lib().rbgpu_set64_get_signed_longs(self.h, i, C.byref(v)))
        return bool(v.value)

    def values(self, i: int) -> np.ndarray:
        """Every value of bitmap i in its map's order: ascending unsigned, or for a signedLongs
        Roaring64NavigableMap the buckets of negative highs first (the signed order of the longs)."""
        highs = self.highs(i)
        if not len(highs):
            return np.zeros(0, np.uint64)
        h = self.bucket_set(i).download()
        parts = [(np.uint64(hi) << np.uint64(32)) | h.values(k).astype(np.uint64) for k, hi in enumerate(highs.tolist())]
        if self.signed_longs(i):
            parts = [p for hi, p in zip(highs.tolist(), parts) if hi >= 1 << 31] + \
                    [p for hi, p in zip(highs.tolist(), parts) if hi < 1 << 31]
        return np.concatenate(parts)

    def _serialize(self, sizes_fn, ser_fn) -> List[bytes]:
        n = len(self)
        if n == 0:
            return []
        sizes = np.zeros(n, np.uint64)
        L.check(sizes_fn(self.h, sizes.ctypes.data_as(L._U64P)))
        total = int(sizes.sum())
        buf = C.create_string_buffer(max(total, 1))
        offs = np.zeros(n + 1, np.uint64)
        L.check(ser_fn(self.h, 0, n, buf, total, offs.ctypes.data_as(L._U64P)))
        raw = buf.raw
        return [raw[int(offs[i]):int(offs[i + 1])] for i in range(n)]

    def serialize_portable(self) -> List[bytes]:
        return self._serialize(L.lib().rbgpu_set64_portable_sizes, L.lib().rbgpu_set64_serialize_portable)

    def serialize_legacy(self) -> List[bytes]:
        """Roaring64NavigableMap.serializeLegacy per bitmap (its default serialize)."""
        return self._serialize(L.lib().rbgpu_set64_legacy_sizes, L.lib().rbgpu_set64_serialize_legacy)

    def serialize_art(self) -> List[bytes]:
        """Roaring64Bitmap.serialize per bitmap (rbgpu_set64_serialize_art)."""
        return self._serialize(L.lib().rbgpu_set64_art_sizes, L.lib().rbgpu_set64_serialize_art)

    def set_signed_longs(self, i: int, flag: bool) -> None:
        L.check(L.lib().rbgpu_set64_set_signed_longs(self.h, i, 1 if flag else 0))


def assemble_host(parts: Sequence[bytes]) -> bytes:
    """rbgpu_shard_assemble_host: the whole bitmap's bytes from its key-ordered shards' bytes (the
    header assembly the device gather runs, on the CPU)."""
    n = len(parts)
    arr = (C.c_char_p * max(n, 1))(*parts)
    lens = np.array([len(p) for p in parts] or [0], np.uint64)
    written = C.c_uint64()
    L.lib().rbgpu_shard_assemble_host(arr, lens.ctypes.data_as(L._U64P), n, None, 0, C.byref(written))
    out = C.create_string_buffer(max(int(written.value), 1))
    L.check(L.lib().rbgpu_shard_assemble_host(arr, lens.ctypes.data_as(L._U64P), n, out, int(written.value),
                                              C.byref(written)))
    return out.raw[:int(written.value)]


_default: Optional[Context] = None


def default_context() -> Context:
    global _default
    if _default is None:
        _default = Context(0)
    return _default

"""Restatement of the reference's 64-bit front end for its set algebra (TEST INFRASTRUCTURE ONLY).

Both 64-bit classes of longlong/ run the 32-bit Container algebra of the oracle (rbref):
  Roaring64NavigableMap  a map high 32 bits -> 32-bit RoaringBitmap (ascending unsigned highs, the
                         default comparator); its in-place and/or/xor/andNot(x2) run the 32-bit
                         RoaringBitmap's in-place op per bucket (longlong/Roaring64NavigableMap.java:
                         773-977) and keep a bucket even when it becomes empty;
  Roaring64Bitmap        an ART over 48-bit high keys -> Container (longlong/Roaring64Bitmap.java:
                         319-660); per key the static container op or its in-place form, an empty
                         and / andNot result removed, an empty xor result KEPT (no isEmpty check).
Grouping Roaring64Bitmap's 48-bit keys by their high 32 bits gives the same bucket view (a bucket exists
while it holds a container).  Bytes: the RoaringFormatSpec 64-bit extension ("portable"): u64 bucket
count, then per bucket u32 high and the 32-bit RoaringBitmap (Roaring64NavigableMap.serializePortable,
longlong/Roaring64NavigableMap.java:1254-1261).  Only tests/ and bench.py's CPU baseline import this.
"""
from __future__ import annotations

import struct
from typing import List, Tuple

from . import rbref as R

AND, OR, XOR, ANDNOT = R.AND, R.OR, R.XOR, R.ANDNOT


class Ref64:
    """[(high, RefBitmap)] in ascending unsigned high order; `signed`: Roaring64NavigableMap's signedLongs
    (its TreeMap then iterates the highs as signed ints, which fixes the serialized bucket order)."""

    __slots__ = ("buckets", "signed")

    def __init__(self, buckets: List[Tuple[int, "R.RefBitmap"]] = None, signed: bool = False):
        self.buckets = list(buckets or [])
        self.signed = signed

    def _map_order(self):
        """The buckets in the map's iteration order (Roaring64NavigableMap.highToBitmap.entrySet())."""
        if not self.signed:
            return self.buckets
        return sorted(self.buckets, key=lambda hb: hb[0] - (1 << 32) if hb[0] >= 1 << 31 else hb[0])

    @classmethod
    def from_legacy(cls, data: bytes) -> "Ref64":
        """Roaring64NavigableMap.deserializeLegacy (:1295-1325): readBoolean signedLongs, readInt count,
        then readInt high + RoaringBitmap.deserialize each (DataInput ints are big-endian)."""
        if len(data) < 5:
            raise IOError("truncated 64-bit bitmap")
        signed = data[0] != 0
        (n,) = struct.unpack_from(">i", data, 1)
        pos, out = 5, []
        for _ in range(n):
            if pos + 4 > len(data):
                raise IOError("truncated 64-bit bitmap")
            (h,) = struct.unpack_from(">I", data, pos)
            pos += 4
            b = R.RefBitmap.deserialize(data[pos:])
            pos += len(b.serialize())
            out.append((h, b))
        out.sort(key=lambda hb: hb[0])  # kept in unsigned order; `signed` restores the map's order
        return cls(out, signed)

    def to_legacy(self) -> bytes:
        """Roaring64NavigableMap.serializeLegacy (:1229-1240): writeBoolean(signedLongs), writeInt(size),
        then writeInt(high) + the RoaringBitmap's serialize per entry, in the map's order."""
        parts = [struct.pack(">?i", self.signed, len(self.buckets))]
        for h, b in self._map_order():
            parts.append(struct.pack(">I", h))
            parts.append(b.serialize())
        return b"".join(parts)

    @classmethod
    def of(cls, values) -> "Ref64":
        """Roaring64NavigableMap / Roaring64Bitmap.bitmapOf(long...): each bucket as RoaringBitmap.bitmapOf."""
        import numpy as np
        v = np.unique(np.asarray(values, dtype=np.uint64))
        hi = (v >> np.uint64(32)).astype(np.uint64)
        out = []
        for h in np.unique(hi):
            out.append((int(h), R.RefBitmap.of((v[hi == h] & np.uint64(0xFFFFFFFF)).astype(np.uint32))))
        return cls(out)

    @classmethod
    def from_portable(cls, data: bytes) -> "Ref64":
        """Roaring64NavigableMap.deserializePortable: u64 count, then (u32 high, RoaringBitmap) each."""
        if len(data) < 8:
            raise IOError("truncated 64-bit bitmap")
        (n,) = struct.unpack_from("<Q", data, 0)
        pos, out = 8, []
        for _ in range(n):
            if pos + 4 > len(data):
                raise IOError("truncated 64-bit bitmap")
            (h,) = struct.unpack_from("<I", data, pos)
            pos += 4
            b = R.RefBitmap.deserialize(data[pos:])
            pos += len(b.serialize())
            out.append((h, b))
        return cls(out)

    def to_portable(self) -> bytes:
        """serializePortable (:1254-1261): the map's entries in its iteration order."""
        parts = [struct.pack("<Q", len(self.buckets))]
        for h, b in self._map_order():
            parts.append(struct.pack("<I", h))
            parts.append(b.serialize())
        return b"".join(parts)

    def cardinality(self) -> int:
        return sum(b.cardinality() for _, b in self.buckets)

    def to_array(self):
        import numpy as np
        if not self.buckets:
            return np.zeros(0, np.uint64)
        return np.concatenate([(np.uint64(h) << np.uint64(32)) | b.to_array().astype(np.uint64)
                               for h, b in self.buckets])

    def clone(self) -> "Ref64":
        return Ref64([(h, b.clone()) for h, b in self.buckets], self.signed)


def _merge(x1: Ref64, x2: Ref64):
    """(high, bucket of x1 or None, bucket of x2 or None) in ascending high order."""
    i = j = 0
    a, b = x1.buckets, x2.buckets
    while i < len(a) or j < len(b):
        if j == len(b) or (i < len(a) and a[i][0] < b[j][0]):
            yield a[i][0], a[i][1], None
            i += 1
        elif i == len(a) or b[j][0] < a[i][0]:
            yield b[j][0], None, b[j][1]
            j += 1
        else:
            yield a[i][0], a[i][1], b[j][1]
            i += 1
            j += 1


def _ncont(b) -> int:
    return len(b.containers())


def bitmap_op(op: int, x1: Ref64, x2: Ref64, inplace: bool, same: bool = False) -> Ref64:
    """Roaring64Bitmap: static and/or/xor/andNot(x1, x2) (:345-390, 421-460, 497-517, 630-650) or the
    in-place x1.op(x2) (:319-343, 392-419, 468-495, 599-628; `same`: x2 == this)."""
    if inplace and same:
        return x1.clone() if op in (AND, OR) else Ref64()  # `if (x2 == this)` return / clear()
    out = []
    for h, a, b in _merge(x1, x2):
        if a is not None and b is not None:
            if op == XOR:
                r = R.xor_keep_empty(a, b)  # Container.xor / ixor, put without an isEmpty check
            elif inplace:
                r = a.clone()
                R.op_inplace(op, r, b)      # iand / ior / iandNot: BitmapContainer.ior(Array) stays a Bitmap
            else:
                r = R.op(op, a, b)          # and / or / andNot
        elif a is not None:
            if op == AND:
                continue                    # key absent from x2: removed / not added
            r = a.clone()
        else:
            if op in (AND, ANDNOT):
                continue
            r = b.clone()                   # or / xor: the key of x2 cloned in
        if _ncont(r):
            out.append((h, r))              # a bucket exists while it holds a container
    return Ref64(out)


def and_cardinality(x1: Ref64, x2: Ref64) -> int:
    """Roaring64Bitmap.andCardinality (:562-592): per matched 48-bit key container1.andCardinality."""
    return sum(R.op(AND, a, b).cardinality() for _, a, b in _merge(x1, x2) if a is not None and b is not None)


def navigable_op(op: int, x1: Ref64, x2: Ref64, same: bool = False) -> Ref64:
    """Roaring64NavigableMap in-place x1.and/or/xor/andNot(x2) (:773-977): per bucket the 32-bit
    RoaringBitmap in-place op; a bucket left empty stays in the map; `same`: x2 == this."""
    if same:
        return x1.clone() if op in (AND, OR) else Ref64(signed=x1.signed)  # return / clear()
    out = []
    for h, a, b in _merge(x1, x2):
        if a is not None and b is not None:
            r = a.clone()
            R.op_inplace(op, r, b)
        elif a is not None:
            if op == AND:
                continue                    # thisIterator.remove()
            r = a
        else:
            if op in (AND, ANDNOT):
                continue
            r = b.clone()                   # pushBitmapForHigh(high, lowBitmap2.clone())
        out.append((h, r))
    return Ref64(out, x1.signed)

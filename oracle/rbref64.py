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
_ARRAY, _BITMAP, _RUN = 0, 1, 2
# art/NodeType.java ordinals (NODE4, NODE16, NODE48, NODE256, LEAF_NODE) and the body bytes of each
# internal node (Node4 int key, Node16 two longs, Node48 32-long childIndex, Node256 4-long bitmapMask)
ART_LEAF = 4
ART_BODY = {0: 4, 1: 16, 2: 256, 3: 32}


def _containers_of(blob: bytes, meta=None):
    """[(key, type, card, nruns, payload)] of a 32-bit RoaringBitmap in the RoaringFormatSpec layout
    (RoaringArray.deserialize, RoaringArray.java:300-380): cookie, run flags, key / card-1 pairs, offsets,
    payloads (a Run payload here without its leading run count).  `meta` (RefBitmap.containers()) gives
    the types and cardinalities when the bitmap may hold an empty container (a kept-empty xor result:
    card-1 = 0xFFFF and no payload in the oracle's bytes)."""
    (cookie,) = struct.unpack_from("<I", blob, 0)
    if cookie & 0xFFFF == 12347:
        n = (cookie >> 16) + 1
        flags, pos = blob[4:4 + (n + 7) // 8], 4 + (n + 7) // 8
        runs = [bool(flags[i >> 3] >> (i & 7) & 1) for i in range(n)]
    else:
        (n,) = struct.unpack_from("<I", blob, 4)
        pos, runs = 8, [False] * n
    kc = struct.unpack_from(f"<{2 * n}H", blob, pos)
    pos += 4 * n
    if cookie & 0xFFFF != 12347 or n >= 4:  # offsets (NO_OFFSET_THRESHOLD = 4 with run containers)
        pos += 4 * n
    out = []
    for i in range(n):
        key, card = kc[2 * i], kc[2 * i + 1] + 1
        if meta is not None and meta[i][2] == 0:
            # A kept-empty container keeps the type its xor produced: an empty Run xor Run is a Run
            # (RunContainer.xor -> toEfficientContainer, RunContainer.java:2445-2482, 2326-2335: the
            # 2 <= min(8192, 2) tie goes to Run), its payload the run count 0; an empty Array / Bitmap
            # xor is an Array with no payload (ArrayContainer.java:1311-1336, BitmapContainer.java:1381-1422).
            if runs[i]:
                (nr,) = struct.unpack_from("<H", blob, pos)
                out.append((key, _RUN, 0, nr, b""))
                pos += 2 + 4 * nr
            else:
                out.append((key, _ARRAY, 0, 0, b""))
            continue
        if runs[i]:
            (nr,) = struct.unpack_from("<H", blob, pos)
            out.append((key, _RUN, card, nr, bytes(blob[pos + 2:pos + 2 + 4 * nr])))
            pos += 2 + 4 * nr
        elif card <= 4096:
            out.append((key, _ARRAY, card, 0, bytes(blob[pos:pos + 2 * card])))
            pos += 2 * card
        else:
            out.append((key, _BITMAP, card, 0, bytes(blob[pos:pos + 8192])))
            pos += 8192
    return out


def _blob_of(conts) -> bytes:
    """The RoaringFormatSpec bytes of [(key, type, card, nruns, payload)] (RoaringArray.serialize,
    RoaringArray.java:900-953: with run containers the cookie 12347 | (n - 1) << 16 and the run flags, offsets
    only from 4 containers on; else 12346, the count and offsets)."""
    n = len(conts)
    has_run = any(t == _RUN for _, t, *_ in conts)
    if has_run:
        flags = bytearray((n + 7) // 8)
        for i, (_, t, *_) in enumerate(conts):
            if t == _RUN:
                flags[i >> 3] |= 1 << (i & 7)
        head = struct.pack("<I", 12347 | (n - 1) << 16) + bytes(flags)
    else:
        head = struct.pack("<II", 12346, n)
    head += b"".join(struct.pack("<HH", k, c - 1) for k, _, c, _, _ in conts)
    bodies = [struct.pack("<H", nr) + p if t == _RUN else p for _, t, _, nr, p in conts]
    if not has_run or n >= 4:
        off = len(head) + 4 * n
        offs = []
        for b in bodies:
            offs.append(off)
            off += len(b)
        head += struct.pack(f"<{n}I", *offs)
    return head + b"".join(bodies)


def _bitmap_of(conts) -> "R.RefBitmap":
    """The RefBitmap of [(key, type, card, nruns, payload)], empty Array / Run containers included: those are
    made the way the reference makes them, as the xor of two equal one-value containers of that type (the
    bitmap's other containers, unmatched, are cloned with their types)."""
    if all(c[2] for c in conts):
        return R.RefBitmap.deserialize(_blob_of(conts))
    full, ph = [], []
    for key, t, card, nr, payload in conts:
        if card:
            full.append((key, t, card, nr, payload))
            continue
        if t == _BITMAP or nr:
            raise IOError("non-canonical empty container")
        x = (key, _RUN, 1, 1, struct.pack("<HH", 0, 0)) if t == _RUN else (key, _ARRAY, 1, 0, struct.pack("<H", 0))
        full.append(x)
        ph.append(x)
    return R.xor_keep_empty(R.RefBitmap.deserialize(_blob_of(full)), R.RefBitmap.deserialize(_blob_of(ph)))


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
        # highToBitmap.put: the TreeMap orders the highs, a repeated high keeps the bitmap read last
        last = {h: b for h, b in out}
        out = sorted(last.items())  # kept in unsigned order; `signed` restores the map's order
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

    @classmethod
    def from_art(cls, data: bytes) -> "Ref64":
        """Roaring64Bitmap.deserialize (longlong/Roaring64Bitmap.java:905-908) = HighLowContainer.deserialize
        (longlong/HighLowContainer.java:246-254): the empty tag, Art.deserializeArt (art/Art.java:314-317,
        373-391: u64 LE key count, then the nodes in preorder) and Containers.deserialize (art/Containers.java:
        276-303).  A leaf's 6 key bytes are the container's high 48 bits; its container index picks the
        container.  Parity unpinned: no reference fixture holds this format."""
        if not data:
            raise IOError("truncated 64-bit bitmap")
        if data[0] == 0:
            return cls()
        pos = 9  # the NOT_EMPTY tag, then Art.keySize (read, not needed: the leaves are counted below)
        leaves = []

        def node():  # Node.deserialize (art/Node.java:169-176, 354-400) and the children in key order
            nonlocal pos
            t, count, plen = data[pos], struct.unpack_from("<H", data, pos + 1)[0], data[pos + 3]
            pos += 4 + plen
            if t == ART_LEAF:  # LeafNode.deserializeNodeBody (art/LeafNode.java:57-62)
                leaves.append((int.from_bytes(data[pos:pos + 6], "big"), struct.unpack_from("<Q", data, pos + 6)[0]))
                pos += 14
                return
            if t not in ART_BODY:
                raise IOError(f"bad ART node type {t}")
            pos += ART_BODY[t]
            for _ in range(count):
                node()

        node()
        (first_n,) = struct.unpack_from("<i", data, pos)
        pos += 4
        conts = {}
        for i in range(first_n):  # the trim mark, then the second-level array with its null slots
            (second_n,) = struct.unpack_from("<i", data, pos + 1)
            pos += 5
            for j in range(second_n):
                tag = data[pos]
                pos += 1
                if tag == 0:
                    continue
                ctype, card = data[pos], struct.unpack_from("<i", data, pos + 1)[0]
                pos += 5
                # Containers.instanceContainer (art/Containers.java:352-378): 0 Run, 1 Bitmap, 2 Array
                if ctype == 0:
                    (nr,) = struct.unpack_from("<H", data, pos)
                    payload, typ = data[pos + 2:pos + 2 + 4 * nr], _RUN
                    pos += 2 + 4 * nr
                elif ctype == 1:
                    payload, typ, nr = data[pos:pos + 8192], _BITMAP, 0
                    pos += 8192
                elif ctype == 2:
                    payload, typ, nr = data[pos:pos + 2 * card], _ARRAY, 0
                    pos += 2 * card
                else:
                    raise IOError(f"bad container type {ctype}")
                conts[(i << 32) | j] = (typ, card, nr, payload)
        pos += 16  # containerSize, firstLevelIdx, secondLevelIdx
        if pos != len(data):
            raise IOError("trailing bytes after the ART containers")
        groups = {}
        for key48, idx in sorted(leaves):
            typ, card, nr, payload = conts[idx]
            # an empty container (a kept-empty xor result) is kept: Containers.deserialize reads it back
            # like any other (art/Containers.java:276-303)
            groups.setdefault(key48 >> 16, []).append((key48 & 0xFFFF, typ, card, nr, payload))
        return cls([(h, _bitmap_of(cs)) for h, cs in sorted(groups.items())])

    def to_art(self, slots=None, cap=None) -> bytes:
        """Roaring64Bitmap.serialize (:880-882) of the bitmap built by inserting its containers in ascending
        key order (what Roaring64Bitmap.and/or/... and addLong in order produce): the ART is then the
        path-compressed radix tree of the 6-byte keys with the smallest node type per child count (Node4
        / 16 / 48 / 256 grow at 5 / 17 / 49 children: art/Node4.java:90-108, Node16.java:140-180,
        Node48.java:180-200), Node48 children at slots in key order; container i at index i of one
        second-level array grown like an ArrayList from 1 (art/Containers.java:78-92, 150-170).
        Parity unpinned (no fixture): the structure is restated, not checked against a Java writer.
        `slots` / `cap` (tests): container i at second-level slot slots[i] of a `cap`-slot array, as a
        history with removals or another insertion order leaves them."""
        conts = []
        for h, b in self.buckets:
            for key16, typ, card, nr, payload in _containers_of(b.serialize(), b.containers()):
                conts.append(((h << 16) | key16, typ, card, nr, payload))
        if not conts:
            return b"\x00"
        keys = [k.to_bytes(6, "big") for k, *_ in conts]
        slot = list(range(len(conts))) if slots is None else list(slots)
        out = [b"\x01", struct.pack("<q", len(conts))]

        def emit(lo, hi, depth):
            if hi - lo == 1:  # LeafNode (art/LeafNode.java:43-47): header, key bytes, LE container index
                out.append(bytes([ART_LEAF, 0, 0, 0]) + keys[lo] + struct.pack("<Q", slot[lo]))
                return
            p = 0
            while depth + p < 6 and all(keys[i][depth + p] == keys[lo][depth + p] for i in range(lo, hi)):
                p += 1
            d = depth + p
            starts = [i for i in range(lo, hi) if i == lo or keys[i][d] != keys[i - 1][d]]
            n = len(starts)
            t = 0 if n <= 4 else 1 if n <= 16 else 2 if n <= 48 else 3
            out.append(bytes([t]) + struct.pack("<H", n) + bytes([p]) + keys[lo][depth:d])
            kb = [keys[i][d] for i in starts]
            if t == 0:    # Node4: int key, child i's byte at bits (3 - i) * 8, written reversed
                out.append(bytes(reversed(bytes(kb + [0] * (4 - n)))))
            elif t == 1:  # Node16: firstV / secondV, bytes 0-7 / 8-15 big-endian, each written reversed
                padded = bytes(kb + [0] * (16 - n))
                out.append(bytes(reversed(padded[:8])) + bytes(reversed(padded[8:])))
            elif t == 2:  # Node48: childIndex, key byte -> child slot (0xFF empty), 8 keys per long, reversed
                ci = bytearray([0xFF] * 256)
                for c, k in enumerate(kb):
                    ci[k] = c
                out.append(b"".join(bytes(reversed(ci[8 * i:8 * i + 8])) for i in range(32)))
            else:         # Node256: bitmapMask, bit k & 63 of long k >> 6, little endian
                m = [0, 0, 0, 0]
                for k in kb:
                    m[k >> 6] |= 1 << (k & 63)
                out.append(struct.pack("<4Q", *m))
            for s, e in zip(starts, starts[1:] + [hi]):
                emit(s, e, d + 1)

        emit(0, len(conts), 0)
        if cap is None:
            cap = 1
            for n in range(2, len(conts) + 1):  # Containers.grow(minCapacity = n)
                if n > cap:
                    cap = max(cap + (cap >> 1), n)
        out.append(struct.pack("<i", 1) + bytes([0xFE]) + struct.pack("<i", cap))  # NOT_TRIMMED_MARK
        at = {sl: i for i, sl in enumerate(slot)}
        for j in range(cap):
            if j not in at:
                out.append(b"\x00")  # NULL_MARK
                continue
            _, typ, card, nr, payload = conts[at[j]]
            ctype = {_RUN: 0, _BITMAP: 1, _ARRAY: 2}[typ]
            out.append(bytes([1, ctype]) + struct.pack("<i", card))
            out.append(struct.pack("<H", nr) + payload if typ == _RUN else payload)
        out.append(struct.pack("<qii", len(conts), 0, max(slot)))
        return b"".join(out)

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

"""Host-side mirror of the reference's Java API for the set-algebra hot path.

Names, argument meaning and error behaviour follow the reference so a caller of
org.roaringbitmap.{RoaringBitmap, FastAggregation, ParallelAggregation} and
org.roaringbitmap.buffer.BufferFastAggregation finds the same surface; every call runs on the
MI355X through librbgpu (no CPU fallback).

  RoaringBitmap.and_/or_/xor/andNot(x1, x2)   static, RoaringBitmap.java:377, 860, 1071, 444
  x1.and_/or_/xor/andNot(x2)                  in place, RoaringBitmap.java:1270, 2481, 3296, 1346
  RoaringBitmap.*Cardinality(x1, x2)           RoaringBitmap.java:413, 916, 931, 944
  RoaringBitmap.or_(*bitmaps)                   RoaringBitmap.java:844 -> FastAggregation.or
  x.runOptimize()                               RoaringBitmap.java:2764
  FastAggregation.and_/or_/xor(*bitmaps)        FastAggregation.java:37, 602, 772
  FastAggregation.naive_and/workShyAnd/...      FastAggregation.java:328, 356, 477, 541, 576
  ParallelAggregation.or_/xor(*bitmaps)         ParallelAggregation.java:161, 182
  BufferFastAggregation.*                       buffer/BufferFastAggregation.java
  BufferParallelAggregation.or_/xor             buffer/BufferParallelAggregation.java:166, 187
  serialize / deserialize                       RoaringArray.java:851-940, 276-348

Python reserves `and`/`or`, so those two carry a trailing underscore.  Called on the class with two
bitmaps, and_/or_/xor/andNot are the static ops; called on an instance with one, they are the in-place
instance ops (the bitmap takes the result, the argument is unchanged).  Deserialize errors raise
IOError (FormatError), like the reference's IOException; non-canonical inputs and the reference's
IllegalArgumentException raise ValueError.  Java overloads that differ only by parameter type
(ImmutableRoaringBitmap... / MutableRoaringBitmap... / Iterator) are separate methods here, named by
the overload (`*_mutable`, `*_iterator`).
"""
from __future__ import annotations

from typing import Optional, Sequence

import numpy as np

from . import _lib as L
from .engine import DeviceSet, default_context


class _StaticOrInPlace:
    """RoaringBitmap.and(x1, x2) (static, a new bitmap) when looked up on the class, x1.and(x2) (in
    place, returns None like the Java void method) when looked up on an instance."""

    def __init__(self, op: int):
        self.op = op

    def __get__(self, obj, cls):
        op = self.op
        if obj is None:
            return lambda x1, x2: cls._pair(op, x1, x2)
        return lambda x2: obj._inplace(op, x2)


class RoaringBitmap:
    """A single 32-bit Roaring bitmap resident in HBM (a one-bitmap DeviceSet)."""

    __slots__ = ("_set",)

    def __init__(self, dset: Optional[DeviceSet] = None):
        if dset is None:
            dset = default_context().upload_values([np.zeros(0, np.uint32)])
        assert len(dset) == 1
        self._set = dset

    # ---- construction / bytes
    @staticmethod
    def bitmapOf(*values) -> "RoaringBitmap":
        vals = np.asarray(values[0] if len(values) == 1 and np.ndim(values[0]) else values, dtype=np.uint32)
        return RoaringBitmap(default_context().upload_values([vals]))

    @staticmethod
    def deserialize(data: bytes) -> "RoaringBitmap":
        return RoaringBitmap(default_context().upload_serialized([data]))

    def serialize(self) -> bytes:
        return self._set.serialize()[0]

    def serializedSizeInBytes(self) -> int:
        return int(self._set.serialized_sizes()[0])

    def getCardinality(self) -> int:
        return int(self._set.cardinalities()[0])

    def getLongSizeInBytes(self) -> int:
        return int(self._set.summaries()[0]["size_in_bytes"])

    def isEmpty(self) -> bool:
        return self._set.n_containers == 0

    def toArray(self) -> np.ndarray:
        return self._set.download().values(0)

    def runOptimize(self) -> bool:
        """RoaringBitmap.runOptimize (RoaringBitmap.java:2764-2775) on the device: each container takes
        its smallest encoding; True when the bitmap holds a Run container afterwards."""
        self._set, any_run = self._set.run_optimize()
        return bool(any_run[0])

    def clone(self) -> "RoaringBitmap":
        return RoaringBitmap(self._set.ctx.extract(self._set, 0, 1))

    def clear(self) -> None:
        self._set = default_context().upload_values([np.zeros(0, np.uint32)])

    def containers(self):
        """[(key, type, card, nruns)] — the container-type view used by insights/BitmapAnalyser."""
        h = self._set.download()
        return list(zip(h.key.tolist(), h.type.tolist(), h.card.tolist(), h.nruns.tolist()))

    def __eq__(self, other) -> bool:
        return isinstance(other, RoaringBitmap) and self.serialize() == other.serialize()

    def __hash__(self):
        return hash(self.serialize())

    def __repr__(self):
        return f"RoaringBitmap(card={self.getCardinality()}, containers={self._set.n_containers})"

    # ---- static pairwise algebra / in-place instance ops
    @staticmethod
    def _pair(op: int, x1: "RoaringBitmap", x2: "RoaringBitmap") -> "RoaringBitmap":
        return RoaringBitmap(default_context().pairwise(op, x1._set, x2._set, npairs=1))

    def _inplace(self, op: int, x2: "RoaringBitmap") -> None:
        # x2 is this very bitmap: the reference's `x2 == this` branches (rbgpu_pairwise_inplace's
        # same-set / same-index case)
        b = self._set if x2 is self else x2._set
        self._set = default_context().pairwise_inplace(op, self._set, b, npairs=1)

    and_ = _StaticOrInPlace(L.AND)
    xor = _StaticOrInPlace(L.XOR)
    andNot = _StaticOrInPlace(L.ANDNOT)

    class _Or(_StaticOrInPlace):
        def __get__(self, obj, cls):
            if obj is not None:
                return lambda x2: obj._inplace(L.OR, x2)

            def or_(*bitmaps):
                if len(bitmaps) == 2 and all(isinstance(b, RoaringBitmap) for b in bitmaps):
                    return cls._pair(L.OR, bitmaps[0], bitmaps[1])
                return FastAggregation.or_(*bitmaps)  # RoaringBitmap.or(RoaringBitmap...) (:844)
            return or_

    or_ = _Or(L.OR)

    @staticmethod
    def _pair_card(op: int, x1, x2) -> int:
        return int(default_context().pairwise_cardinality(op, x1._set, x2._set, npairs=1)[0])

    @staticmethod
    def andCardinality(x1, x2) -> int:
        return RoaringBitmap._pair_card(L.AND, x1, x2)

    @staticmethod
    def orCardinality(x1, x2) -> int:
        return RoaringBitmap._pair_card(L.OR, x1, x2)

    @staticmethod
    def xorCardinality(x1, x2) -> int:
        return RoaringBitmap._pair_card(L.XOR, x1, x2)

    @staticmethod
    def andNotCardinality(x1, x2) -> int:
        return RoaringBitmap._pair_card(L.ANDNOT, x1, x2)


def _gather(bitmaps: Sequence[RoaringBitmap]):
    """One device set holding each distinct bitmap once, and the member list naming them in call order:
    a bitmap passed twice is the same object twice (naive_and skips its smallest member by identity,
    FastAggregation.java:337-341)."""
    ctx = default_context()
    index, uniq, members = {}, [], []
    for b in bitmaps:
        if id(b) not in index:
            index[id(b)] = len(uniq)
            uniq.append(b)
        members.append(index[id(b)])
    dset = ctx.upload_serialized([b.serialize() for b in uniq])
    return dset, np.asarray(members, np.uint32)


def _flatten(bitmaps) -> Sequence[RoaringBitmap]:
    if len(bitmaps) == 1 and not isinstance(bitmaps[0], RoaringBitmap):
        return list(bitmaps[0])
    return list(bitmaps)


def _wide(sem: int, bitmaps, empty_ok: bool = True) -> RoaringBitmap:
    bms = _flatten(bitmaps)
    if not bms and empty_ok:
        return RoaringBitmap()
    if not bms:
        dset, members = default_context().upload_values([np.zeros(0, np.uint32)]), np.zeros(0, np.uint32)
    else:
        dset, members = _gather(bms)
    return RoaringBitmap(default_context().wide(sem, dset, members))


def _check_buffer(buffer, nbitmaps: int, always: bool) -> None:
    """The long[] aggregation-buffer overloads: IllegalArgumentException below 1024 words (checked when
    the work-shy path runs, FastAggregation.java:51-63, :477-481), then Arrays.fill(buffer, 0)."""
    if (always or nbitmaps > 10) and len(buffer) < 1024:
        raise ValueError("buffer should have at least 1024 elements.")


def _is_buffer(x, more: bool) -> bool:
    """A long[] aggregation buffer (words), as opposed to a bitmap or a list of bitmaps."""
    if isinstance(x, np.ndarray):
        return True
    if isinstance(x, (list, tuple)):
        return (len(x) == 0 and more) or (len(x) > 0 and all(isinstance(v, (int, np.integer)) for v in x))
    return False


def _zero(buffer) -> None:
    try:
        buffer[:] = [0] * len(buffer) if isinstance(buffer, list) else 0
    except TypeError:
        pass


class FastAggregation:
    """org.roaringbitmap.FastAggregation (FastAggregation.java)."""

    @staticmethod
    def and_(*bitmaps) -> RoaringBitmap:
        """and(RoaringBitmap...) (:37-42); and(long[] aggregationBuffer, RoaringBitmap...) (:51-63) when
        the first argument is a word buffer."""
        if bitmaps and _is_buffer(bitmaps[0], len(bitmaps) > 1):
            buffer, rest = bitmaps[0], bitmaps[1:]
            _check_buffer(buffer, len(_flatten(rest)) if rest else 0, False)
            try:
                return _wide(L.FAST_AND, rest)
            finally:
                _zero(buffer)
        return _wide(L.FAST_AND, bitmaps)

    @staticmethod
    def and_iterator(bitmaps) -> RoaringBitmap:
        """and(Iterator) (:26-28) = naive_and(Iterator): the fold from the first bitmap."""
        return _wide(L.NAIVE_AND_ITER, [list(bitmaps)])

    @staticmethod
    def or_(*bitmaps) -> RoaringBitmap:
        return _wide(L.FAST_OR, bitmaps)

    @staticmethod
    def xor(*bitmaps) -> RoaringBitmap:
        return _wide(L.FAST_XOR, bitmaps)

    @staticmethod
    def naive_and(*bitmaps) -> RoaringBitmap:
        return _wide(L.NAIVE_AND, bitmaps)

    @staticmethod
    def naive_and_iterator(bitmaps) -> RoaringBitmap:
        return _wide(L.NAIVE_AND_ITER, [list(bitmaps)])

    @staticmethod
    def workShyAnd(buffer, *bitmaps) -> RoaringBitmap:
        """workShyAnd(long[] buffer, RoaringBitmap...) (:356-396)."""
        return _wide(L.WORKSHY_AND, bitmaps)

    @staticmethod
    def workAndMemoryShyAnd(buffer, *bitmaps) -> RoaringBitmap:
        """workAndMemoryShyAnd(long[] buffer, RoaringBitmap...) (:477-514): the workShyAnd result; the
        buffer must hold at least 1024 words."""
        _check_buffer(buffer, len(_flatten(bitmaps)) if bitmaps else 0, True)
        return _wide(L.WORKSHY_AND, bitmaps)

    @staticmethod
    def naive_or(*bitmaps) -> RoaringBitmap:
        return _wide(L.FAST_OR, bitmaps)

    @staticmethod
    def naive_xor(*bitmaps) -> RoaringBitmap:
        return _wide(L.FAST_XOR, bitmaps)

    @staticmethod
    def horizontal_or(*bitmaps) -> RoaringBitmap:
        """horizontal_or(List / varargs) (FastAggregation.java:124-231); the Iterator overload
        (:110-112) is naive_or."""
        return _wide(L.HORIZONTAL_OR, bitmaps)

    @staticmethod
    def horizontal_xor(*bitmaps) -> RoaringBitmap:
        return _wide(L.HORIZONTAL_XOR, bitmaps)

    @staticmethod
    def priorityqueue_or(*bitmaps) -> RoaringBitmap:
        """priorityqueue_or(RoaringBitmap...) (FastAggregation.java:675-721) and priorityqueue_or(Iterator)
        (:615-664, the same queue): lazy ORs of the two smallest bitmaps (getLongSizeInBytes) on the
        device, the survivor repaired."""
        return _wide(L.PQ_OR, bitmaps)

    @staticmethod
    def priorityqueue_xor(*bitmaps) -> RoaringBitmap:
        return _wide(L.PQ_XOR, bitmaps)

    @staticmethod
    def andCardinality(*bitmaps) -> int:
        bms = _flatten(bitmaps)
        if not bms:
            return 0
        if len(bms) == 1:
            return bms[0].getCardinality()
        if len(bms) == 2:
            return RoaringBitmap.andCardinality(bms[0], bms[1])
        dset, members = _gather(bms)
        return default_context().wide_cardinality(L.AND, dset, members)

    @staticmethod
    def orCardinality(*bitmaps) -> int:
        bms = _flatten(bitmaps)
        if not bms:
            return 0
        if len(bms) == 1:
            return bms[0].getCardinality()
        if len(bms) == 2:
            return RoaringBitmap.orCardinality(bms[0], bms[1])
        dset, members = _gather(bms)
        return default_context().wide_cardinality(L.OR, dset, members)


class ParallelAggregation:
    """org.roaringbitmap.ParallelAggregation (ParallelAggregation.java): key-parallel on the GPU."""

    @staticmethod
    def or_(*bitmaps) -> RoaringBitmap:
        return _wide(L.PAR_OR, bitmaps)

    @staticmethod
    def xor(*bitmaps) -> RoaringBitmap:
        return _wide(L.PAR_XOR, bitmaps)


class BufferFastAggregation:
    """org.roaringbitmap.buffer.BufferFastAggregation over ImmutableRoaringBitmap / MutableRoaringBitmap
    (buffer/BufferFastAggregation.java): the same container algebra as FastAggregation; where the
    results differ the device runs the buffer's own semantics (rbgpu.h rb_wide_sem RB_BUFFER_*)."""

    @staticmethod
    def and_(*bitmaps) -> RoaringBitmap:
        """and(ImmutableRoaringBitmap...) / and(long[], ImmutableRoaringBitmap...) (:29-58): workShyAnd
        above 10 bitmaps, else naive_and."""
        return FastAggregation.and_(*bitmaps)

    @staticmethod
    def and_iterator(bitmaps, buffer=None) -> RoaringBitmap:
        """and(Iterator) / and(long[], Iterator) (:67-91): workShyAnd over the iterator (FastAggregation's
        and(Iterator) is naive_and); an empty iterator gives an empty bitmap."""
        bms = list(bitmaps)
        try:
            return _wide(L.WORKSHY_AND, [bms])
        finally:
            if buffer is not None:
                _zero(buffer)

    @staticmethod
    def and_mutable(*bitmaps) -> RoaringBitmap:
        """and(MutableRoaringBitmap...) (:101-103) = and(Iterator): workShyAnd."""
        return _wide(L.WORKSHY_AND, bitmaps)

    @staticmethod
    def naive_and(*bitmaps) -> RoaringBitmap:
        """naive_and(ImmutableRoaringBitmap...) (:348-370): from the bitmap with the fewest containers."""
        return _wide(L.NAIVE_AND, bitmaps)

    @staticmethod
    def naive_and_mutable(*bitmaps) -> RoaringBitmap:
        """naive_and(MutableRoaringBitmap...) (:408-418) / naive_and(Iterator) (:384-394): from the first."""
        return _wide(L.NAIVE_AND_ITER, bitmaps)

    @staticmethod
    def workShyAnd(buffer, *bitmaps) -> RoaringBitmap:
        return _wide(L.WORKSHY_AND, bitmaps)

    @staticmethod
    def workAndMemoryShyAnd(buffer, *bitmaps) -> RoaringBitmap:
        """workAndMemoryShyAnd(long[], ImmutableRoaringBitmap...) (:627-667)."""
        return FastAggregation.workAndMemoryShyAnd(buffer, *bitmaps)

    @staticmethod
    def or_(*bitmaps) -> RoaringBitmap:
        """or / naive_or(ImmutableRoaringBitmap... / Iterator) (:675-692, 776-790): naivelazyor."""
        return _wide(L.FAST_OR, bitmaps)

    naive_or = or_

    @staticmethod
    def or_mutable(*bitmaps) -> RoaringBitmap:
        """or / naive_or(MutableRoaringBitmap...) (:711-717, 797-799): answer.lazyor(b) per bitmap."""
        return _wide(L.BUFFER_NAIVE_OR, bitmaps)

    naive_or_mutable = or_mutable

    @staticmethod
    def xor(*bitmaps) -> RoaringBitmap:
        return _wide(L.FAST_XOR, bitmaps)

    naive_xor = xor

    @staticmethod
    def horizontal_or(*bitmaps) -> RoaringBitmap:
        return _wide(L.HORIZONTAL_OR, bitmaps)

    @staticmethod
    def horizontal_xor(*bitmaps) -> RoaringBitmap:
        return _wide(L.HORIZONTAL_XOR, bitmaps)

    @staticmethod
    def priorityqueue_or(*bitmaps) -> RoaringBitmap:
        """priorityqueue_or(ImmutableRoaringBitmap...) (:810-866): ordered by serializedSizeInBytes."""
        return _wide(L.BUFFER_PQ_OR, bitmaps)

    @staticmethod
    def priorityqueue_or_iterator(bitmaps) -> RoaringBitmap:
        """priorityqueue_or(Iterator) (:869-930): ordered by ImmutableRoaringBitmap.getLongSizeInBytes."""
        return _wide(L.BUFFER_PQ_OR_ITER, [list(bitmaps)])

    @staticmethod
    def priorityqueue_xor(*bitmaps) -> RoaringBitmap:
        """priorityqueue_xor(ImmutableRoaringBitmap...) (:933-958): IllegalArgumentException (ValueError)
        below 2 bitmaps."""
        return _wide(L.BUFFER_PQ_XOR, bitmaps, empty_ok=False)


class BufferParallelAggregation:
    """org.roaringbitmap.buffer.BufferParallelAggregation (buffer/BufferParallelAggregation.java): the
    per-key folds are ParallelAggregation's (:194-230), so or / xor are RB_PAR_OR / RB_PAR_XOR."""

    @staticmethod
    def or_(*bitmaps) -> RoaringBitmap:
        """or(ImmutableRoaringBitmap...) (:166-180)."""
        return _wide(L.PAR_OR, bitmaps)

    @staticmethod
    def xor(*bitmaps) -> RoaringBitmap:
        """xor(ImmutableRoaringBitmap...) (:187-192)."""
        return _wide(L.PAR_XOR, bitmaps)


class _Bitmap64:
    """Shared surface of the two 64-bit classes (one 64-bit bitmap resident in HBM as buckets)."""

    __slots__ = ("_set",)
    FLAVOR = L.RB64_BITMAP

    def __init__(self, dset=None):
        self._set = dset if dset is not None else default_context().upload_values64([np.zeros(0, np.uint64)])

    @classmethod
    def bitmapOf(cls, *values):
        vals = np.asarray(values[0] if len(values) == 1 and np.ndim(values[0]) else values, dtype=np.uint64)
        return cls(default_context().upload_values64([vals]))

    @classmethod
    def deserializePortable(cls, data: bytes):
        """Roaring64NavigableMap.deserializePortable (the RoaringFormatSpec 64-bit extension)."""
        return cls(default_context().upload_portable64([data]))

    def serializePortable(self) -> bytes:
        return self._set.serialize_portable()[0]

    def getLongCardinality(self) -> int:
        return int(self._set.cardinalities()[0])

    def isEmpty(self) -> bool:
        """getLongCardinality() == 0 (Roaring64NavigableMap.java:1148, Roaring64Bitmap.java:837): emptied
        buckets and kept empty xor containers do not count."""
        return self.getLongCardinality() == 0

    def toArray(self) -> np.ndarray:
        """Every value, ascending unsigned (Roaring64Bitmap.java:946, Roaring64NavigableMap.java:1409):
        read from the device buckets, so a kept empty container contributes nothing."""
        return self._set.values(0)

    def select(self, j: int) -> int:
        """select(j) (Roaring64Bitmap.java:106, Roaring64NavigableMap.java:351): IllegalArgumentException
        (ValueError) past the cardinality."""
        v = self.toArray()
        if not 0 <= j < len(v):
            raise ValueError(f"select {j} when the cardinality is {len(v)}")
        return int(v[j])

    def clone(self):
        """A device copy (rbgpu_set64_extract), the kept empty containers included."""
        return type(self)(self._set.extract(0, 1))

    def _inplace(self, op: int, x2) -> None:
        b = self._set if x2 is self else x2._set  # x2 == this: the same set and index on both sides
        self._set = default_context().pairwise64(self.FLAVOR, op, self._set, b, npairs=1, inplace=True)

    def and_(self, x2) -> None:
        self._inplace(L.AND, x2)

    def or_(self, x2) -> None:
        self._inplace(L.OR, x2)

    def xor(self, x2) -> None:
        self._inplace(L.XOR, x2)

    def andNot(self, x2) -> None:
        self._inplace(L.ANDNOT, x2)


class Roaring64NavigableMap(_Bitmap64):
    """org.roaringbitmap.longlong.Roaring64NavigableMap (longlong/Roaring64NavigableMap.java): in-place
    and/or/xor/andNot(x2) per bucket with the 32-bit RoaringBitmap's in-place ops (:773-977).  serialize /
    deserialize use the default SERIALIZATION_MODE_LEGACY format (:51, 1207-1252, 1276-1325)."""

    __slots__ = ()
    FLAVOR = L.RB64_NAVIGABLE

    def __init__(self, dset=None, signedLongs: bool = False):
        super().__init__(dset)
        if signedLongs:
            self._set.set_signed_longs(0, True)

    @classmethod
    def deserializeLegacy(cls, data: bytes):
        """deserializeLegacy (:1295-1325): signedLongs, then the buckets (IOError on bad bytes)."""
        return cls(default_context().upload_legacy64([data]))

    deserialize = deserializeLegacy

    def serializeLegacy(self) -> bytes:
        return self._set.serialize_legacy()[0]

    serialize = serializeLegacy


class _StaticOrInPlace64(_StaticOrInPlace):
    def __get__(self, obj, cls):
        op = self.op
        if obj is None:  # Roaring64Bitmap.and(x1, x2) etc. (static)
            return lambda x1, x2: cls(default_context().pairwise64(L.RB64_BITMAP, op, x1._set, x2._set, npairs=1))
        return lambda x2: obj._inplace(op, x2)


class Roaring64Bitmap(_Bitmap64):
    """org.roaringbitmap.longlong.Roaring64Bitmap (longlong/Roaring64Bitmap.java): static and in-place
    and/or/xor/andNot (:319-660) over 48-bit keys; an empty xor result is kept under its key."""

    __slots__ = ()
    FLAVOR = L.RB64_BITMAP

    @staticmethod
    def andCardinality(x1, x2) -> int:
        """Roaring64Bitmap.andCardinality (longlong/Roaring64Bitmap.java:562-592), on the device."""
        return int(default_context().pairwise64_cardinality(L.AND, x1._set, x2._set, npairs=1)[0])

    @classmethod
    def deserialize(cls, data: bytes):
        """deserialize (:905-908): HighLowContainer's ART + Containers stream (rbgpu_set64_from_art)."""
        return cls(default_context().upload_art64([data]))

    def serialize(self) -> bytes:
        """serialize (:880-882), the canonical stream of this bitmap (rbgpu_set64_serialize_art)."""
        return self._set.serialize_art()[0]

    and_ = _StaticOrInPlace64(L.AND)
    or_ = _StaticOrInPlace64(L.OR)
    xor = _StaticOrInPlace64(L.XOR)
    andNot = _StaticOrInPlace64(L.ANDNOT)

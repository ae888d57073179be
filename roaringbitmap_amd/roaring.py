"""Host-side mirror of the reference's Java API for the set-algebra hot path.

Names, argument meaning and error behaviour follow the reference so a caller of
org.roaringbitmap.{RoaringBitmap, FastAggregation, ParallelAggregation} finds the same
surface; every call runs on the MI355X through librbgpu (no CPU fallback).

  RoaringBitmap.and_/or_/xor/andNot(x1, x2)   RoaringBitmap.java:377, 860, 1071, 444
  RoaringBitmap.*Cardinality(x1, x2)           RoaringBitmap.java:413, 916, 931, 944
  RoaringBitmap.or_(*bitmaps)                   RoaringBitmap.java:844 -> FastAggregation.or
  FastAggregation.and_/or_/xor(*bitmaps)        FastAggregation.java:37, 602, 772
  FastAggregation.naive_and/workShyAnd/...      FastAggregation.java:328, 356, 541, 576
  ParallelAggregation.or_/xor(*bitmaps)         ParallelAggregation.java:161, 182
  serialize / deserialize                       RoaringArray.java:851-940, 276-348

Python reserves `and`/`or`, so those two carry a trailing underscore.  Deserialize errors
raise IOError (FormatError), like the reference's IOException; non-canonical inputs raise
ValueError (InvalidArgument).
"""
from __future__ import annotations

from typing import Iterable, Optional, Sequence

import numpy as np

from . import _lib as L
from .engine import Context, DeviceSet, default_context, soa_from_values


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

    def isEmpty(self) -> bool:
        return self._set.n_containers == 0

    def toArray(self) -> np.ndarray:
        return self._set.download().values(0)

    def runOptimize(self) -> bool:
        """RoaringBitmap.runOptimize (RoaringBitmap.java:2764): re-encode where a Run is smaller."""
        vals = self.toArray()
        soa = soa_from_values([vals], run_optimize=True)
        self._set = default_context().upload_soa(soa)
        return bool((soa.type == L.RUN).any())

    def clone(self) -> "RoaringBitmap":
        return RoaringBitmap.deserialize(self.serialize())

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

    # ---- static pairwise algebra
    @staticmethod
    def _pair(op: int, x1: "RoaringBitmap", x2: "RoaringBitmap") -> "RoaringBitmap":
        return RoaringBitmap(default_context().pairwise(op, x1._set, x2._set, npairs=1))

    @staticmethod
    def and_(x1: "RoaringBitmap", x2: "RoaringBitmap") -> "RoaringBitmap":
        return RoaringBitmap._pair(L.AND, x1, x2)

    @staticmethod
    def xor(x1: "RoaringBitmap", x2: "RoaringBitmap") -> "RoaringBitmap":
        return RoaringBitmap._pair(L.XOR, x1, x2)

    @staticmethod
    def andNot(x1: "RoaringBitmap", x2: "RoaringBitmap") -> "RoaringBitmap":
        return RoaringBitmap._pair(L.ANDNOT, x1, x2)

    @staticmethod
    def or_(*bitmaps) -> "RoaringBitmap":
        if len(bitmaps) == 2 and all(isinstance(b, RoaringBitmap) for b in bitmaps):
            return RoaringBitmap._pair(L.OR, bitmaps[0], bitmaps[1])
        return FastAggregation.or_(*bitmaps)  # RoaringBitmap.or(RoaringBitmap...) (RoaringBitmap.java:844)

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


def _gather(bitmaps: Sequence[RoaringBitmap]) -> DeviceSet:
    ctx = default_context()
    return ctx.upload_serialized([b.serialize() for b in bitmaps])


def _flatten(bitmaps) -> Sequence[RoaringBitmap]:
    if len(bitmaps) == 1 and not isinstance(bitmaps[0], RoaringBitmap):
        return list(bitmaps[0])
    return list(bitmaps)


def _wide(sem: int, bitmaps) -> RoaringBitmap:
    bms = _flatten(bitmaps)
    if not bms:
        return RoaringBitmap()
    return RoaringBitmap(default_context().wide(sem, _gather(bms)))


class FastAggregation:
    """org.roaringbitmap.FastAggregation (FastAggregation.java)."""

    @staticmethod
    def and_(*bitmaps) -> RoaringBitmap:
        return _wide(L.FAST_AND, bitmaps)

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
    def workShyAnd(*bitmaps) -> RoaringBitmap:
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
        """priorityqueue_or(RoaringBitmap...) (FastAggregation.java:675-721): lazy ORs of the two
        smallest bitmaps (getLongSizeInBytes) on the device, the survivor repaired."""
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
        return default_context().wide_cardinality(L.AND, _gather(bms))

    @staticmethod
    def orCardinality(*bitmaps) -> int:
        bms = _flatten(bitmaps)
        if not bms:
            return 0
        if len(bms) == 1:
            return bms[0].getCardinality()
        if len(bms) == 2:
            return RoaringBitmap.orCardinality(bms[0], bms[1])
        return default_context().wide_cardinality(L.OR, _gather(bms))


class ParallelAggregation:
    """org.roaringbitmap.ParallelAggregation (ParallelAggregation.java): key-parallel on the GPU."""

    @staticmethod
    def or_(*bitmaps) -> RoaringBitmap:
        return _wide(L.PAR_OR, bitmaps)

    @staticmethod
    def xor(*bitmaps) -> RoaringBitmap:
        return _wide(L.PAR_XOR, bitmaps)

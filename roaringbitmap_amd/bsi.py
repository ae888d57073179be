"""Host-side mirror of the reference's bit-sliced index (bsi module) for the compare hot path.

  Roaring64BitmapSliceIndex / RoaringBitmapSliceIndex   bsi/src/main/java/org/roaringbitmap/bsi/
    setValue(columnId, value)        longlong/Roaring64BitmapSliceIndex.java:291-326
    compare(op, startOrValue, end, foundSet)              :460-503 (O'Neil, oNeilCompare :410-446)
    getExistenceBitmap / bitCount / runOptimize          :141-168

The slices and the existence bitmap live in HBM as one DeviceSet (slices bA[0..n), then ebM) and a
query runs as one fused MI355X pass per high key (librbgpu rbgpu_bsi_compare).  Values are
unsigned 64-bit; the reference stores Java longs and cannot hold bit 63 (setValue tests
`(value & (1L << i)) > 0`), so the two agree on every value below 2^63.
"""
from __future__ import annotations

from typing import Iterable, Optional, Tuple

import numpy as np

from . import _lib as L
from .engine import DeviceSet, default_context
from .roaring import RoaringBitmap

Operation = type("Operation", (), {"EQ": L.BSI_EQ, "NEQ": L.BSI_NEQ, "LE": L.BSI_LE, "LT": L.BSI_LT,
                                   "GE": L.BSI_GE, "GT": L.BSI_GT, "RANGE": L.BSI_RANGE})


class Roaring64BitmapSliceIndex:
    def __init__(self, min_value: int = 0, max_value: int = 0):
        if min_value < 0:
            raise ValueError("Values should be non-negative")
        self._cols = {}                 # columnId -> value (host staging until the next query)
        self.minValue, self.maxValue = 0, 0
        self._nbits = max(0, int(max_value).bit_length())
        self._dev: Optional[DeviceSet] = None
        self._run_optimized = False

    # ---- construction (setValue semantics, Roaring64BitmapSliceIndex.java:291-326)
    def setValue(self, column_id: int, value: int) -> None:
        if not self._cols:
            self.minValue = self.maxValue = value
            self._nbits = max(self._nbits, max(1, int(value).bit_length()))
        elif self.minValue > value:
            self.minValue = value
        elif self.maxValue < value:
            self.maxValue = value
            self._nbits = max(self._nbits, int(value).bit_length())
        self._cols[int(column_id)] = int(value)
        self._dev = None

    def setValues(self, pairs: Iterable[Tuple[int, int]]) -> None:
        for c, v in pairs:
            self.setValue(c, v)

    @classmethod
    def from_device(cls, dset: DeviceSet, min_value: int, max_value: int) -> "Roaring64BitmapSliceIndex":
        """Wrap a device-resident BSI (slices then ebM), e.g. rbgpu_generate_bsi's."""
        b = cls()
        b._dev, b.minValue, b.maxValue, b._nbits = dset, min_value, max_value, len(dset) - 1
        b._cols = None
        return b

    def runOptimize(self) -> None:
        self._run_optimized = True
        self._dev = None

    def bitCount(self) -> int:
        return self._nbits

    def _device(self) -> DeviceSet:
        if self._dev is None:
            cols = np.fromiter(self._cols.keys(), dtype=np.uint64, count=len(self._cols))
            vals = np.fromiter(self._cols.values(), dtype=np.uint64, count=len(self._cols))
            order = np.argsort(cols)
            cols, vals = cols[order], vals[order]
            bitmaps = [cols[((vals >> np.uint64(i)) & np.uint64(1)) == 1].astype(np.uint32)
                       for i in range(self._nbits)] + [cols.astype(np.uint32)]
            self._dev = default_context().upload_values(bitmaps, run_optimize=self._run_optimized)
        return self._dev

    def getExistenceBitmap(self) -> RoaringBitmap:
        d = self._device()
        return RoaringBitmap(default_context().extract(d, len(d) - 1))

    def getLongCardinality(self) -> int:
        return int(self._device().cardinalities()[-1])

    # ---- the query hot path
    def compare(self, operation: int, start_or_value: int, end: int = 0,
                found_set: Optional[RoaringBitmap] = None) -> RoaringBitmap:
        d = self._device()
        found = found_set._set if found_set is not None else None
        return RoaringBitmap(d.ctx.bsi_compare(operation, d, start_or_value, end, self.minValue, self.maxValue,
                                               found))


RoaringBitmapSliceIndex = Roaring64BitmapSliceIndex  # the 32-bit index runs the same compare

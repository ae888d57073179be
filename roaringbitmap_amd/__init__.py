"""roaringbitmap_amd — MI355X-native engine for RoaringBitmap's set-algebra hot path.

Batched pairwise and/or/xor/andNot and wide FastAggregation / ParallelAggregation run as
hand-written gfx950 HIP kernels in librbgpu.so (C ABI: include/rbgpu.h).  Results are
bit-exact to the Java reference (identical RoaringFormatSpec bytes and cardinalities).
"""
from . import _lib
from ._lib import (AND, ANDNOT, ARRAY, BITMAP, FAST_AND, FAST_OR, FAST_XOR, NAIVE_AND, NAIVE_AND_ITER, OR,
                   PAR_OR, PAR_XOR, RUN, WL_FILTER_POSTING, WL_WIDE_DENSE, WL_WIDE_MIXED, WL_WIDE_RUNS,
                   WORKSHY_AND, XOR, FormatError, InvalidArgument, RbError)
from .engine import Context, DeviceSet, HostSoA, default_context, soa_from_values
from .roaring import (BufferFastAggregation, BufferParallelAggregation, FastAggregation, ParallelAggregation, Roaring64Bitmap,
                      Roaring64NavigableMap, RoaringBitmap)
from .bsi import Operation, Roaring64BitmapSliceIndex, RoaringBitmapSliceIndex
from ._lib import BSI_EQ, BSI_GE, BSI_GT, BSI_LE, BSI_LT, BSI_NEQ, BSI_RANGE
from ._lib import HORIZONTAL_OR, HORIZONTAL_XOR, PQ_OR, PQ_XOR
from ._lib import BUFFER_NAIVE_OR, BUFFER_PQ_OR, BUFFER_PQ_OR_ITER, BUFFER_PQ_XOR
from .engine import Comm, DeviceSet64
from ._lib import RB64_BITMAP, RB64_NAVIGABLE

__all__ = [
    "AND", "OR", "XOR", "ANDNOT", "ARRAY", "BITMAP", "RUN",
    "FAST_OR", "FAST_AND", "WORKSHY_AND", "NAIVE_AND", "FAST_XOR", "PAR_OR", "PAR_XOR", "NAIVE_AND_ITER",
    "HORIZONTAL_OR", "HORIZONTAL_XOR", "PQ_OR", "PQ_XOR", "Comm",
    "BUFFER_NAIVE_OR", "BUFFER_PQ_OR", "BUFFER_PQ_OR_ITER", "BUFFER_PQ_XOR", "BufferFastAggregation", "BufferParallelAggregation",
    "WL_FILTER_POSTING", "WL_WIDE_DENSE", "WL_WIDE_MIXED", "WL_WIDE_RUNS",
    "Context", "DeviceSet", "HostSoA", "default_context", "soa_from_values",
    "RoaringBitmap", "FastAggregation", "ParallelAggregation", "Roaring64Bitmap", "Roaring64NavigableMap",
    "DeviceSet64", "RB64_BITMAP", "RB64_NAVIGABLE",
    "Roaring64BitmapSliceIndex", "RoaringBitmapSliceIndex", "Operation",
    "BSI_EQ", "BSI_NEQ", "BSI_LE", "BSI_LT", "BSI_GE", "BSI_GT", "BSI_RANGE",
    "RbError", "FormatError", "InvalidArgument",
]

"""ctypes binding of the CPU oracle ``librbref.so`` (see rbref.h).

TEST INFRASTRUCTURE ONLY: imported by tests/, __graft_entry__.smoke() and bench.py's
cpu_baseline leg as the parity checker / timed CPU baseline.  The product package
(``roaringbitmap_amd``) never imports this module.
"""
from __future__ import annotations

import ctypes as C
import os
import subprocess

_HERE = os.path.dirname(os.path.abspath(__file__))
_LIB_PATH = os.path.join(_HERE, "librbref.so")

AND, OR, XOR, ANDNOT = 0, 1, 2, 3
(FAST_OR, FAST_AND, WORKSHY_AND, NAIVE_AND, FAST_XOR, PAR_OR, PAR_XOR, NAIVE_AND_ITER, HORIZONTAL_OR, HORIZONTAL_XOR,
 PQ_OR, PQ_XOR, BUFFER_NAIVE_OR, BUFFER_PQ_OR, BUFFER_PQ_OR_ITER, BUFFER_PQ_XOR) = range(16)
ARRAY, BITMAP, RUN = 0, 1, 2


def build() -> str:
    """Compile the oracle in place (gcc is in the image)."""
    subprocess.run(["make", "-s", "-C", _HERE], check=True)
    return _LIB_PATH


def _load():
    if not os.path.exists(_LIB_PATH):
        build()
    lib = C.CDLL(_LIB_PATH)
    P = C.c_void_p
    sig = {
        "rbref_new": (P, []),
        "rbref_free": (None, [P]),
        "rbref_clone": (P, [P]),
        "rbref_bitmap_of": (P, [C.POINTER(C.c_uint32), C.c_size_t]),
        "rbref_run_optimize": (C.c_int, [P]),
        "rbref_cardinality": (C.c_uint64, [P]),
        "rbref_container_count": (C.c_uint32, [P]),
        "rbref_container_info": (C.c_int, [P, C.c_uint32, C.POINTER(C.c_uint16), C.POINTER(C.c_uint8),
                                           C.POINTER(C.c_uint32), C.POINTER(C.c_uint32)]),
        "rbref_to_array": (C.c_uint64, [P, C.POINTER(C.c_uint32), C.c_uint64]),
        "rbref_deserialize": (C.c_int, [C.c_char_p, C.c_size_t, C.POINTER(P)]),
        "rbref_serialized_size": (C.c_uint64, [P]),
        "rbref_serialize": (C.c_int, [P, C.c_void_p, C.c_uint64]),
        "rbref_from_soa": (C.c_int, [C.c_uint32, P, P, P, P, P, P, C.POINTER(P)]),
        "rbref_op": (P, [C.c_int, P, P]),
        "rbref_op_cardinality": (C.c_int64, [C.c_int, P, P]),
        "rbref_op_inplace": (C.c_int, [C.c_int, P, P]),
        "rbref_xor_keep_empty": (P, [P, P]),
        "rbref_wide": (P, [C.c_int, C.POINTER(P), C.c_size_t]),
        "rbref_wide_cardinality": (C.c_int64, [C.c_int, C.POINTER(P), C.c_size_t]),
        "rbref_wide_mt": (P, [C.c_int, C.POINTER(P), C.c_size_t, C.c_int]),
        "rbref_pairwise_batch": (C.c_int, [C.c_int, C.POINTER(P), C.POINTER(P), C.c_size_t, C.c_int,
                                           C.POINTER(C.c_uint64), C.POINTER(C.c_uint64)]),
        "rbref_bsi_compare": (P, [C.POINTER(P), C.c_size_t, P, C.c_int, C.c_uint64, C.c_uint64, P, C.c_uint64,
                                  C.c_uint64]),
        "rbref_bsi_compare_keys": (C.c_uint64, [C.POINTER(P), C.c_size_t, C.c_size_t, C.c_int, C.c_uint64,
                                               C.c_uint64, C.c_uint64, C.c_uint64, C.c_int]),
    }
    for name, (res, args) in sig.items():
        fn = getattr(lib, name)
        fn.restype = res
        fn.argtypes = args
    return lib


_lib = None


def lib():
    global _lib
    if _lib is None:
        _lib = _load()
    return _lib


class RefBitmap:
    """Owning handle to an oracle bitmap."""

    __slots__ = ("h",)

    def __init__(self, handle):
        if not handle:
            raise RuntimeError("null oracle bitmap")
        self.h = handle

    def __del__(self):
        if getattr(self, "h", None) and _lib is not None:
            _lib.rbref_free(self.h)
            self.h = None

    # -- construction
    @classmethod
    def of(cls, values) -> "RefBitmap":
        import numpy as np
        arr = np.ascontiguousarray(np.asarray(values, dtype=np.uint32))
        return cls(lib().rbref_bitmap_of(arr.ctypes.data_as(C.POINTER(C.c_uint32)), arr.size))

    @classmethod
    def deserialize(cls, data: bytes) -> "RefBitmap":
        out = C.c_void_p()
        rc = lib().rbref_deserialize(data, len(data), C.byref(out))
        if rc != 0:
            raise IOError(f"invalid RoaringFormatSpec input (rc={rc})")
        return cls(out.value)

    def clone(self) -> "RefBitmap":
        return RefBitmap(lib().rbref_clone(self.h))

    # -- queries
    def serialize(self) -> bytes:
        n = lib().rbref_serialized_size(self.h)
        buf = C.create_string_buffer(int(n))
        rc = lib().rbref_serialize(self.h, buf, n)
        assert rc == 0
        return buf.raw[: int(n)]

    def cardinality(self) -> int:
        return int(lib().rbref_cardinality(self.h))

    def run_optimize(self) -> bool:
        return bool(lib().rbref_run_optimize(self.h))

    def containers(self):
        """[(key, type, card, nruns)] in key order."""
        out = []
        k, t, c, r = C.c_uint16(), C.c_uint8(), C.c_uint32(), C.c_uint32()
        for i in range(lib().rbref_container_count(self.h)):
            lib().rbref_container_info(self.h, i, C.byref(k), C.byref(t), C.byref(c), C.byref(r))
            out.append((k.value, t.value, c.value, r.value))
        return out

    def to_array(self):
        import numpy as np
        n = self.cardinality()
        arr = np.empty(n, dtype=np.uint32)
        lib().rbref_to_array(self.h, arr.ctypes.data_as(C.POINTER(C.c_uint32)), n)
        return arr


def op(opcode: int, a: RefBitmap, b: RefBitmap) -> RefBitmap:
    return RefBitmap(lib().rbref_op(opcode, a.h, b.h))


def op_cardinality(opcode: int, a: RefBitmap, b: RefBitmap) -> int:
    return int(lib().rbref_op_cardinality(opcode, a.h, b.h))


def xor_keep_empty(a: RefBitmap, b: RefBitmap) -> RefBitmap:
    return RefBitmap(lib().rbref_xor_keep_empty(a.h, b.h))


def op_inplace(opcode: int, a: RefBitmap, b: RefBitmap) -> None:
    assert lib().rbref_op_inplace(opcode, a.h, b.h) == 0


def _handles(bitmaps):
    arr = (C.c_void_p * len(bitmaps))(*[b.h for b in bitmaps])
    return arr


def wide(sem: int, bitmaps) -> RefBitmap:
    h = lib().rbref_wide(sem, _handles(bitmaps), len(bitmaps))
    if not h:  # the reference throws IllegalArgumentException (BufferFastAggregation.priorityqueue_xor)
        raise ValueError("Expecting at least 2 bitmaps")
    return RefBitmap(h)


def wide_mt(sem: int, bitmaps, threads: int) -> RefBitmap:
    """The same aggregation key-parallel on `threads` host threads (rbref_wide_mt)."""
    return RefBitmap(lib().rbref_wide_mt(sem, _handles(bitmaps), len(bitmaps), threads))


def wide_cardinality(opcode: int, bitmaps) -> int:
    return int(lib().rbref_wide_cardinality(opcode, _handles(bitmaps), len(bitmaps)))


def pairwise_batch(opcode: int, a, b, threads: int = 1):
    card, conts = C.c_uint64(), C.c_uint64()
    lib().rbref_pairwise_batch(opcode, _handles(a), _handles(b), len(a), threads, C.byref(card), C.byref(conts))
    return card.value, conts.value


def from_soa(keys, types, cards, nruns, payload, offsets) -> RefBitmap:
    """Build one oracle bitmap from host SoA numpy arrays (one bitmap's slice)."""
    import numpy as np
    keys = np.ascontiguousarray(keys, dtype=np.uint16)
    types = np.ascontiguousarray(types, dtype=np.uint8)
    cards = np.ascontiguousarray(cards, dtype=np.uint32)
    nruns = np.ascontiguousarray(nruns, dtype=np.uint16)
    payload = np.ascontiguousarray(payload, dtype=np.uint8)
    offsets = np.ascontiguousarray(offsets, dtype=np.uint64)
    out = C.c_void_p()
    rc = lib().rbref_from_soa(len(keys), keys.ctypes.data, types.ctypes.data, cards.ctypes.data,
                              nruns.ctypes.data, payload.ctypes.data, offsets.ctypes.data, C.byref(out))
    if rc != 0:
        raise ValueError("bad SoA slice")
    return RefBitmap(out.value)


# ---------------------------------------------------------------------------------------------
# Bit-sliced index (bsi module): a restatement of Roaring64BitmapSliceIndex / RoaringBitmapSliceIndex
# compare on top of the oracle's static container ops (the slices, the existence bitmap and every
# intermediate are RoaringBitmaps combined with the static and/or/andNot, exactly like the
# reference — bsi/src/main/java/org/roaringbitmap/bsi/longlong/Roaring64BitmapSliceIndex.java and
# .../bsi/RoaringBitmapSliceIndex.java).
BSI_EQ, BSI_NEQ, BSI_LE, BSI_LT, BSI_GE, BSI_GT, BSI_RANGE = range(7)  # BitmapSliceIndex.Operation


def bsi_build(columns, values):
    """setValue(column, value) for each pair on a fresh BSI (Roaring64BitmapSliceIndex.java:291-326):
    slices are bitmapOf-built (add() only), bitCount = binary length of the largest value, min/max
    tracked by ensureCapacityInternal.  Values are taken as unsigned 64-bit."""
    import numpy as np
    cols = np.asarray(columns, dtype=np.uint64)
    vals = np.asarray(values, dtype=np.uint64)
    if len(cols) == 0:
        return [], RefBitmap.of(np.zeros(0, np.uint32)), 0, 0
    # last write wins per column (setValue overwrites every slice bit and re-adds to ebM)
    _, last = np.unique(cols[::-1], return_index=True)
    keep = len(cols) - 1 - last
    cols, vals = cols[keep], vals[keep]
    vmax, vmin = int(vals.max()), int(vals.min())
    nbits = max(1, vmax.bit_length())
    slices = [RefBitmap.of(cols[((vals >> np.uint64(i)) & np.uint64(1)) == 1].astype(np.uint32))
              for i in range(nbits)]
    return slices, RefBitmap.of(cols.astype(np.uint32)), vmin, vmax


def _empty():
    import numpy as np
    return RefBitmap.of(np.zeros(0, np.uint32))


def _compare_using_min_max(ebm, op_, start, end, found, vmin, vmax):
    """Roaring64BitmapSliceIndex.compareUsingMinMax (RoaringBitmapSliceIndex.java:505-577)."""
    all_ = ebm.clone() if found is None else op(AND, ebm, found)
    empty = _empty()
    if op_ == BSI_LT:
        if start > vmax:
            return all_
        if start <= vmin:
            return empty
    elif op_ == BSI_LE:
        if start >= vmax:
            return all_
        if start < vmin:
            return empty
    elif op_ == BSI_GT:
        if start < vmin:
            return all_
        if start >= vmax:
            return empty
    elif op_ == BSI_GE:
        if start <= vmin:
            return all_
        if start > vmax:
            return empty
    elif op_ == BSI_EQ:
        if vmin == vmax and vmin == start:
            return all_
        if start < vmin or start > vmax:
            return empty
    elif op_ == BSI_NEQ:
        if vmin == vmax:
            return empty if vmin == start else all_
    elif op_ == BSI_RANGE:
        if start <= vmin and end >= vmax:
            return all_
        if start > vmax or end < vmin:
            return empty
    return None


def _oneil(slices, ebm, op_, predicate, found):
    """oNeilCompare (RoaringBitmapSliceIndex.java:432-472)."""
    fixed = ebm if found is None else found
    gt, lt, eq = _empty(), _empty(), ebm
    for i in range(len(slices) - 1, -1, -1):
        if (predicate >> i) & 1:
            lt = op(OR, lt, op(ANDNOT, eq, slices[i]))
            eq = op(AND, eq, slices[i])
        else:
            gt = op(OR, gt, op(AND, eq, slices[i]))
            eq = op(ANDNOT, eq, slices[i])
    eq = op(AND, fixed, eq)
    if op_ == BSI_EQ:
        return eq
    if op_ == BSI_NEQ:
        return op(ANDNOT, fixed, eq)
    if op_ == BSI_GT:
        return op(AND, gt, fixed)
    if op_ == BSI_LT:
        return op(AND, lt, fixed)
    if op_ == BSI_LE:
        return op(AND, op(OR, lt, eq), fixed)
    if op_ == BSI_GE:
        return op(AND, op(OR, gt, eq), fixed)
    raise ValueError(op_)


def bsi_compare(slices, ebm, op_, start, end, found, vmin, vmax):
    """compare(operation, startOrValue, end, foundSet) (RoaringBitmapSliceIndex.java:475-503)."""
    r = _compare_using_min_max(ebm, op_, start, end, found, vmin, vmax)
    if r is not None:
        return r
    if op_ == BSI_RANGE:
        return op(AND, _oneil(slices, ebm, BSI_GE, start, found), _oneil(slices, ebm, BSI_LE, end, found))
    return _oneil(slices, ebm, op_, start, found)


def bsi_compare_cpp(slices, ebm, op_, start, end, found, vmin, vmax) -> RefBitmap:
    """rbref_bsi_compare: the C++ twin of bsi_compare (the same compareUsingMinMax / oNeilCompare steps over
    the same static ops), which the BSI CPU baseline times without the interpreter in the loop."""
    return RefBitmap(lib().rbref_bsi_compare(_handles(slices), len(slices), ebm.h, op_, start, end,
                                             found.h if found is not None else None, vmin, vmax))


def bsi_compare_keys(per_key, op_, start, end, vmin, vmax, threads: int = 1) -> int:
    """rbref_bsi_compare_keys: per_key = [(slices, ebm)] of independent per-high-key indexes, compared on
    `threads` host threads (contiguous key ranges); the total result cardinality."""
    ns = len(per_key[0][0]) if per_key else 0
    flat = [b for sl, eb in per_key for b in list(sl) + [eb]]
    return int(lib().rbref_bsi_compare_keys(_handles(flat), len(per_key), ns, op_, start, end, vmin, vmax, threads))

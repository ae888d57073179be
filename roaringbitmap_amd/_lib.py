"""ctypes binding of librbgpu.so (include/rbgpu.h).

The HIP extension is the only compute path: importing this module without the built
library raises immediately (there is no CPU fallback in the product).
"""
from __future__ import annotations

import ctypes as C
import os

_HERE = os.path.dirname(os.path.abspath(__file__))
# RBGPU_LIB selects an alternative in-tree build (kernel variants under scripts/ experiments)
LIB_PATH = os.environ.get("RBGPU_LIB") or os.path.join(_HERE, "librbgpu.so")

RB_OK, RB_EFORMAT, RB_EINVAL, RB_ENOMEM, RB_EDEVICE = 0, -1, -2, -3, -4
AND, OR, XOR, ANDNOT = 0, 1, 2, 3
ARRAY, BITMAP, RUN = 0, 1, 2
FAST_OR, FAST_AND, WORKSHY_AND, NAIVE_AND, FAST_XOR, PAR_OR, PAR_XOR, NAIVE_AND_ITER = range(8)
HORIZONTAL_OR, HORIZONTAL_XOR, PQ_OR, PQ_XOR = 8, 9, 10, 11  # global-order semantics (rbgpu.h rb_wide_sem)
# buffer/ (BufferFastAggregation) entry points whose results differ from FastAggregation's
BUFFER_NAIVE_OR, BUFFER_PQ_OR, BUFFER_PQ_OR_ITER, BUFFER_PQ_XOR = 12, 13, 14, 15
PQ_SEMS = (PQ_OR, PQ_XOR, BUFFER_PQ_OR, BUFFER_PQ_OR_ITER, BUFFER_PQ_XOR)  # whole results only
RB64_BITMAP, RB64_NAVIGABLE = 0, 1  # rbgpu.h rb64_flavor: Roaring64Bitmap / Roaring64NavigableMap
EMPTY_BITMAP = 0xFFFFFFFF           # RB_EMPTY_BITMAP pair index
WL_FILTER_POSTING, WL_WIDE_DENSE, WL_WIDE_MIXED, WL_WIDE_RUNS = range(4)
BSI_EQ, BSI_NEQ, BSI_LE, BSI_LT, BSI_GE, BSI_GT, BSI_RANGE = range(7)  # BitmapSliceIndex.Operation


class RbSoa(C.Structure):
    _fields_ = [
        ("n_bitmaps", C.c_uint32),
        ("n_containers", C.c_uint64),
        ("payload_bytes", C.c_uint64),
        ("begin", C.c_void_p),
        ("key", C.c_void_p),
        ("type", C.c_void_p),
        ("card", C.c_void_p),
        ("nruns", C.c_void_p),
        ("offset", C.c_void_p),
        ("payload", C.c_void_p),
    ]


class RbDeviceView(C.Structure):  # rb_device_view: the rb_soa layout with device addresses
    _fields_ = RbSoa._fields_


UNKNOWN_COUNT = 0xFFFFFFFFFFFFFFFF  # RB_UNKNOWN_COUNT


class RbBitmapSummary(C.Structure):
    _fields_ = [("cardinality", C.c_uint64), ("n_containers", C.c_uint64), ("n_run_containers", C.c_uint64),
                ("payload_bytes", C.c_uint64), ("size_in_bytes", C.c_uint64)]


class RbStats(C.Structure):
    _fields_ = [
        ("tasks", C.c_uint64),
        ("input_bytes", C.c_uint64),
        ("output_bytes", C.c_uint64),
        ("result_containers", C.c_uint64),
        ("main_kernel_ms", C.c_double),
        ("main_kernel_bytes", C.c_uint64),
        ("total_ms", C.c_double),
        ("main_kernel", C.c_char * 64),
        ("n_kernels", C.c_uint32),
        ("kernel_name", (C.c_char * 48) * 4),
        ("kernel_ms", C.c_double * 4),
        ("kernel_bytes", C.c_uint64 * 4),
        ("kernel_items", C.c_uint64 * 4),
        ("result_cardinality", C.c_uint64),
        ("call_us", C.c_double),
    ]


class RbShardSummary(C.Structure):
    _fields_ = [("cardinality", C.c_uint64), ("n_containers", C.c_uint64), ("n_run_containers", C.c_uint64),
                ("payload_bytes", C.c_uint64), ("serialized_size", C.c_uint64), ("payload_offset", C.c_uint64),
                ("container_offset", C.c_uint64), ("local_serialized", C.c_uint64)]


COMM_ID_BYTES = 128

# rb_host_transport (rbgpu.h): a caller's host channel for the multi-GPU exchange
HT_ALL_GATHER = C.CFUNCTYPE(C.c_int, C.c_void_p, C.c_void_p, C.c_void_p, C.c_uint64)
HT_ALL_REDUCE = C.CFUNCTYPE(C.c_int, C.c_void_p, C.POINTER(C.c_uint64), C.c_uint32)
HT_SEND = C.CFUNCTYPE(C.c_int, C.c_void_p, C.c_void_p, C.c_uint64, C.c_int)
HT_RECV = C.CFUNCTYPE(C.c_int, C.c_void_p, C.c_void_p, C.c_uint64, C.c_int)


class RbHostTransport(C.Structure):
    _fields_ = [("user", C.c_void_p), ("nranks", C.c_int), ("rank", C.c_int), ("all_gather", HT_ALL_GATHER),
                ("all_reduce_sum_u64", HT_ALL_REDUCE), ("send", HT_SEND), ("recv", HT_RECV)]

# every symbol include/rbgpu.h declares, with its ctypes signature
_P = C.c_void_p
_U32P = C.POINTER(C.c_uint32)
_U64P = C.POINTER(C.c_uint64)
SIGNATURES = {
    "rbgpu_device_count": (C.c_int, []),
    "rbgpu_open": (C.c_int, [C.c_int, C.POINTER(_P)]),
    "rbgpu_close": (None, [_P]),
    "rbgpu_last_error": (C.c_char_p, []),
    "rbgpu_synchronize": (C.c_int, [_P]),
    "rbgpu_get_stats": (C.c_int, [_P, C.POINTER(RbStats)]),
    "rbgpu_set_from_serialized": (C.c_int, [_P, C.POINTER(C.c_char_p), _U64P, C.c_uint32, C.POINTER(_P)]),
    "rbgpu_set_from_serialized_device": (C.c_int, [_P, C.c_void_p, _U64P, C.c_uint32, C.POINTER(_P)]),
    "rbgpu_set_from_soa": (C.c_int, [_P, C.POINTER(RbSoa), C.POINTER(_P)]),
    "rbgpu_set_free": (None, [_P]),
    "rbgpu_set_bitmap_count": (C.c_uint32, [_P]),
    "rbgpu_set_container_count": (C.c_uint64, [_P]),
    "rbgpu_set_payload_capacity": (C.c_uint64, [_P]),
    "rbgpu_set_cardinalities": (C.c_int, [_P, _U64P]),
    "rbgpu_set_serialized_sizes": (C.c_int, [_P, _U64P]),
    "rbgpu_set_serialize": (C.c_int, [_P, C.c_uint32, C.c_uint32, C.c_void_p, C.c_uint64, _U64P]),
    "rbgpu_set_serialize_device": (C.c_int, [_P, C.c_uint32, C.c_uint32, C.c_void_p, C.c_uint64, _U64P]),
    "rbgpu_set_download": (C.c_int, [_P, C.c_uint32, C.c_uint32, C.POINTER(RbSoa)]),
    # index arrays as void* (engine passes plain addresses: see engine._idx_addr)
    "rbgpu_pairwise": (C.c_int, [_P, C.c_int, _P, _P, _P, _P, C.c_uint32, C.POINTER(_P)]),
    "rbgpu_pairwise_cardinality": (C.c_int, [_P, C.c_int, _P, _P, _P, _P, C.c_uint32, _U64P]),
    "rbgpu_pairwise_async": (C.c_int, [_P, C.c_int, _P, _P, _P, _P, C.c_uint32, C.c_void_p, C.POINTER(_P)]),
    "rbgpu_set_wait": (C.c_int, [_P]),
    "rbgpu_set_device_view": (C.c_int, [_P, C.POINTER(RbDeviceView)]),
    "rbgpu_pairwise_inplace": (C.c_int, [_P, C.c_int, _P, _P, _P, _P, C.c_uint32, C.POINTER(_P)]),
    "rbgpu_set_run_optimize": (C.c_int, [_P, C.POINTER(_P), C.c_void_p]),
    "rbgpu_set_setup_stats": (C.c_int, [_P, C.POINTER(C.c_double), _U64P]),
    "rbgpu_set_setup_parts": (C.c_int, [_P, C.POINTER(C.c_double), _U64P]),
    "rbgpu_set64_from_portable": (C.c_int, [_P, C.POINTER(C.c_char_p), _U64P, C.c_uint32, C.POINTER(_P)]),
    "rbgpu_set64_from_buckets": (C.c_int, [_P, _U32P, _U64P, C.c_uint32, C.POINTER(_P)]),
    "rbgpu_set64_free": (None, [_P]),
    "rbgpu_set64_bitmap_count": (C.c_uint32, [_P]),
    "rbgpu_set64_buckets": (C.c_int, [_P, C.c_uint32, _U32P, C.c_uint64, _U64P]),
    "rbgpu_set64_bucket_set": (C.c_int, [_P, C.c_uint32, C.POINTER(_P)]),
    "rbgpu_set64_extract": (C.c_int, [_P, C.c_uint32, C.c_uint32, C.POINTER(_P)]),
    "rbgpu_set64_cardinalities": (C.c_int, [_P, _U64P]),
    "rbgpu_set64_portable_sizes": (C.c_int, [_P, _U64P]),
    "rbgpu_set64_serialize_portable": (C.c_int, [_P, C.c_uint32, C.c_uint32, C.c_void_p, C.c_uint64, _U64P]),
    "rbgpu_set64_from_legacy": (C.c_int, [_P, C.POINTER(C.c_char_p), _U64P, C.c_uint32, C.POINTER(_P)]),
    "rbgpu_set64_legacy_sizes": (C.c_int, [_P, _U64P]),
    "rbgpu_set64_serialize_legacy": (C.c_int, [_P, C.c_uint32, C.c_uint32, C.c_void_p, C.c_uint64, _U64P]),
    "rbgpu_set64_from_art": (C.c_int, [_P, C.POINTER(C.c_char_p), _U64P, C.c_uint32, C.POINTER(_P)]),
    "rbgpu_set64_art_sizes": (C.c_int, [_P, _U64P]),
    "rbgpu_set64_serialize_art": (C.c_int, [_P, C.c_uint32, C.c_uint32, C.c_void_p, C.c_uint64, _U64P]),
    "rbgpu_set64_set_signed_longs": (C.c_int, [_P, C.c_uint32, C.c_int]),
    "rbgpu_set64_get_signed_longs": (C.c_int, [_P, C.c_uint32, C.POINTER(C.c_int)]),
    "rbgpu_pairwise64_cardinality": (C.c_int, [_P, C.c_int, _P, _P, _P, _P, C.c_uint32, _U64P]),
    "rbgpu_pairwise64": (C.c_int, [_P, C.c_int, C.c_int, C.c_int, _P, _P, _P, _P, C.c_uint32, C.POINTER(_P)]),
    "rbgpu_wide": (C.c_int, [_P, C.c_int, _P, _U32P, C.c_uint32, C.POINTER(_P)]),
    "rbgpu_wide_keys": (C.c_int, [_P, C.c_int, _P, _U32P, C.c_uint32, C.c_uint32, C.c_uint32, C.POINTER(_P)]),
    "rbgpu_wide_cardinality": (C.c_int, [_P, C.c_int, _P, _U32P, C.c_uint32, _U64P]),
    "rbgpu_set_key_bytes": (C.c_int, [_P, _U64P]),
    "rbgpu_set_range_counts": (C.c_int, [_P, _U32P, C.c_uint32, C.c_uint32, C.c_uint32, _U64P]),
    "rbgpu_set_type_stats": (C.c_int, [_P, _U64P]),
    "rbgpu_set_summaries": (C.c_int, [_P, C.c_uint32, C.c_uint32, C.POINTER(RbBitmapSummary)]),
    "rbgpu_bsi_compare": (C.c_int, [_P, _P, C.c_int, C.c_uint64, C.c_uint64, C.c_uint64, C.c_uint64, _P,
                                    C.POINTER(_P)]),
    "rbgpu_bsi_compare_keys": (C.c_int, [_P, _P, C.c_int, C.c_uint64, C.c_uint64, C.c_uint64, C.c_uint64, _P,
                                         C.c_uint32, C.c_uint32, C.POINTER(_P)]),
    "rbgpu_generate_bsi_keys": (C.c_int, [_P, C.c_uint32, C.c_uint64, C.c_uint64, C.c_uint32, C.c_uint32,
                                          C.POINTER(_P)]),
    "rbgpu_set_extract": (C.c_int, [_P, C.c_uint32, C.c_uint32, C.POINTER(_P)]),
    "rbgpu_generate_bsi": (C.c_int, [_P, C.c_uint32, C.c_uint64, C.c_uint64, C.POINTER(_P)]),
    "rbgpu_generate_keys": (C.c_int, [_P, C.c_int, C.c_uint32, C.c_uint64, C.c_uint32, C.c_uint32, C.POINTER(_P)]),
    "rbgpu_generate": (C.c_int, [_P, C.c_int, C.c_uint32, C.c_uint64, C.POINTER(_P), C.POINTER(_P)]),
    "rbgpu_comm_unique_id": (C.c_int, [C.c_void_p]),
    "rbgpu_comm_init": (C.c_int, [_P, C.c_void_p, C.c_int, C.c_int, C.POINTER(_P)]),
    "rbgpu_comm_destroy": (None, [_P]),
    "rbgpu_comm_allreduce_sum": (C.c_int, [_P, _U64P, C.c_uint32]),
    "rbgpu_shard_summarize": (C.c_int, [_P, _P, C.POINTER(RbShardSummary)]),
    "rbgpu_comm_init_host": (C.c_int, [_P, C.POINTER(RbHostTransport), C.POINTER(_P)]),
    "rbgpu_shard_summarize_serialized": (C.c_int, [_P, C.c_char_p, C.c_uint64, C.POINTER(RbShardSummary)]),
    "rbgpu_shard_gather_host": (C.c_int, [_P, C.c_char_p, C.c_uint64, C.POINTER(RbShardSummary), C.c_int,
                                          C.c_void_p, C.c_uint64]),
    "rbgpu_comm_naive_and_order": (C.c_int, [_P, _U32P, _U64P, C.c_uint32, C.c_int, _U32P, _U32P]),
    "rbgpu_wide_sharded": (C.c_int, [_P, C.c_int, _P, _U32P, C.c_uint32, C.c_uint32, C.c_uint32, C.POINTER(_P),
                                     C.POINTER(RbShardSummary)]),
    "rbgpu_bsi_compare_sharded": (C.c_int, [_P, _P, C.c_int, C.c_uint64, C.c_uint64, C.c_uint64, C.c_uint64, _P,
                                            C.c_uint32, C.c_uint32, C.POINTER(_P), C.POINTER(RbShardSummary)]),
    "rbgpu_shard_gather_serialized": (C.c_int, [_P, _P, C.POINTER(RbShardSummary), C.c_int, C.c_void_p,
                                                C.c_uint64]),
    "rbgpu_shard_assemble_host": (C.c_int, [C.POINTER(C.c_char_p), _U64P, C.c_uint32, C.c_void_p, C.c_uint64,
                                            _U64P]),
}


class RbError(Exception):
    def __init__(self, code: int, msg: str):
        super().__init__(f"rbgpu error {code}: {msg}")
        self.code = code


class FormatError(RbError, IOError):
    """RB_EFORMAT — the reference throws IOException (InvalidRoaringFormat)."""


class InvalidArgument(RbError, ValueError):
    """RB_EINVAL — the reference throws IllegalArgumentException."""


_lib = None


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            raise ImportError(
                f"{LIB_PATH} is missing: build the HIP extension first "
                "(python -c 'import __graft_entry__ as g; g.build()')")
        # One HIP runtime per process: torch ships its own libamdhip64 under the same soname, and
        # whichever loads first serves both.  Loading torch's first keeps torch.cuda usable beside the
        # library (the reverse order leaves torch reporting "No HIP GPUs are available").
        try:
            import torch  # noqa: F401
        except ImportError:
            pass
        L = C.CDLL(LIB_PATH)
        for name, (res, args) in SIGNATURES.items():
            fn = getattr(L, name)
            fn.restype = res
            fn.argtypes = args
        _lib = L
    return _lib


def check(rc: int) -> None:
    if rc == RB_OK:
        return
    msg = (lib().rbgpu_last_error() or b"").decode(errors="replace")
    if rc == RB_EFORMAT:
        raise FormatError(rc, msg)
    if rc == RB_EINVAL:
        raise InvalidArgument(rc, msg)
    raise RbError(rc, msg)

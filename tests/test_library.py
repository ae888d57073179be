"""The C-ABI library loads on CPU and exports every symbol include/rbgpu.h declares."""
import os
import re

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _declared_symbols():
    txt = open(os.path.join(ROOT, "include", "rbgpu.h")).read()
    return sorted(set(re.findall(r"\b(rbgpu_[a-z0-9_]+)\s*\(", txt)))


def test_header_symbols_exported():
    import roaringbitmap_amd._lib as L
    lib = L.lib()
    declared = _declared_symbols()
    assert len(declared) >= 20
    for name in declared:
        assert hasattr(lib, name), name
    assert set(declared) == set(L.SIGNATURES), "ctypes signatures out of sync with rbgpu.h"


def test_no_device_fails_loudly():
    import roaringbitmap_amd as rb
    if rb.Context.device_count() > 0:
        pytest.skip("a device is visible")
    with pytest.raises(rb.RbError):
        rb.Context(0)


def test_host_soa_builder_round_trip():
    import numpy as np

    import roaringbitmap_amd as rb
    from datasets import synthetic_bitmaps
    bms = synthetic_bitmaps(20, seed=3)
    soa = rb.soa_from_values(bms, run_optimize=True)
    for i, v in enumerate(bms):
        assert np.array_equal(soa.values(i), np.unique(v))
    # canonical typing: Array <= 4096 < Bitmap, Run only when strictly smaller
    for t, c, r in zip(soa.type, soa.card, soa.nruns):
        if t == rb.ARRAY:
            assert c <= 4096
        elif t == rb.BITMAP:
            assert c > 4096
        else:
            assert 2 + 4 * int(r) < min(8192, 2 * int(c))


def test_host_soa_matches_oracle_bytes(oracle):
    """soa_from_values (bitmapOf + runOptimize) builds the same containers as the oracle."""
    import numpy as np

    import roaringbitmap_amd as rb
    from datasets import synthetic_bitmaps
    bms = synthetic_bitmaps(30, seed=11)
    for ro in (False, True):
        soa = rb.soa_from_values(bms, run_optimize=ro)
        for i, v in enumerate(bms):
            ref = oracle.RefBitmap.of(v)
            if ro:
                ref.run_optimize()
            lo, hi = int(soa.begin[i]), int(soa.begin[i + 1])
            got = list(zip(soa.key[lo:hi].tolist(), soa.type[lo:hi].tolist(), soa.card[lo:hi].tolist(),
                           soa.nruns[lo:hi].tolist()))
            assert got == ref.containers()

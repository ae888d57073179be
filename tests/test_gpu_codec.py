"""Device RoaringFormatSpec codec (codec.hip): the GPU parser and writer against the oracle's bytes and
against the host codec (format.cpp, selected with RBGPU_HOST_CODEC=1) — identical sets, bytes and
error codes, including the reference's crash-prone fixtures, truncations and corrupted headers."""
import os

import numpy as np
import pytest
import torch  # loaded before librbgpu initialises HIP: torch bundles its own HIP runtime


from datasets import fixture_bytes, load_realdata

pytestmark = pytest.mark.gpu


def _bitmap_zoo(oracle, rng):
    """Shapes that stress the byte layout: empty, one value, < 4 containers with runs (no offset
    table), odd-cardinality arrays (odd payload starts), Bitmap / full-Run containers, many keys."""
    out = [oracle.RefBitmap.of(np.zeros(0, np.uint32)), oracle.RefBitmap.of(np.array([7], np.uint32))]
    full = np.arange(65536, dtype=np.uint32)
    shapes = [
        np.array([1, 3, 5], np.uint32),
        np.concatenate([full, full + (5 << 16)]),
        np.concatenate([np.arange(100, 300, dtype=np.uint32), (3 << 16) + np.arange(0, 9000, 2, dtype=np.uint32)]),
        np.unique(rng.integers(0, 1 << 22, 40001)).astype(np.uint32),
        np.unique(rng.integers(0, 1 << 31, 3001)).astype(np.uint32),
        np.unique(np.concatenate([np.arange(k << 16, (k << 16) + 5000 + 7 * k) for k in range(9)])).astype(np.uint32),
    ]
    for v in shapes:
        for ro in (False, True):
            r = oracle.RefBitmap.of(v)
            if ro:
                r.run_optimize()
            out.append(r)
    for _ in range(20):
        nk = int(rng.integers(1, 12))
        keys = np.sort(rng.choice(4096, nk, replace=False))
        vals = [((int(k) << 16) + np.unique(rng.integers(0, 65536, int(rng.choice([1, 3, 77, 4095, 4097, 30000])))))
                for k in keys]
        r = oracle.RefBitmap.of(np.concatenate(vals).astype(np.uint32))
        if rng.integers(2):
            r.run_optimize()
        out.append(r)
    return out


def _host_codec(flag: bool):
    if flag:
        os.environ["RBGPU_HOST_CODEC"] = "1"
    else:
        os.environ.pop("RBGPU_HOST_CODEC", None)


def _outcome(ctx, blobs):
    try:
        s = ctx.upload_serialized(blobs)
    except (IOError, ValueError) as e:
        return type(e).__name__
    d = s.download()
    rb_bytes = s.serialize()
    return (d.begin.tolist(), d.key.tolist(), d.type.tolist(), d.card.tolist(), d.nruns.tolist(), rb_bytes)


def test_round_trip_zoo(ctx, oracle):
    rng = np.random.default_rng(11)
    refs = _bitmap_zoo(oracle, rng)
    blobs = [r.serialize() for r in refs]
    s = ctx.upload_serialized(blobs)
    assert s.serialize() == blobs
    assert [int(c) for c in s.cardinalities()] == [r.cardinality() for r in refs]
    # sub-ranges of the set (first / count) as well
    assert s.serialize(3, 7) == blobs[3:10]


def test_device_matches_host_codec(ctx, oracle):
    rng = np.random.default_rng(12)
    blobs = [r.serialize() for r in _bitmap_zoo(oracle, rng)]
    try:
        _host_codec(True)
        want = _outcome(ctx, blobs)
    finally:
        _host_codec(False)
    got = _outcome(ctx, blobs)
    assert got[:6] == want[:6]


def test_fixtures_and_realdata(ctx):
    w, wo = fixture_bytes("bitmapwithruns.bin"), fixture_bytes("bitmapwithoutruns.bin")
    blobs = [w, wo]
    s = ctx.upload_serialized(blobs)
    assert s.serialize() == blobs and list(s.cardinalities()) == [200100, 200100]
    vals = load_realdata("census1881")
    h = ctx.upload_values(vals, run_optimize=True).serialize()
    assert ctx.upload_serialized(h).serialize() == h


def test_errors_match_host_codec(ctx, oracle):
    """Every crash-prone fixture, every truncation of small bitmaps and random header / payload
    corruption: the device parser accepts exactly what the host parser accepts, with equal sets, and
    rejects the rest with the same error class (IOError = RB_EFORMAT, ValueError = RB_EINVAL)."""
    rng = np.random.default_rng(13)
    cases = [[fixture_bytes(f"crashproneinput{i}.bin")] for i in range(1, 9)]
    small = [oracle.RefBitmap.of(np.array([1, 2, 3, 70000, 70001, 1 << 20], np.uint32)),
             oracle.RefBitmap.of(np.arange(0, 200000, 3, dtype=np.uint32))]
    small[0].run_optimize()
    r2 = oracle.RefBitmap.of(np.concatenate([np.arange(k << 16, (k << 16) + 300) for k in range(6)]).astype(np.uint32))
    r2.run_optimize()
    small.append(r2)
    good = small[1].serialize()
    for r in small:
        b = r.serialize()
        cases += [[b[:n]] for n in range(0, min(len(b), 120))]
        cases += [[good, b[: len(b) - k]] for k in (1, 2, 5)]
        for _ in range(60):
            m = bytearray(b)
            pos = int(rng.integers(0, min(len(m), 200)))
            m[pos] ^= 1 << int(rng.integers(0, 8))
            cases.append([good, bytes(m)])
    mism = 0
    for blobs in cases:
        try:
            _host_codec(True)
            want = _outcome(ctx, blobs)
        finally:
            _host_codec(False)
        got = _outcome(ctx, blobs)
        if isinstance(want, str):
            assert got == want, (blobs[-1][:16].hex(), len(blobs[-1]))
        else:
            assert not isinstance(got, str), got
            assert got[:6] == want[:6]
            mism += 1
    assert mism > 10  # some corruptions (payload bits) still parse; they must parse identically


def test_wrong_offset_table_is_ignored_like_the_reference(ctx, oracle):
    """RoaringArray.deserialize skips the offset table: a wrong table still parses (sequential walk)."""
    vals = np.concatenate([np.arange(k << 16, (k << 16) + 10 + k) for k in range(6)]).astype(np.uint32)
    r = oracle.RefBitmap.of(vals)
    b = bytearray(r.serialize())
    n = 6  # no-run format: cookie, size, 4n descriptive, then 4n offsets
    for k in range(n):
        b[8 + 4 * n + 4 * k: 12 + 4 * n + 4 * k] = (12345 + k).to_bytes(4, "little")
    s = ctx.upload_serialized([bytes(b)])
    assert s.cardinalities()[0] == len(vals)
    assert s.serialize() == [r.serialize()]


def test_device_resident_entry_points(ctx, oracle):
    rng = np.random.default_rng(14)
    blobs = [r.serialize() for r in _bitmap_zoo(oracle, rng)]
    offs = np.zeros(len(blobs) + 1, np.uint64)
    offs[1:] = np.cumsum([len(b) for b in blobs])
    src = torch.tensor(np.frombuffer(b"".join(blobs) + b"\0" * 4, np.uint8), device="cuda:0")
    torch.cuda.synchronize()
    s = ctx.upload_serialized_device(src.data_ptr(), offs)
    dst = torch.zeros(int(offs[-1]) + 64, dtype=torch.uint8, device="cuda:0")
    got = s.serialize_device(dst.data_ptr(), dst.numel())
    assert np.array_equal(got, offs)
    host = dst.cpu().numpy().tobytes()
    assert host[: int(offs[-1])] == b"".join(blobs)
    assert host[int(offs[-1]):] == b"\0" * 64  # nothing written past the end
    with pytest.raises(ValueError):
        s.serialize_device(dst.data_ptr(), int(offs[-1]) - 1)

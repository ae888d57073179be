"""Test data: the reference's real-roaring-dataset zips (copied under tests/golden/realdata, read
in zip entry order like ZipRealDataRetriever.fetchBitPositions, real-roaring-dataset/src/main/
java/org/roaringbitmap/ZipRealDataRetriever.java:40-70) and seeded synthetic bitmaps that hit
every container-type branch of the reference's set algebra."""
from __future__ import annotations

import os
import zipfile
from functools import lru_cache

import numpy as np

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")
DATASETS = ["census1881", "census1881_srt", "uscensus2000", "wikileaks-noquotes", "wikileaks-noquotes_srt"]

# jmh/src/test/java/org/roaringbitmap/realdata/RealDataBenchmark{And,Or,Xor,AndNot,WideOrNaive,
# WideAndNaive}Test.java — EXPECTED_RESULTS (sum over consecutive pairs; wide over all bitmaps)
EXPECTED = {
    "census1881": dict(AND=23, OR=2007691, XOR=2007668, ANDNOT=1003836, WIDE_OR=988653, WIDE_AND=0),
    "census1881_srt": dict(AND=206, OR=1360167, XOR=1359961, ANDNOT=679375, WIDE_OR=656346, WIDE_AND=0),
    "uscensus2000": dict(AND=0, OR=11954, XOR=11954, ANDNOT=5970, WIDE_OR=5985, WIDE_AND=0),
    "wikileaks-noquotes": dict(AND=3327, OR=541893, XOR=538566, ANDNOT=271605, WIDE_OR=242540, WIDE_AND=0),
    "wikileaks-noquotes_srt": dict(AND=152, OR=574463, XOR=574311, ANDNOT=286904, WIDE_OR=236436, WIDE_AND=0),
}


@lru_cache(maxsize=None)
def load_realdata(name: str):
    z = zipfile.ZipFile(os.path.join(GOLDEN, "realdata", name + ".zip"))
    out = []
    for info in z.infolist():
        txt = z.read(info).decode().strip()
        vals = np.array([int(x) for x in txt.split(",") if x.strip()], dtype=np.uint32) if txt else \
            np.zeros(0, np.uint32)
        out.append(vals)
    return out


def fixture_bytes(name: str) -> bytes:
    with open(os.path.join(GOLDEN, "testdata", name), "rb") as f:
        return f.read()


def ornot_fuzz_bitmaps() -> tuple:
    """The two serialized bitmaps (l, r) of testdata/ornot-fuzz-failure.json, decoded as
    TestRoaringBitmapOrNot.testBigOrNot does (TestRoaringBitmapOrNot.java:381-390): mixed
    Array/Bitmap/Run containers, disjoint key sets."""
    import base64
    import json
    with open(os.path.join(GOLDEN, "testdata", "ornot-fuzz-failure.json")) as f:
        info = json.load(f)
    return tuple(base64.b64decode(s) for s in info["bitmaps"][:2])


def range_bitmap_bytes(limit: int) -> bytes:
    """RoaringFormatSpec bytes of [0, limit) as Run containers (what RoaringBitmap.add(0, limit)
    yields via Container.rangeOfOnes (Container.java:29-37), which returns a RunContainer above 2 values), written
    directly since 2^32-scale ranges cannot go through a value list."""
    import struct
    assert 0 < limit <= 1 << 32 and (limit - 1) & 0xFFFF >= 2, "last container must hold > 2 values"
    nkeys = (limit - 1 >> 16) + 1
    lens = [0xFFFF] * (nkeys - 1) + [(limit - 1) & 0xFFFF]
    out = [struct.pack("<I", 12347 | (nkeys - 1) << 16), b"\xff" * (nkeys // 8)]
    if nkeys % 8:
        out.append(bytes([(1 << (nkeys % 8)) - 1]))
    out.append(b"".join(struct.pack("<HH", k, ln) for k, ln in enumerate(lens)))
    header = sum(len(b) for b in out)
    if nkeys >= 4:  # NO_OFFSET_THRESHOLD: offsets follow the descriptive header
        header += 4 * nkeys
        out.append(b"".join(struct.pack("<I", header + 6 * k) for k in range(nkeys)))
    out.append(b"".join(struct.pack("<HHH", 1, 0, ln) for ln in lens))
    return b"".join(out)


def _container_values(rng: np.random.Generator, kind: str) -> np.ndarray:
    """Low 16-bit values of one container of a given shape."""
    if kind == "single":
        return np.array([rng.integers(0, 65536)], np.uint32)
    if kind == "tiny":  # < 32 values: hits the |Array| < 32 branches of RunContainer.xor / andNot
        return np.unique(rng.integers(0, 65536, size=int(rng.integers(1, 32)))).astype(np.uint32)
    if kind == "sparse":
        return np.unique(rng.integers(0, 65536, size=int(rng.integers(32, 2000)))).astype(np.uint32)
    if kind in ("a4095", "a4096", "b4097"):
        n = {"a4095": 4095, "a4096": 4096, "b4097": 4097}[kind]
        return np.sort(rng.choice(65536, size=n, replace=False)).astype(np.uint32)
    if kind == "dense":
        p = rng.uniform(0.07, 0.93)
        return np.nonzero(rng.random(65536) < p)[0].astype(np.uint32)
    if kind == "full":
        return np.arange(65536, dtype=np.uint32)
    if kind == "almostfull":
        return np.setdiff1d(np.arange(65536), rng.integers(0, 65536, size=int(rng.integers(1, 5)))).astype(np.uint32)
    if kind in ("runs", "fewruns", "manyruns"):
        nr = {"runs": int(rng.integers(1, 300)), "fewruns": int(rng.integers(1, 6)),
              "manyruns": int(rng.integers(1500, 2500))}[kind]
        cuts = np.sort(rng.choice(65537, size=2 * nr, replace=False))
        vals = [np.arange(cuts[2 * i], cuts[2 * i + 1]) for i in range(nr)]
        v = np.concatenate(vals).astype(np.uint32) if vals else np.zeros(0, np.uint32)
        return v[v < 65536]
    if kind == "contig":  # one contiguous block straddling the 4096 threshold
        s = int(rng.integers(0, 60000))
        return np.arange(s, min(65536, s + int(rng.integers(1, 5000))), dtype=np.uint32)
    raise ValueError(kind)


KINDS = ["single", "tiny", "sparse", "a4095", "a4096", "b4097", "dense", "full", "almostfull",
         "runs", "fewruns", "manyruns", "contig"]


def synthetic_bitmaps(n: int, seed: int, max_keys: int = 6, key_space: int = 10, kinds=KINDS):
    """n bitmaps over a small key space so pairs share keys often; every container shape above."""
    rng = np.random.default_rng(seed)
    out = []
    for _ in range(n):
        nk = int(rng.integers(0, max_keys + 1))
        keys = np.sort(rng.choice(key_space, size=min(nk, key_space), replace=False))
        parts = [(_container_values(rng, kinds[int(rng.integers(0, len(kinds)))]) | (np.uint32(k) << 16))
                 for k in keys]
        out.append(np.concatenate(parts).astype(np.uint32) if parts else np.zeros(0, np.uint32))
    return out

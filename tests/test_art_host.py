"""The product's Roaring64Bitmap ART codec (roaringbitmap_amd/csrc/set64.hip, the host-only part between
its "ART codec" markers) compiled alone with g++ and driven on the CPU against the oracle's restatement
(oracle/rbref64.py): the canonical emit equals the oracle's bytes for trees of every node type, and the
parser returns the oracle's containers for canonical streams and for other container-slot layouts.
Parity unpinned (no reference fixture of the format, see test_oracle64.test_oracle64_art_format)."""
import ctypes as C
import os
import subprocess

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SRC = os.path.join(ROOT, "roaringbitmap_amd", "csrc", "set64.hip")

HARNESS = r"""
#include <algorithm>
#include <cstdint>
#include <cstring>
#include <vector>
#include "rbgpu.h"
namespace {
uint32_t rd32(const uint8_t *p) { uint32_t v; std::memcpy(&v, p, 4); return v; }
uint16_t rd16(const uint8_t *p) { uint16_t v; std::memcpy(&v, p, 2); return v; }
uint64_t payload_bytes(int t, uint32_t card, uint32_t nruns) {
  return t == RB_ARRAY ? 2ull * card : t == RB_BITMAP ? 8192ull : 4ull * nruns;
}
%s
}
extern "C" {
// containers in ascending 48-bit key order -> the stream (returns its size; writes when dst)
uint64_t h_emit(uint64_t n, const uint64_t *key, const uint8_t *type, const uint32_t *card, const uint16_t *nruns,
                const uint64_t *off, const uint8_t *payload, uint8_t *dst) {
  std::vector<uint64_t> begin{0, n};
  std::vector<uint16_t> k16(n + 1);
  rb_soa soa{1, n, 0, begin.data(), k16.data(), const_cast<uint8_t *>(type), const_cast<uint32_t *>(card),
             const_cast<uint16_t *>(nruns), const_cast<uint64_t *>(off), const_cast<uint8_t *>(payload)};
  ArtView v;
  for (uint64_t i = 0; i < n; ++i) { v.key.push_back(key[i]); v.cont.push_back(i); }
  return art_stream(v, soa, dst);
}
// the stream -> container count (or -1), and when key != NULL the containers
int64_t h_parse(const uint8_t *p, uint64_t len, uint64_t *key, uint8_t *type, uint32_t *card, uint16_t *nruns,
                uint64_t *at) {
  std::vector<ArtCont> out;
  if (art_parse(p, len, out)) return -1;
  for (size_t i = 0; key && i < out.size(); ++i) {
    key[i] = out[i].key; type[i] = out[i].t; card[i] = out[i].card; nruns[i] = out[i].nr;
    at[i] = (uint64_t)(out[i].payload - p);
  }
  return (int64_t)out.size();
}
}
"""


@pytest.fixture(scope="module")
def codec(tmp_path_factory):
    src = open(SRC).read()
    a = src.index("// ---- ART codec (host only")
    b = src.index("// ---- end of the ART codec")
    d = tmp_path_factory.mktemp("art")
    cpp, so = d / "art.cpp", d / "art.so"
    cpp.write_text(HARNESS % src[a:b])
    subprocess.run(["g++", "-std=c++17", "-O1", "-shared", "-fPIC", "-I", os.path.join(ROOT, "include"),
                    str(cpp), "-o", str(so)], check=True)
    L = C.CDLL(str(so))
    L.h_emit.restype = C.c_uint64
    L.h_parse.restype = C.c_int64
    return L


def _conts(ref):
    """The oracle's containers of a Ref64 in key order: (key48, type, card, nruns, payload)."""
    from oracle import rbref64 as R64
    out = []
    for h, b in ref.buckets:
        for k, t, c, nr, p in R64._containers_of(b.serialize(), b.containers()):
            out.append(((h << 16) | k, t, c, nr, p))
    return out


def _emit(L, conts):
    n = len(conts)
    key = np.array([c[0] for c in conts] or [0], np.uint64)
    typ = np.array([c[1] for c in conts] or [0], np.uint8)
    card = np.array([c[2] for c in conts] or [0], np.uint32)
    nr = np.array([c[3] for c in conts] or [0], np.uint16)
    off = np.cumsum([0] + [len(c[4]) for c in conts])[:max(n, 1)].astype(np.uint64)
    pay = np.frombuffer(b"".join(c[4] for c in conts) + b"\0" * 16, np.uint8)
    args = [n] + [x.ctypes.data_as(C.c_void_p) for x in (key, typ, card, nr, off, pay)]
    size = L.h_emit(*args, None)
    dst = (C.c_uint8 * size)()
    assert L.h_emit(*args, dst) == size
    return bytes(dst)


def _parse(L, data):
    buf = np.frombuffer(data, np.uint8)
    n = L.h_parse(buf.ctypes.data_as(C.c_void_p), len(data), None, None, None, None, None)
    if n < 0:
        return None
    m = max(n, 1)
    key, typ, card = np.zeros(m, np.uint64), np.zeros(m, np.uint8), np.zeros(m, np.uint32)
    nr, at = np.zeros(m, np.uint16), np.zeros(m, np.uint64)
    L.h_parse(buf.ctypes.data_as(C.c_void_p), len(data), *[x.ctypes.data_as(C.c_void_p) for x in (key, typ, card, nr, at)])
    out = []
    for i in range(n):
        t, c, r = int(typ[i]), int(card[i]), int(nr[i])
        size = 2 * c if t == 0 else 8192 if t == 1 else 4 * r
        out.append((int(key[i]), t, c, r, data[int(at[i]):int(at[i]) + size]))
    return out


def test_art_codec_matches_oracle(codec):
    from oracle import rbref64 as R64
    from test_oracle64 import _art_sets
    for r in _art_sets():
        conts = _conts(r)
        data = r.to_art()
        assert _emit(codec, conts) == data
        assert _parse(codec, data) == conts
        n = len(conts)
        if n > 1:  # another slot layout (null slots, permuted indices): the same containers
            slots = list(np.random.default_rng(n).permutation(n + 5)[:n])
            assert _parse(codec, r.to_art(slots=slots, cap=n + 5)) == conts
        for cut in (1, len(data) // 2, len(data) - 1):
            if cut < len(data) and len(data) > 1:
                assert _parse(codec, data[:cut]) is None
    # a kept-empty xor container (card 0, an Array with no values) is written and read as such
    x = R64.bitmap_op(R64.XOR, R64.Ref64.of([1, 2, 1 << 40]), R64.Ref64.of([1, 2]), False)
    conts = _conts(x)
    assert any(c[2] == 0 for c in conts)
    assert _emit(codec, conts) == x.to_art() and _parse(codec, x.to_art()) == conts

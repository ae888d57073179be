"""Pure-Python model of the wave64 algorithms in roaringbitmap_amd/csrc/wave.hpp.

It replays, lane by lane, the register layout (lane L holds container words 128k + 2L + h
in w[2k+h]), the cross-lane scans and the rank arithmetic the kernels use, so the index
logic can be checked on the CPU against plain set arithmetic (tests/test_wave_model.py).
"""
from __future__ import annotations

import numpy as np

M64 = (1 << 64) - 1


def to_lanes(words):
    return [[int(words[128 * (j >> 1) + 2 * L + (j & 1)]) for j in range(16)] for L in range(64)]


def from_lanes(W):
    words = [0] * 1024
    for L in range(64):
        for j in range(16):
            words[128 * (j >> 1) + 2 * L + (j & 1)] = W[L][j]
    return words


def bits_to_words(bits):
    return [int(x) for x in np.packbits(np.asarray(bits, np.uint8), bitorder="little").view(np.uint64)]


def prefix_xor64(x):
    for s in (1, 2, 4, 8, 16, 32):
        x ^= (x << s) & M64
    return x


def expand_runs(runs):
    """Toggle start and end+1 of every run, then prefix-xor with the wave parity carry."""
    t = [0] * 1024
    for s, ln in runs:
        t[s >> 6] ^= 1 << (s & 63)
        e1 = s + ln + 1
        if e1 < 65536:
            t[e1 >> 6] ^= 1 << (e1 & 63)
    T = to_lanes(t)
    q = [0] * 64
    p0 = [0] * 64
    for L in range(64):
        for k in range(8):
            a = bin(T[L][2 * k]).count("1") & 1
            b = bin(T[L][2 * k + 1]).count("1") & 1
            q[L] |= (a ^ b) << k
            p0[L] |= a << k
    incl = [0] * 64
    acc = 0
    for L in range(64):
        acc ^= q[L]
        incl[L] = acc
    tot = incl[63]
    W = [[0] * 16 for _ in range(64)]
    for L in range(64):
        excl = incl[L] ^ q[L]
        for k in range(8):
            rowc = bin(tot & ((1 << k) - 1)).count("1") & 1
            c0 = rowc ^ ((excl >> k) & 1)
            c1 = c0 ^ ((p0[L] >> k) & 1)
            W[L][2 * k] = prefix_xor64(T[L][2 * k]) ^ (M64 if c0 else 0)
            W[L][2 * k + 1] = prefix_xor64(T[L][2 * k + 1]) ^ (M64 if c1 else 0)
    return W


def _neighbours(W):
    top1 = [sum(((W[L][2 * k + 1] >> 63) & 1) << k for k in range(8)) for L in range(64)]
    bot0 = [sum((W[L][2 * k] & 1) << k for k in range(8)) for L in range(64)]
    prev_top = [top1[L - 1] if L else ((top1[63] << 1) & 0xFE) for L in range(64)]
    next_bot = [bot0[L + 1] if L < 63 else ((bot0[0] >> 1) & 0x7F) for L in range(64)]
    return prev_top, next_bot


def _starts(W, prev_top, L, j):
    k, w = j >> 1, W[L][j]
    prev = (W[L][j - 1] >> 63) if (j & 1) else ((prev_top[L] >> k) & 1)
    return w & ~(((w << 1) & M64) | prev) & M64


def _ends(W, next_bot, L, j):
    k, w = j >> 1, W[L][j]
    nxt = ((next_bot[L] >> k) & 1) if (j & 1) else (W[L][j + 1] & 1)
    return w & ~((w >> 1) | (nxt << 63)) & M64


def _bits(x):
    while x:
        b = (x & -x).bit_length() - 1
        yield b
        x &= x - 1


def metrics(W):
    prev_top, _ = _neighbours(W)
    c = sum(bin(W[L][j]).count("1") for L in range(64) for j in range(16))
    r = sum(bin(_starts(W, prev_top, L, j)).count("1") for L in range(64) for j in range(16))
    return c, r


def emit_array(W):
    n = [[bin(W[L][2 * k]).count("1") + bin(W[L][2 * k + 1]).count("1") for k in range(8)] for L in range(64)]
    tot = [sum(n[L][k] for L in range(64)) for k in range(8)]
    out = {}
    for L in range(64):
        rowoff = 0
        for k in range(8):
            pos = rowoff + sum(n[l][k] for l in range(L))
            rowoff += tot[k]
            for h in range(2):
                base = (128 * k + 2 * L + h) << 6
                for b in _bits(W[L][2 * k + h]):
                    out[pos] = base + b
                    pos += 1
    return [out[i] for i in range(len(out))]


def emit_runs(W):
    prev_top, next_bot = _neighbours(W)
    ns = [[bin(_starts(W, prev_top, L, 2 * k)).count("1") + bin(_starts(W, prev_top, L, 2 * k + 1)).count("1")
           for k in range(8)] for L in range(64)]
    tot = [sum(ns[L][k] for L in range(64)) for k in range(8)]
    S, E = {}, {}
    for L in range(64):
        rowoff = 0
        for k in range(8):
            sp = rowoff + sum(ns[l][k] for l in range(L))
            rowoff += tot[k]
            for h in range(2):
                j = 2 * k + h
                open_ = ((W[L][j - 1] >> 63) if h else ((prev_top[L] >> k) & 1)) & (W[L][j] & 1)
                ep = sp - open_
                base = (128 * k + 2 * L + h) << 6
                for b in _bits(_starts(W, prev_top, L, j)):
                    S[sp] = base + b
                    sp += 1
                for b in _bits(_ends(W, next_bot, L, j)):
                    E[ep] = base + b
                    ep += 1
    return [(S[i], E[i] - S[i]) for i in range(len(S))]

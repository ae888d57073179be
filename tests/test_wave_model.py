"""CPU check of the wave64 index arithmetic of csrc/wave.hpp through its Python model."""
import numpy as np
import pytest

import wave_model as WM


def _true_runs(bits):
    d = np.diff(np.concatenate([[0], bits.astype(np.int8), [0]]))
    s, e = np.nonzero(d == 1)[0], np.nonzero(d == -1)[0] - 1
    return [(int(a), int(b - a)) for a, b in zip(s, e)]


def _random_bits(rng, kind):
    if kind == "runs":
        nr = int(rng.integers(1, 2000))
        cuts = np.sort(rng.choice(65537, size=2 * nr, replace=False))
        bits = np.zeros(65536, bool)
        for i in range(nr):
            bits[cuts[2 * i]:cuts[2 * i + 1]] = True
        return bits
    if kind == "dense":
        return rng.random(65536) < rng.uniform(0.05, 0.95)
    if kind == "sparse":
        bits = np.zeros(65536, bool)
        bits[rng.integers(0, 65536, size=int(rng.integers(1, 4096)))] = True
        return bits
    if kind == "word_edges":  # runs that start / end exactly on 64-bit word boundaries
        bits = np.zeros(65536, bool)
        for w in rng.choice(1024, size=40, replace=False):
            a = int(w) * 64
            bits[a:a + 64 * int(rng.integers(1, 3))] = True
        return bits
    if kind == "full":
        return np.ones(65536, bool)
    raise ValueError(kind)


@pytest.mark.parametrize("kind", ["runs", "dense", "sparse", "word_edges", "full"])
def test_emission_and_metrics(kind):
    rng = np.random.default_rng(sum(map(ord, kind)))
    for _ in range(3):
        bits = _random_bits(rng, kind)
        W = WM.to_lanes(WM.bits_to_words(bits))
        c, r = WM.metrics(W)
        runs = _true_runs(bits)
        assert c == int(bits.sum()) and r == len(runs)
        assert WM.emit_runs(W) == runs
        if c <= 4096:
            assert WM.emit_array(W) == np.nonzero(bits)[0].tolist()


def test_run_expansion_matches_bits():
    rng = np.random.default_rng(9)
    for kind in ("runs", "word_edges", "full"):
        bits = _random_bits(rng, kind)
        W = WM.expand_runs(_true_runs(bits))
        assert WM.from_lanes(W) == WM.bits_to_words(bits)

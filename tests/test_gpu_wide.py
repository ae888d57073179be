"""Parity of the wide aggregations (FastAggregation / ParallelAggregation) with the oracle."""
import numpy as np
import pytest

from datasets import DATASETS, EXPECTED, load_realdata, synthetic_bitmaps

pytestmark = pytest.mark.gpu
SEMS = ["FAST_OR", "FAST_AND", "WORKSHY_AND", "NAIVE_AND", "FAST_XOR", "PAR_OR", "PAR_XOR", "NAIVE_AND_ITER"]


def _check(ctx, oracle, s, refs, sem_name, members):
    import roaringbitmap_amd as rb
    sem = getattr(rb, sem_name)
    got = ctx.wide(sem, s, members).serialize()[0]
    want = oracle.wide(getattr(oracle, sem_name), [refs[m] for m in members]).serialize()
    assert got == want, (sem_name, list(members)[:12])


@pytest.mark.parametrize("name", DATASETS)
def test_realdata_wide(ctx, oracle, name):
    import roaringbitmap_amd as rb
    for ro in (False, True):
        s = ctx.upload_values(load_realdata(name), run_optimize=ro)
        refs = [oracle.RefBitmap.deserialize(b) for b in s.serialize()]
        allm = np.arange(len(refs), dtype=np.uint32)
        for sem in SEMS:
            _check(ctx, oracle, s, refs, sem, allm)
        assert int(ctx.wide(rb.FAST_OR, s).cardinalities()[0]) == EXPECTED[name]["WIDE_OR"]
        assert int(ctx.wide(rb.FAST_AND, s).cardinalities()[0]) == EXPECTED[name]["WIDE_AND"]
        assert ctx.wide_cardinality(rb.OR, s) == EXPECTED[name]["WIDE_OR"]
        # a window of consecutive bitmaps, where AND results are non-empty
        for lo in (0, 50, 120):
            win = allm[lo:lo + 3]
            for sem in SEMS:
                _check(ctx, oracle, s, refs, sem, win)


@pytest.mark.parametrize("seed", [5, 6, 7, 8])
def test_synthetic_wide_all_semantics(ctx, oracle, seed):
    bms = synthetic_bitmaps(60, seed=seed, max_keys=6, key_space=6)
    rng = np.random.default_rng(seed)
    for ro in (False, True):
        s = ctx.upload_values(bms, run_optimize=ro)
        refs = [oracle.RefBitmap.deserialize(b) for b in s.serialize()]
        for n in (1, 2, 3, 5, 11, 15, 16, 17, 40):
            members = rng.integers(0, len(bms), size=n).astype(np.uint32)  # duplicates allowed
            for sem in SEMS:
                _check(ctx, oracle, s, refs, sem, members)


def test_runs_only_chains(ctx, oracle):
    """Run-heavy keys shared by every bitmap: exercises EFF in the xor / and chains and the
    lazyIOR Run states of ParallelAggregation.or."""
    rng = np.random.default_rng(3)
    bms = []
    for _ in range(24):
        parts = []
        for k in range(3):
            core = int(rng.integers(0, 60000))
            v = [np.arange(core, core + 2048)]
            for _ in range(int(rng.integers(0, 6))):
                a = int(rng.integers(0, 65000))
                v.append(np.arange(a, a + int(rng.integers(1, 300))))
            parts.append((np.unique(np.concatenate(v)) % 65536).astype(np.uint32) | np.uint32(k << 16))
        bms.append(np.concatenate(parts))
    s = ctx.upload_values(bms, run_optimize=True)
    refs = [oracle.RefBitmap.deserialize(b) for b in s.serialize()]
    for n in (2, 4, 8, 12, 15, 16, 24):
        members = np.arange(n, dtype=np.uint32)
        for sem in SEMS:
            _check(ctx, oracle, s, refs, sem, members)


def test_generated_wide_or_sample(ctx, oracle):
    """Device-generated config-3 shape (reduced): FAST_OR over 64 dense bitmaps."""
    import roaringbitmap_amd as rb
    a, _ = ctx.generate(rb.WL_WIDE_MIXED, 24, seed=9)
    refs = [oracle.RefBitmap.deserialize(b) for b in a.serialize()]
    for sem in ("FAST_OR", "PAR_OR", "FAST_XOR", "PAR_XOR", "FAST_AND"):
        _check(ctx, oracle, a, refs, sem, np.arange(24, dtype=np.uint32))

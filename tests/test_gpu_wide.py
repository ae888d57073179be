"""Parity of the wide aggregations (FastAggregation / ParallelAggregation) with the oracle."""
import numpy as np
import pytest

from datasets import DATASETS, EXPECTED, load_realdata, synthetic_bitmaps

pytestmark = pytest.mark.gpu
SEMS = ["FAST_OR", "FAST_AND", "WORKSHY_AND", "NAIVE_AND", "FAST_XOR", "PAR_OR", "PAR_XOR", "NAIVE_AND_ITER",
        "HORIZONTAL_OR", "HORIZONTAL_XOR", "PQ_OR", "PQ_XOR",
        "BUFFER_NAIVE_OR", "BUFFER_PQ_OR", "BUFFER_PQ_OR_ITER", "BUFFER_PQ_XOR"]
PQ = ("PQ_OR", "PQ_XOR", "BUFFER_PQ_OR", "BUFFER_PQ_OR_ITER", "BUFFER_PQ_XOR")
SHARDABLE = [x for x in SEMS if x not in PQ]  # priorityqueue_or/xor: whole results only


def _check(ctx, oracle, s, refs, sem_name, members):
    import roaringbitmap_amd as rb
    sem = getattr(rb, sem_name)
    try:
        want = oracle.wide(getattr(oracle, sem_name), [refs[m] for m in members]).serialize()
    except ValueError:  # BufferFastAggregation.priorityqueue_xor below 2 bitmaps
        with pytest.raises(rb.InvalidArgument):
            ctx.wide(sem, s, members)
        return
    got = ctx.wide(sem, s, members).serialize()[0]
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


def test_key_range_shards_reassemble(ctx, oracle):
    """rbgpu_wide_keys over a byte-balanced partition, concatenated in key order, gives the
    single-call result byte for byte; NAIVE_AND via the globally ordered member list."""
    import roaringbitmap_amd as rb
    from roaringbitmap_amd.sharding import partition_keys, serialize_parts
    bms = synthetic_bitmaps(40, seed=31, max_keys=8, key_space=12)
    s = ctx.upload_values(bms, run_optimize=True)
    kb = s.key_bytes()
    refs = [oracle.RefBitmap.deserialize(b) for b in s.serialize()]
    for n in (8, 11, 17):
        members = np.arange(n, dtype=np.uint32)
        for sem in SHARDABLE:
            want_bm = oracle.wide(getattr(oracle, sem), [refs[m] for m in members])
            want = want_bm.serialize()
            mem, sem_shard = members, getattr(rb, sem)
            if sem == "NAIVE_AND" or (sem == "FAST_AND" and n <= 10):
                sizes = [len(refs[m].containers()) for m in members]
                first = int(np.argmin(sizes))  # the smallest, first on ties (FastAggregation.java:328-346)
                mem = np.array([members[first]] + [m for i, m in enumerate(members) if i != first], np.uint32)
                sem_shard = rb.NAIVE_AND_ITER
            for parts in (3, 5):
                if sem == "NAIVE_AND":  # the ranks' range counts sum to the container counts
                    cnt = sum(s.range_counts(members, r) for r in partition_keys(kb, parts))
                    assert cnt.tolist() == [len(refs[m].containers()) for m in members]
                shards = [ctx.wide(sem_shard, s, mem, key_range=r) for r in partition_keys(kb, parts)]
                got = serialize_parts([sh.download() for sh in shards])
                assert got == want, (sem, n, parts)
                summ = [sh.summaries()[0] for sh in shards]
                assert sum(x["cardinality"] for x in summ) == want_bm.cardinality()


def test_generated_key_shards_equal_full_dataset(ctx):
    """rbgpu_generate_keys: shards of a partition hold exactly the full dataset's containers."""
    import roaringbitmap_amd as rb
    for wl in (rb.WL_WIDE_DENSE, rb.WL_WIDE_MIXED, rb.WL_WIDE_RUNS):
        n = 3 if wl == rb.WL_WIDE_RUNS else 8
        full, _ = ctx.generate(wl, n, seed=17)
        hf = full.download()
        ranges = [(0, 1000), (1000, 40000), (40000, 65536)]
        shards = [ctx.generate_keys(wl, n, lo, hi, seed=17).download() for lo, hi in ranges]
        for b in range(n):
            want = [hf.container_payload(i).tobytes() + bytes([hf.type[i]]) + int(hf.key[i]).to_bytes(2, "little")
                    for i in range(int(hf.begin[b]), int(hf.begin[b + 1]))]
            got = []
            for h in shards:
                got += [h.container_payload(i).tobytes() + bytes([h.type[i]]) + int(h.key[i]).to_bytes(2, "little")
                        for i in range(int(h.begin[b]), int(h.begin[b + 1]))]
            assert got == want, (wl, b)


def test_run_fastpath_config4_shape(ctx, oracle):
    """Config-4 shape (every key, Run containers with a shared core run + <= 7 random runs): the
    Run-list fast path (wide_runs.hip) must give the oracle's bytes for naive_or / workShyAnd /
    naive_xor, and the same bytes as the generic per-key kernel."""
    import os

    import roaringbitmap_amd as rb
    a, _ = ctx.generate(rb.WL_WIDE_RUNS, 24, seed=3)
    refs = [oracle.RefBitmap.deserialize(b) for b in a.serialize()]
    members = np.arange(24, dtype=np.uint32)
    for sem in ("FAST_OR", "FAST_AND", "WORKSHY_AND", "FAST_XOR", "PAR_XOR"):
        want = oracle.wide(getattr(oracle, sem), [refs[m] for m in members]).serialize()
        got = ctx.wide(getattr(rb, sem), a, members).serialize()[0]
        assert got == want, sem
        os.environ["RBGPU_NO_RUN_FASTPATH"] = "1"
        try:
            assert ctx.wide(getattr(rb, sem), a, members).serialize()[0] == want, sem
        finally:
            del os.environ["RBGPU_NO_RUN_FASTPATH"]
    # a subset and odd counts (workShyAnd vs naive_and switch at 10, xor removals)
    for n in (2, 3, 11):
        sub = members[:n]
        for sem in ("FAST_OR", "FAST_AND", "FAST_XOR"):
            want = oracle.wide(getattr(oracle, sem), [refs[m] for m in sub]).serialize()
            assert ctx.wide(getattr(rb, sem), a, sub).serialize()[0] == want, (sem, n)


def test_run_fastpath_mixed_keys_fall_back(ctx, oracle):
    """Keys where some container is not a small Run (Array, Bitmap, > 8 runs) are routed to the
    generic kernel inside the same call; XOR chains that empty a key mid-way remove it."""
    import roaringbitmap_amd as rb
    rng = np.random.default_rng(9)
    bms = []
    for i in range(30):
        parts = []
        for k in range(8):
            if k < 4:  # small-run keys: shared core + few runs; some identical -> XOR cancels
                core = 1000 * k
                v = [np.arange(core, core + 700)]
                for _ in range(int(rng.integers(0, 4))):
                    s = int(rng.integers(0, 65000))
                    v.append(np.arange(s, s + int(rng.integers(1, 200))))
                if i % 5 == 0:
                    v = [np.arange(core, core + 700)]
            else:      # mixed keys
                kind = ["a4095", "dense", "runs", "fewruns"][(i + k) % 4]
                from datasets import _container_values
                v = [_container_values(rng, kind)]
            parts.append((np.unique(np.concatenate(v)) % 65536).astype(np.uint32) | np.uint32(k << 16))
        bms.append(np.concatenate(parts))
    s = ctx.upload_values(bms, run_optimize=True)
    refs = [oracle.RefBitmap.deserialize(b) for b in s.serialize()]
    for n in (2, 5, 12, 30):
        members = np.arange(n, dtype=np.uint32)
        for sem in ("FAST_OR", "FAST_AND", "WORKSHY_AND", "FAST_XOR"):
            want = oracle.wide(getattr(oracle, sem), [refs[m] for m in members]).serialize()
            assert ctx.wide(getattr(rb, sem), s, members).serialize()[0] == want, (sem, n)


def test_tiled_grouping_keeps_member_order(ctx, oracle):
    """Containers are grouped by key with a counting sort over (member block x key range) tiles;
    with tiny tiles (many member blocks and key ranges, ragged last tiles, duplicate members) every
    semantics must still match the oracle byte for byte, also over a key sub-range."""
    import os

    import roaringbitmap_amd as rb
    a, _ = ctx.generate(rb.WL_WIDE_MIXED, 20, seed=13)
    refs = [oracle.RefBitmap.deserialize(b) for b in a.serialize()]
    members = np.array(list(range(20)) + [3, 7], dtype=np.uint32)
    wants = {sem: oracle.wide(getattr(oracle, sem), [refs[m] for m in members]).serialize() for sem in SEMS}
    for tile in ("3,100", "1,256", "7,33", "64,1"):
        os.environ["RBGPU_GROUP_TILE"] = tile
        try:
            for sem in SEMS:
                assert ctx.wide(getattr(rb, sem), a, members).serialize()[0] == wants[sem], (sem, tile)
            got = ctx.wide(rb.FAST_XOR, a, members, key_range=(1234, 40000)).download()
            full = oracle.RefBitmap.deserialize(wants["FAST_XOR"])
            keys = [int(k) for k in got.key]
            assert all(1234 <= k < 40000 for k in keys)
            want_c = [(k, t, c) for k, t, c, _ in full.containers() if 1234 <= k < 40000]
            assert list(zip(keys, got.type.tolist(), got.card.tolist())) == want_c, tile
        finally:
            del os.environ["RBGPU_GROUP_TILE"]


def test_workshy_and_lane_lists(ctx, oracle):
    """Lane-parallel workShyAnd (k_wide_runs_and): long member chains (several steps per lane, the
    early exit once every list is empty), every LR result type straight from the interval lists
    (full container -> Run, > 4096 -> Bitmap, <= 4096 -> Array, empty -> dropped), and list
    overflow (> 16 intervals) routed to the generic kernel."""
    rng = np.random.default_rng(21)
    nb, nkeys = 150, 40
    per_key = [[] for _ in range(nb)]
    for k in range(nkeys):
        kind = k % 5
        holes_all = rng.choice(65000, size=(nb, 7), replace=True)
        for b in range(nb):
            if kind == 0:    # full container in every bitmap -> AND is full -> Run(0, 65535)
                v = np.arange(65536)
            elif kind == 1:  # big ranges with 7 small holes each -> > 4096 values, > 16 intervals
                keep = np.ones(65536, bool)
                for h in holes_all[b]:
                    keep[h:h + 5] = False
                v = np.nonzero(keep)[0]
            elif kind == 2:  # a shared core of 3000 + random extra runs -> Array
                parts = [np.arange(20000, 23000)]
                for _ in range(int(rng.integers(0, 7))):
                    s0 = int(rng.integers(0, 65000))
                    parts.append(np.arange(s0, s0 + int(rng.integers(1, 300))))
                v = np.unique(np.concatenate(parts))
            elif kind == 3:  # two disjoint families -> AND empty
                v = np.arange(1000, 2000) if b % 2 else np.arange(3000, 4000)
            else:            # the same 5000-wide band with one varying hole -> Bitmap, few intervals
                keep = np.zeros(65536, bool)
                keep[10000:15000] = True
                h = int(rng.integers(10000, 15000))
                keep[h:h + 3] = False
                v = np.nonzero(keep)[0]
            per_key[b].append((v.astype(np.uint32) % 65536) | np.uint32(k << 16))
    bms = [np.concatenate(p) for p in per_key]
    s = ctx.upload_values(bms, run_optimize=True)
    refs = [oracle.RefBitmap.deserialize(x) for x in s.serialize()]
    for n in (11, 64, 150):
        members = np.arange(n, dtype=np.uint32)
        for sem in ("WORKSHY_AND", "FAST_AND"):
            _check(ctx, oracle, s, refs, sem, members)


def test_batched_xor_long_chains(ctx, oracle):
    """Batch-parallel naive_xor over Run-heavy keys (wide_xor.hip): chains of several 32-container
    batches with ragged tails; keys whose XOR empties mid-batch and at batch boundaries (removal,
    then a clone); tiny results (the Array state and its |A| < 32 rule); runs touching 0 and 65535;
    tie groups (shared run boundaries); dense results (the Bitmap state); and a full container that
    routes its key to the generic kernel.  Bytes must equal the oracle's and the generic path's."""
    import os

    import roaringbitmap_amd as rb
    rng = np.random.default_rng(33)
    nb, nkeys = 101, 12
    per_bitmap = [[] for _ in range(nb)]
    for k in range(nkeys):
        kind = k % 6
        prev = None
        for b in range(nb):
            if kind == 0:    # config-4 shape: shared core run + up to 7 random runs
                parts = [np.arange(5000, 6024)]
                for _ in range(int(rng.integers(0, 8))):
                    s0 = int(rng.integers(0, 65000))
                    parts.append(np.arange(s0, s0 + int(rng.integers(1, 257))))
                v = np.unique(np.concatenate(parts))
            elif kind == 1:  # repeats: the running XOR empties (b % 7 == 1 repeats b-1)
                if prev is not None and b % 7 == 1:
                    v = prev
                else:
                    s0 = int(rng.integers(0, 60000))
                    v = np.arange(s0, s0 + int(rng.integers(1, 3000)))
            elif kind == 2:  # tiny containers: small results, Array state, |A| < 32
                s0 = int(rng.integers(0, 40))
                v = np.unique(np.concatenate([np.arange(s0, s0 + int(rng.integers(1, 4))),
                                              np.arange(50 + s0, 52 + s0)]))
            elif kind == 3:  # runs at both ends of the key
                v = np.concatenate([np.arange(0, int(rng.integers(1, 500))),
                                    np.arange(int(rng.integers(65000, 65535)), 65536)])
            elif kind == 4:  # shared boundaries (ties) and dense results -> Bitmap state
                cuts = np.sort(rng.choice(np.arange(0, 65536, 4096), size=8, replace=False))
                v = np.unique(np.concatenate([np.arange(c, c + 2000 + 7 * (b % 3)) for c in cuts]))
            else:            # one full container in the chain -> the key takes the generic path
                v = np.arange(65536) if b == 40 else np.arange(100 * (b % 9), 100 * (b % 9) + 900)
            prev = v
            per_bitmap[b].append((v.astype(np.uint32) % 65536) | np.uint32(k << 16))
    bms = [np.unique(np.concatenate(p)).astype(np.uint32) for p in per_bitmap]
    s = ctx.upload_values(bms, run_optimize=True)
    refs = [oracle.RefBitmap.deserialize(x) for x in s.serialize()]
    for n in (nb, 64, 33, 32, 31):
        members = np.arange(n, dtype=np.uint32)
        want = oracle.wide(oracle.FAST_XOR, [refs[m] for m in members]).serialize()
        assert ctx.wide(rb.FAST_XOR, s, members).serialize()[0] == want, n
    members = rng.permutation(nb).astype(np.uint32)
    want = oracle.wide(oracle.FAST_XOR, [refs[m] for m in members]).serialize()
    assert ctx.wide(rb.FAST_XOR, s, members).serialize()[0] == want
    os.environ["RBGPU_NO_RUN_FASTPATH"] = "1"
    try:
        assert ctx.wide(rb.FAST_XOR, s, members).serialize()[0] == want
    finally:
        del os.environ["RBGPU_NO_RUN_FASTPATH"]


def _runs_container(rng, nruns, lo, hi, maxlen):
    """Sorted values of <= nruns random runs of length 4..maxlen inside [lo, hi) (overlaps merge; >= 4
    values per run keeps runOptimize's choice a Run container)."""
    v = []
    for _ in range(nruns):
        s0 = int(rng.integers(lo, hi - 4))
        v.append(np.arange(s0, min(s0 + int(rng.integers(4, maxlen + 1)), hi)))
    return np.unique(np.concatenate(v))


def test_xor_fastforward_threshold_regimes(ctx, oracle):
    """naive_xor's fast-forward (wide_xor.hip) skips per-step metrics only where no step can cross a
    type threshold; chains built to hover at each threshold must still give the oracle's bytes, and the
    same bytes with the fast-forward off (RBGPU_XOR_NO_FASTFWD=1):
      key 0  config-4 shape (shared core + random runs): long AB stretches (Bitmap), Run stretches early;
      key 1  values in [0, 8192): c hovers around 4096 (Array <-> Bitmap at every few steps);
      key 2  tiny runs in [0, 64): c near 32 (the |A| < 32 EFF rule of Array ^ Run);
      key 3  many 4-6 value runs in [0, 12000): r around 2047 and 2r ~ c (Run <-> Bitmap by EFF);
      key 4  repeated members: the chain empties (key removed, next member cloned as a Run)."""
    import os

    import roaringbitmap_amd as rb
    rng = np.random.default_rng(44)
    nb = 260
    per = [[] for _ in range(nb)]
    prev = None
    for b in range(nb):
        parts = [np.unique(np.concatenate([np.arange(7000, 8024), _runs_container(rng, 7, 0, 65536, 256)])),
                 _runs_container(rng, int(rng.integers(1, 9)), 0, 8192, 400),
                 _runs_container(rng, int(rng.integers(1, 4)), 0, 64, 10),
                 _runs_container(rng, 8, 0, 12000, 6)]
        if prev is not None and b % 5 == 1:
            parts.append(prev)
        else:
            prev = _runs_container(rng, 6, 30000, 36000, 300)
            parts.append(prev)
        per[b] = np.concatenate([(p.astype(np.uint32) % 65536) | np.uint32(k << 16) for k, p in enumerate(parts)])
    s = ctx.upload_values(per, run_optimize=True)
    h = s.download()
    assert set(h.type.tolist()) == {rb.RUN} and int(h.nruns.max()) <= 8  # all members take the Run path
    refs = [oracle.RefBitmap.deserialize(x) for x in s.serialize()]
    for n in (nb, 200, 129, 64, 65):
        members = np.arange(n, dtype=np.uint32)
        want = oracle.wide(oracle.FAST_XOR, [refs[m] for m in members]).serialize()
        assert ctx.wide(rb.FAST_XOR, s, members).serialize()[0] == want, n
        os.environ["RBGPU_XOR_NO_FASTFWD"] = "1"
        try:
            assert ctx.wide(rb.FAST_XOR, s, members).serialize()[0] == want, n
        finally:
            del os.environ["RBGPU_XOR_NO_FASTFWD"]


def test_xor_union_stretches(ctx, oracle):
    """naive_xor union stretches (wide_xor.hip, RBG_XOR_UNION): whole windows of 64 members are
    XORed without re-measuring while |P \\ U'| >= 32 (U' = the windows' runs rounded out to 64-bit
    words); chains of 1100 members so stretches span many windows and close on that bound:
      key 0  config-4 shape: stretches of several windows, closed as U' covers the key;
      key 1  runs confined to [0, 8192) with c ~ 4096: U' covers P within a window or two (the
             window is refused, the per-window rules take it);
      key 2  the same plus a fixed 20-value run at 60000 in member 0 only: |P \\ U'| hovers near 32;
      key 3  the same with a 40-value run (|P \\ U'| >= 40 holds: one stretch to the end).
    Bytes must equal the oracle's and those with the fast-forward off."""
    import os

    import roaringbitmap_amd as rb
    rng = np.random.default_rng(55)
    nb = 1100
    per = []
    for b in range(nb):
        p0 = np.unique(np.concatenate([np.arange(20000, 21024), _runs_container(rng, 7, 0, 65536, 256)]))
        p1 = _runs_container(rng, int(rng.integers(1, 9)), 0, 8192, 400)
        p2 = _runs_container(rng, int(rng.integers(1, 8)), 0, 8192, 400)
        p3 = _runs_container(rng, int(rng.integers(1, 8)), 0, 8192, 400)
        if b == 0:
            p2 = np.unique(np.concatenate([p2, np.arange(60000, 60020)]))
            p3 = np.unique(np.concatenate([p3, np.arange(60000, 60040)]))
        parts = [p0, p1, p2, p3]
        per.append(np.concatenate([(p.astype(np.uint32) % 65536) | np.uint32(k << 16) for k, p in enumerate(parts)]))
    s = ctx.upload_values(per, run_optimize=True)
    h = s.download()
    assert set(h.type.tolist()) == {rb.RUN} and int(h.nruns.max()) <= 8
    refs = [oracle.RefBitmap.deserialize(x) for x in s.serialize()]
    for n in (nb, 700, 321):
        members = np.arange(n, dtype=np.uint32)
        want = oracle.wide(oracle.FAST_XOR, [refs[m] for m in members]).serialize()
        assert ctx.wide(rb.FAST_XOR, s, members).serialize()[0] == want, n
        os.environ["RBGPU_XOR_NO_FASTFWD"] = "1"
        try:
            assert ctx.wide(rb.FAST_XOR, s, members).serialize()[0] == want, n
        finally:
            del os.environ["RBGPU_XOR_NO_FASTFWD"]


def test_queue_order_ties(ctx, oracle):
    """horizontal_or / horizontal_xor / priorityqueue_xor where many containers of a key tie on
    cardinality (the java.util.PriorityQueue's tie order then picks which types meet first) and
    bitmaps tie on getLongSizeInBytes."""
    rng = np.random.default_rng(17)
    bms = []
    for i in range(26):
        parts = []
        for k in range(4):
            c = [100, 100, 3000, 5000][k]
            if (i + k) % 3 == 0:  # a run of c values
                a = int(rng.integers(0, 65536 - c))
                v = np.arange(a, a + c)
            else:  # c scattered values
                v = rng.choice(65536, size=c, replace=False)
            parts.append(np.sort(v).astype(np.uint32) | np.uint32(k << 16))
        bms.append(np.concatenate(parts))
    import roaringbitmap_amd as rb
    for ro in (False, True):
        s = ctx.upload_values(bms, run_optimize=ro)
        refs = [oracle.RefBitmap.deserialize(b) for b in s.serialize()]
        for n in (2, 3, 7, 26):
            members = np.arange(n, dtype=np.uint32)
            for sem in ("HORIZONTAL_OR", "HORIZONTAL_XOR", "PQ_OR", "PQ_XOR"):
                _check(ctx, oracle, s, refs, sem, members)
        members = np.array([3, 3, 5, 5, 5, 9], np.uint32)  # duplicates: empty xor containers kept
        for sem in ("HORIZONTAL_XOR", "PQ_XOR", "HORIZONTAL_OR", "PQ_OR"):
            _check(ctx, oracle, s, refs, sem, members)
    assert ctx.wide(rb.PQ_XOR, s, np.zeros(0, np.uint32)).n_containers == 0


def test_priorityqueue_or_lazy_roles(ctx, oracle):
    """FastAggregation.priorityqueue_or on the device (api.hip pq_or, pairwise.hip lazy_or_type): the
    queue's three lazy roles (static lazyor, in-place lazyor, lazyorfromlazyinputs) meet
      key 0  a Run of 1500 two-value runs and Arrays in its gaps: lazyorToRun keeps Runs of 2048..4096
             runs (stored as bitmap words, sized 4r + 4), then more than 4096 -> a lazy Bitmap;
      key 1  half-density Bitmaps whose union is full, and small Arrays that complete an exact Bitmap
             (BitmapContainer.or(Array) -> full Run only when the Bitmap is not lazy);
      key 2  Arrays whose cardinalities sum around ARRAY_LAZY_LOWERBOUND (1024);
    over random member lists (duplicates allowed) with and without runOptimize."""
    rng = np.random.default_rng(77)
    pool = []
    for b in range(10):
        parts = []
        if b % 3 == 0:
            k0 = np.concatenate([np.arange(4 * i, 4 * i + 2) for i in range(1500)])
        else:
            lo = int(rng.integers(0, 1400))
            k0 = 4 * np.arange(lo, lo + int(rng.integers(200, 1100))) + 3
        parts.append(k0)
        if b % 4 == 0:
            k1 = np.flatnonzero(rng.random(65536) < 0.5)
        elif b % 4 == 1:
            k1 = np.setdiff1d(np.arange(65536), np.arange(0, 600))
        elif b % 4 == 2:
            s0 = int(rng.integers(0, 2)) * 300
            k1 = np.arange(s0, s0 + 300)
        else:
            k1 = np.flatnonzero(rng.random(65536) >= 0.5)
        parts.append(k1)
        parts.append(np.sort(rng.choice(65536, size=int(rng.integers(300, 700)), replace=False)))
        pool.append(np.concatenate([(np.asarray(p, np.int64) % 65536).astype(np.uint32) | np.uint32(k << 16)
                                    for k, p in enumerate(parts)]))
    for ro in (False, True):
        s = ctx.upload_values(pool, run_optimize=ro)
        refs = [oracle.RefBitmap.deserialize(x) for x in s.serialize()]
        for n in (1, 2, 3, 4, 5, 7, 10, 16):
            for _ in range(3):
                members = rng.integers(0, len(pool), size=n).astype(np.uint32)
                _check(ctx, oracle, s, refs, "PQ_OR", members)


def test_range_counts_contract(ctx):
    """rbgpu_set_range_counts: per-member container counts in a key range (the sharded naive_and's
    global order), members NULL = every bitmap, and its argument checks."""
    import pytest
    import roaringbitmap_amd as rb
    bms = synthetic_bitmaps(12, seed=41, max_keys=8, key_space=12)
    s = ctx.upload_values(bms, run_optimize=True)
    h = s.download()
    full = np.diff(h.begin.astype(np.int64))
    assert s.range_counts().tolist() == full.tolist()
    members = np.array([3, 0, 3, 7], np.uint32)
    assert s.range_counts(members).tolist() == full[members].tolist()
    for lo, hi in ((0, 5), (5, 12), (12, 65536), (4, 4)):
        want = [int(((h.key[h.begin[m]:h.begin[m + 1]] >= lo) & (h.key[h.begin[m]:h.begin[m + 1]] < hi)).sum())
                for m in members]
        assert s.range_counts(members, (lo, hi)).tolist() == want
    with pytest.raises(rb.InvalidArgument):
        s.range_counts(members, (7, 3))
    with pytest.raises(rb.InvalidArgument):
        s.range_counts(np.array([12], np.uint32))


def _dense_mixed(rng, n, keys):
    """n bitmaps that all hold exactly the high keys `keys` (a dense set), mixed container kinds."""
    from datasets import _container_values
    kinds = ["single", "tiny", "sparse", "a4095", "b4097", "dense", "full", "runs", "fewruns", "contig"]
    bms = []
    for i in range(n):
        parts = [(_container_values(rng, kinds[(i * 7 + k * 3 + int(rng.integers(0, 3))) % len(kinds)]) |
                  np.uint32(k << 16)) for k in keys]
        bms.append(np.concatenate(parts).astype(np.uint32))
    return bms


def test_dense_sets_skip_grouping(ctx, oracle):
    """A set whose bitmaps all hold exactly the keys [dense_lo, dense_hi) takes the ungrouped path
    (container ids from the member bases, cached packed / key-major records): every semantics, member
    orders (set order -> cached krec, permuted / subset / duplicates -> per-call transpose), key-range
    shards that clip the dense range, and the same bytes with the grouping forced
    (RBGPU_NO_DENSE_GROUPING=1).  Keys of mixed container types go to the generic kernel with dense ids."""
    import os

    import roaringbitmap_amd as rb
    from roaringbitmap_amd.sharding import serialize_parts
    rng = np.random.default_rng(41)
    bms = _dense_mixed(rng, 13, range(5, 13))
    for ro in (False, True):
        s = ctx.upload_values(bms, run_optimize=ro)
        refs = [oracle.RefBitmap.deserialize(b) for b in s.serialize()]
        orders = [np.arange(13, dtype=np.uint32), np.arange(12, -1, -1, dtype=np.uint32),
                  np.array([3, 1, 4, 1, 5, 9, 2, 6, 5, 3, 5, 8], np.uint32), np.array([7, 2], np.uint32)]
        for members in orders:
            for sem in SEMS:
                _check(ctx, oracle, s, refs, sem, members)
        members = orders[0]
        for sem in SHARDABLE:
            if sem == "NAIVE_AND":
                continue  # a shard picks its own smallest member (NAIVE_AND_ITER is the sharded form)
            want = ctx.wide(getattr(rb, sem), s, members).serialize()[0]
            for ranges in ([(0, 7), (7, 10), (10, 65536)], [(0, 5), (5, 13), (13, 65536)], [(0, 12), (12, 65536)]):
                shards = [ctx.wide(getattr(rb, sem), s, members, key_range=r) for r in ranges]
                assert serialize_parts([sh.download() for sh in shards]) == want, (sem, ranges)
            os.environ["RBGPU_NO_DENSE_GROUPING"] = "1"
            try:
                assert ctx.wide(getattr(rb, sem), s, members).serialize()[0] == want, sem
            finally:
                del os.environ["RBGPU_NO_DENSE_GROUPING"]


def test_dense_run_shard_records(ctx, oracle):
    """Config-4 shape generated as a key-range shard (dense_lo > 0): workShyAnd through the packed
    records, naive_xor through the set's cached key-major records (set order) and through per-call
    transposed records (reversed order), naive_or through dense ids — all equal to the oracle.  Even
    member and key counts build the key-major records two containers per lane (128-key tiles); an odd
    key count (odd member bases) or an odd member count takes the 64 x 64 tiles."""
    import roaringbitmap_amd as rb
    for nb, lo, hi in ((40, 300, 700), (40, 300, 701), (41, 300, 700)):
        a = ctx.generate_keys(rb.WL_WIDE_RUNS, nb, lo, hi, seed=5)
        refs = [oracle.RefBitmap.deserialize(b) for b in a.serialize()]
        for members in (np.arange(nb, dtype=np.uint32), np.arange(nb - 1, -1, -1, dtype=np.uint32)):
            for sem in ("FAST_OR", "FAST_AND", "WORKSHY_AND", "FAST_XOR", "PAR_XOR"):
                _check(ctx, oracle, a, refs, sem, members)
            # the cached records are reused call after call
            for _ in range(2):
                _check(ctx, oracle, a, refs, "FAST_XOR", members)


def test_soa_run_count_on_non_run_containers_is_ignored(ctx, oracle):
    """The format ignores the run count of an Array / Bitmap entry; rbgpu_set_from_soa stores 0 there, since
    workShyAnd's SoA reads and naive_xor's 4-B records take "run count > 0" for "a Run" (round 6).  A key whose
    members are Runs and one Array with a stray count of 3 must still come out as the oracle's."""
    import roaringbitmap_amd as rb
    from type_pins import ARRAY, RUN, one_container_soa, oracle_bitmap, r, u
    conts = [(RUN, u(r(0, 3000), r(5000, 5100))), (RUN, u(r(100, 2900), r(5050, 5060))),
             (ARRAY, np.arange(0, 6000, 3, dtype=np.uint32)), (RUN, r(200, 2000))]
    soa = one_container_soa(conts)
    soa.nruns[2] = 3  # the Array's stray run count
    s = ctx.upload_soa(soa)
    assert int(s.download().nruns[2]) == 0
    refs = [oracle_bitmap(oracle, t, v) for t, v in conts]
    for sem_name in ("WORKSHY_AND", "FAST_AND", "FAST_XOR", "FAST_OR"):
        for members in ([0, 1, 2, 3], [2, 0, 1], [0, 1, 3]):
            _check(ctx, oracle, s, refs, sem_name, np.array(members, np.uint32))


def test_xor_records_first_call_and_reuse(ctx, oracle):
    """naive_xor on a fresh dense set builds the key-major 4-B records on its first call, from the SoA or — when the
    set already has packed records (a call in another member order built them) — from those; the calls after it
    reuse them.  Even and odd key / member counts (two-container and 64 x 64 tiles)."""
    import roaringbitmap_amd as rb
    for nb, lo, hi, mrec_first in ((64, 0, 1024, False), (33, 100, 613, True), (40, 256, 512, False)):
        a = ctx.generate_keys(rb.WL_WIDE_RUNS, nb, lo, hi, seed=9)
        refs = [oracle.RefBitmap.deserialize(b) for b in a.serialize()]
        ident = np.arange(nb, dtype=np.uint32)
        seq = ([ident[::-1].copy()] if mrec_first else []) + [ident, ident]
        for members in seq:
            _check(ctx, oracle, a, refs, "FAST_XOR", members)
        a.close()

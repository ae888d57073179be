"""The 64-bit oracle (oracle/rbref64.py) pinned by the reference's own 64-bit fixtures: the
RoaringFormatSpec 64-bit extension files of TestRoaring64NavigableMap.testSerialization_* (CRoaring's
testdata; TestRoaring64NavigableMap.java:1644-1724) — cardinality, bucket count, select() values and the
byte-identical re-serialization (checkConsistencyWithResource)."""
import os

import numpy as np
import pytest

GOLD = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "testdata")
MAXU = (1 << 32) - 1
# (file, cardinality, buckets, {select index: value})  TestRoaring64NavigableMap.java:1644-1724
FIXTURES64 = [
    ("64mapempty.bin", 0, 0, {}),
    ("64map32bitvals.bin", 10, 1, {0: 0, 9: 9}),
    ("64mapspreadvals.bin", 100, 10, {0: 0, 9: 9, 90: (9 << 32) + 0, 91: (9 << 32) + 1, 99: (9 << 32) + 9}),
    ("64maphighvals.bin", 121, 11, {0: ((MAXU - 10) << 32) + (MAXU - 10), 10: ((MAXU - 10) << 32) + MAXU,
                                    110: (MAXU << 32) + (MAXU - 10), 111: (MAXU << 32) + (MAXU - 9),
                                    120: (MAXU << 32) + MAXU}),
]


def read(name):
    with open(os.path.join(GOLD, name), "rb") as f:
        return f.read()


@pytest.mark.parametrize("name,card,nb,sel", FIXTURES64, ids=[f[0] for f in FIXTURES64])
def test_oracle64_fixtures(name, card, nb, sel):
    from oracle import rbref64 as R64
    data = read(name)
    b = R64.Ref64.from_portable(data)
    assert b.cardinality() == card and len(b.buckets) == nb
    vals = b.to_array()
    for j, v in sel.items():
        assert int(vals[j]) == v
    assert b.to_portable() == data


def test_oracle64_ops_contract():
    """The per-class rules the device follows: Roaring64Bitmap keeps an empty xor container under its key,
    Roaring64NavigableMap keeps a bucket whose RoaringBitmap became empty, x.op(x) takes the `x2 == this`
    branches; content always equals the set algebra."""
    from oracle import rbref as R
    from oracle import rbref64 as R64
    x = R64.Ref64.of([5, 6, (3 << 32) + 7, (3 << 32) + 70000])
    y = R64.Ref64.of([5, 6, (3 << 32) + 8, (9 << 32) + 1])
    art = R64.bitmap_op(R.XOR, x, y, inplace=False)
    assert [h for h, _ in art.buckets] == [0, 3, 9]
    assert art.buckets[0][1].containers()[0][2] == 0          # the empty container of key 0 is kept
    nav = R64.navigable_op(R.XOR, x, y)
    assert [h for h, _ in nav.buckets] == [0, 3, 9] and nav.buckets[0][1].cardinality() == 0
    assert len(nav.buckets[0][1].containers()) == 0            # RoaringBitmap.xor drops it; the bucket stays
    for op in (R.AND, R.OR, R.XOR, R.ANDNOT):
        sx, sy = set(x.to_array().tolist()), set(y.to_array().tolist())
        want = {R.AND: sx & sy, R.OR: sx | sy, R.XOR: sx ^ sy, R.ANDNOT: sx - sy}[op]
        for r in (R64.bitmap_op(op, x, y, False), R64.bitmap_op(op, x, y, True), R64.navigable_op(op, x, y)):
            assert sorted(r.to_array().tolist()) == sorted(want)
    assert R64.navigable_op(R.AND, x, y).to_array().tolist() == [5, 6]
    assert [h for h, _ in R64.navigable_op(R.AND, x, y).buckets] == [0, 3]  # bucket 3 stays, empty
    assert R64.bitmap_op(R.XOR, x, x, True, same=True).buckets == []
    assert R64.navigable_op(R.OR, x, x, same=True).to_portable() == x.to_portable()


def test_oracle64_legacy_format():
    """Roaring64NavigableMap.serializeLegacy / deserializeLegacy (the default SERIALIZATION_MODE_LEGACY,
    Roaring64NavigableMap.java:51, 1229-1240, 1295-1325): signedLongs byte, big-endian int count and highs,
    little-endian RoaringBitmaps, in the map's order.  The reference holds no legacy fixture (parity
    unpinned); its tests pin the size (checkSerializeBytes: 1 + 4 + sum(4 + bucket bytes),
    TestRoaring64NavigableMap.java:66-73, 775-790) and the signed / unsigned value order after a clone
    through this format (testSerialization_MultipleBuckets_Signed / _Unsigned, :741-773)."""
    import struct

    from oracle import rbref64 as R64
    vals = np.array([(-123) & (2**64 - 1), 123, 2**63 - 1], np.uint64)
    for signed, order in ((True, [(-123) & (2**64 - 1), 123, 2**63 - 1]), (False, [123, 2**63 - 1, (-123) & (2**64 - 1)])):
        m = R64.Ref64.of(vals)
        m.signed = signed
        data = m.to_legacy()
        assert len(data) == 1 + 4 + sum(4 + len(b.serialize()) for _, b in m.buckets)
        assert data[0] == int(signed) and struct.unpack_from(">i", data, 1)[0] == 3
        back = R64.Ref64.from_legacy(data)
        assert back.signed == signed and back.to_legacy() == data
        highs = [struct.unpack_from(">I", data, p)[0] for p in _legacy_high_positions(data)]
        assert [(h << 32) | int(b.to_array()[0]) for h, b in
                sorted(back.buckets, key=lambda hb: hb[0] if not signed else (hb[0] ^ (1 << 31)))] == order
        assert highs == [v >> 32 for v in order]
    rng = np.random.default_rng(3)
    for _ in range(5):
        v = np.unique(rng.integers(0, 2**64 - 1, 300, dtype=np.uint64) >> np.uint64(int(rng.integers(0, 40))))
        m = R64.Ref64.of(v)
        for signed in (False, True):
            m.signed = signed
            assert R64.Ref64.from_legacy(m.to_legacy()).to_legacy() == m.to_legacy()
    with pytest.raises((IOError, ValueError, Exception)):
        R64.Ref64.from_legacy(b"\x00\x00\x00")


def _legacy_high_positions(data):
    from oracle import rbref as R
    import struct
    (n,) = struct.unpack_from(">i", data, 1)
    pos, out = 5, []
    for _ in range(n):
        out.append(pos)
        pos += 4
        pos += len(R.RefBitmap.deserialize(data[pos:]).serialize())
    return out


def _art_sets():
    """64-bit sets whose ARTs cover every node type: one 48-bit key; two keys differing in the last byte
    (a Node4 with a 5-byte prefix); 5 / 17 / 49 children under one node (Node16 / Node48 / Node256 by
    growth); keys spread over the 48-bit space (several levels, prefixes of every length)."""
    from oracle import rbref64 as R64
    rng = np.random.default_rng(11)
    out = [R64.Ref64(), R64.Ref64.of([5]), R64.Ref64.of([5, (1 << 16) | 7])]
    for nkids in (5, 17, 49, 300):
        keys = np.arange(nkids, dtype=np.uint64) * np.uint64(3)
        out.append(R64.Ref64.of((keys << np.uint64(16)) | np.uint64(9)))
    spread = rng.integers(0, 1 << 48, size=200, dtype=np.uint64)
    vals = [(spread << np.uint64(16)) | rng.integers(0, 65536, size=200).astype(np.uint64)]
    for k in rng.choice(200, 20, replace=False):  # some dense keys (Bitmap / Run containers)
        vals.append((spread[k] << np.uint64(16)) + np.arange(5000, 30000, dtype=np.uint64))
    r = R64.Ref64.of(np.concatenate(vals))
    for _, b in r.buckets[::2]:
        b.run_optimize()
    out.append(r)
    return out


def test_oracle64_art_format():
    """Roaring64Bitmap.serialize / deserialize (HighLowContainer: ART + Containers) restated in
    oracle/rbref64.py.  Parity unpinned: the reference holds no fixture of this format, so this pins the
    restatement by one hand-decoded stream (two 48-bit keys differing in the last byte: a Node4 with a
    5-byte prefix over two leaves, one 2-slot container array) and round trips over every node type."""
    from oracle import rbref64 as R64
    two = R64.Ref64.of([5, (1 << 16) | 7]).to_art()
    want = bytes.fromhex(
        "01" "0200000000000000"                         # NOT_EMPTY_TAG, Art.keySize = 2 (LE long)
        "00" "0200" "05" "0000000000" "00000100"        # Node4: count 2, prefix 00x5, key bytes 0, 1 (reversed int)
        "04" "0000" "00" "000000000000" "0000000000000000"  # LeafNode: key 0, container index 0
        "04" "0000" "00" "000000000001" "0100000000000000"  # LeafNode: key 1, container index 1
        "01000000" "fe" "02000000"                      # one first-level array, NOT_TRIMMED_MARK, 2 slots
        "01" "02" "01000000" "0500"                     # NOT_NULL, ArrayContainer (type 2), card 1, value 5
        "01" "02" "01000000" "0700"
        "0200000000000000" "00000000" "01000000")       # containerSize, firstLevelIdx, secondLevelIdx
    assert two == want
    assert R64.Ref64().to_art() == b"\x00"
    for r in _art_sets():
        data = r.to_art()
        back = R64.Ref64.from_art(data)
        assert np.array_equal(back.to_array(), r.to_array())
        assert back.to_art() == data
        n = sum(len(b.containers()) for _, b in r.buckets)
        if n > 1:  # another container placement (a history with removals): same set
            slots = list(np.random.default_rng(n).permutation(n + 3)[:n])
            other = r.to_art(slots=slots, cap=n + 3)
            assert other != data and np.array_equal(R64.Ref64.from_art(other).to_array(), r.to_array())
    # the root's type byte (after the tag and the key count): 5 / 17 / 49 children grow Node16 / 48 / 256
    assert [r.to_art()[9] for r in _art_sets()[3:6]] == [1, 2, 3]
    with pytest.raises((IOError, Exception)):
        R64.Ref64.from_art(two[:-1])


def test_oracle64_art_kept_empty_types():
    """Roaring64Bitmap.xor(x, x) keeps every container empty under its key (Roaring64Bitmap.java:421-460:
    put with no isEmpty check) with the type its container xor returns: an empty Run xor Run is a Run
    (RunContainer.java:2445-2482 -> toEfficientContainer :2326-2335, 2 + 4*0 <= min(8192, 2*0 + 2), the tie
    goes to Run), an empty Array xor Array or Bitmap xor Bitmap an Array (ArrayContainer.java:1311-1336,
    BitmapContainer.java:1381-1422).  The ART stream carries that type byte (art/Containers.java: 0 Run with
    its run count, 2 Array) — the case GPUTEST_r04 found the restatement typing every empty container as an
    Array."""
    from oracle import rbref64 as R64
    run = np.arange(100, 20000, dtype=np.uint64)                      # one Run after runOptimize
    arr = (np.uint64(1) << np.uint64(16)) + np.arange(0, 900, 3, dtype=np.uint64)      # an Array
    bmp = (np.uint64(2) << np.uint64(16)) + np.arange(0, 60000, 3, dtype=np.uint64)    # a Bitmap
    x = R64.Ref64.of(np.concatenate([run, arr, bmp]))
    for _, b in x.buckets:
        b.run_optimize()
    assert [c[1] for c in x.buckets[0][1].containers()] == [2, 0, 1]   # Run, Array, Bitmap (rbref enum)
    r = R64.bitmap_op(R64.XOR, x, x, False)
    assert [(c[1], c[2]) for c in r.buckets[0][1].containers()] == [(2, 0), (0, 0), (0, 0)]
    art = r.to_art()
    # three leaves after the Node4 root; the container array follows: 1 first-level array, 0xFE, 3 slots
    at = art.index(bytes([1, 0, 0, 0, 0xFE, 3, 0, 0, 0])) + 9
    assert art[at:at + 8] == bytes([1, 0, 0, 0, 0, 0, 0, 0])          # NOT_NULL, Run, card 0, nbrruns 0
    assert art[at + 8:at + 14] == bytes([1, 2, 0, 0, 0, 0])           # NOT_NULL, Array, card 0
    assert art[at + 14:at + 20] == bytes([1, 2, 0, 0, 0, 0])
    back = R64.Ref64.from_art(art)       # Containers.deserialize keeps the empty containers
    assert back.to_art() == art and back.cardinality() == 0
    assert [(c[1], c[2]) for c in back.buckets[0][1].containers()] == [(2, 0), (0, 0), (0, 0)]

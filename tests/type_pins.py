"""The reference's container-type assertions (`instanceof` pins) on the set-algebra path, as data.

Byte parity is a container-TYPE question: for canonical inputs the result SET of every op
is unique, the type fixes the bytes.  These are the type decisions the reference's own tests assert,
restated as (inputs, entry point, expected type) so they can run on the oracle (test_type_pins.py) and
through the device (test_gpu_type_pins.py).  Paths are relative to
/root/reference/RoaringBitmap/src/test/java/org/roaringbitmap/.

Inventory of the 88 `instanceof` lines of the four container test files:

  file                     lines  on the path (here)  not on the path
  TestContainer.java          41  12                  27 Container.not/inot range flips (:254-627),
                                                       2 commented out (:851, :861)
  TestRunContainer.java       28  23                  3 not/inot (:1093, :2031, :2058),
                                                       2 commented out (:2906, :2951)
  TestBitmapContainer.java    11  11                  -
  TestArrayContainer.java      8   8                  -

`not(range)` is RoaringBitmap.flip, which SURVEY §8a leaves off the hot path; a flip is NOT an XOR with a
Run container type-wise (Array.not keeps AB, Run XOR Array with |A| < 32 goes EFF), so those pins cannot
be restated through and/or/xor/andNot.  Two of the on-path pins (TestArrayContainer:118-125, :210-219) and
one input (TestBitmapContainer:579) use ArrayContainers of 32768 values, which no canonical RoaringBitmap
holds; they run on the oracle as written and on the device with the canonical (Bitmap) form of the
same set, where the reference's rule gives the same type.
"""
from __future__ import annotations

from dataclasses import dataclass, field
from typing import List, Optional, Tuple

import numpy as np

ARRAY, BITMAP, RUN = 0, 1, 2
TYPE_NAME = {ARRAY: "Array", BITMAP: "Bitmap", RUN: "Run"}


def r(a, b, step=1):
    return np.arange(a, b, step, dtype=np.uint32)


def u(*parts):
    return np.unique(np.concatenate([np.asarray(p, dtype=np.uint32) for p in parts]))


@dataclass
class Pin:
    name: str
    cite: str                          # file:line of the assertion(s)
    inputs: List[Tuple[int, np.ndarray]]  # (container type, low 16-bit values) of one container each
    how: str                           # op:AND|OR|XOR|ANDNOT, inplace:OR, wide:FAST_OR|PAR_OR, runopt, build
    expect: Optional[int]              # expected result container type (None: the reference does not pin it)
    card: Optional[int] = None         # expected result cardinality when the reference asserts it
    npins: int = 1                     # instanceof lines this case covers
    note: str = ""
    tags: List[str] = field(default_factory=list)

    def canonical(self) -> bool:
        """Every input is what a RoaringBitmap can hold (Array <= 4096 < Bitmap)."""
        for t, v in self.inputs:
            if t == ARRAY and len(v) > 4096:
                return False
            if t == BITMAP and len(v) <= 4096:
                return False
        return True

    def canonical_inputs(self):
        """The same sets with non-canonical Arrays / Bitmaps re-typed by the AB rule."""
        out = []
        for t, v in self.inputs:
            if t == ARRAY and len(v) > 4096:
                t = BITMAP
            elif t == BITMAP and len(v) <= 4096:
                t = ARRAY
            out.append((t, v))
        return out


FULL = r(0, 65536)

PINS: List[Pin] = [
    # ------------------------------------------------------------------ TestContainer.java
    Pin("TestContainer.or6", "TestContainer.java:804-821",
        [(RUN, r(0, 6144, 6)), (RUN, r(3, 6144, 6))], "op:OR", ARRAY, 2048),
    Pin("TestContainer.testRunOptimize1", "TestContainer.java:890-899",
        [(ARRAY, u(r(1, 10), [50000, 50001]))], "runopt", RUN),
    Pin("TestContainer.testRunOptimize1A", "TestContainer.java:903-911",
        [(ARRAY, [1, 2, 3, 4, 6, 8, 9, 50000, 50003])], "runopt", ARRAY),
    Pin("TestContainer.testRunOptimize2", "TestContainer.java:914-923",
        [(BITMAP, r(0, 40000))], "runopt", RUN),
    Pin("TestContainer.testRunOptimize2A", "TestContainer.java:927-936",
        [(BITMAP, r(0, 40000, 2))], "runopt", BITMAP),
    Pin("TestContainer.testRunOptimize3", "TestContainer.java:938-947",
        [(RUN, u(r(1, 10), [50000, 50001]))], "runopt", RUN),
    Pin("TestContainer.testRunOptimize3A", "TestContainer.java:949-958",
        [(RUN, [1, 3, 5, 7, 9, 11, 17, 21, 50000, 50002])], "runopt", ARRAY),
    Pin("TestContainer.testRunOptimize3B", "TestContainer.java:961-970",
        [(RUN, r(100, 30000, 2))], "runopt", BITMAP),
    Pin("TestContainer.transitionTest/4096", "TestContainer.java:978-984",
        [(ARRAY, r(0, 4096))], "build", ARRAY, 4096, npins=2),
    Pin("TestContainer.transitionTest/4097", "TestContainer.java:985-987",
        [(ARRAY, r(0, 4097))], "build", BITMAP, 4097),
    Pin("TestContainer.transitionTest/remove", "TestContainer.java:988-990",
        [(BITMAP, r(0, 4097)), (ARRAY, [4096])], "op:ANDNOT", ARRAY, 4096,
        note="BitmapContainer.remove back to 4096 values == Bitmap \\ {4096} (AB rule)"),
    # ------------------------------------------------------------------ TestRunContainer.java
    Pin("TestRunContainer.orFullToRunContainer", "TestRunContainer.java:2634-2642",
        [(RUN, r(0, 1 << 15)), (BITMAP, r(1 << 15, 1 << 16))], "op:OR", RUN, 65536, npins=2),
    Pin("TestRunContainer.orFullToRunContainer2", "TestRunContainer.java:2644-2652",
        [(RUN, r(1024 - 200, 1 << 16)), (ARRAY, r(0, 1024))], "op:OR", RUN, 65536, npins=2),
    Pin("TestRunContainer.orFullToRunContainer3", "TestRunContainer.java:2654-2662",
        [(RUN, r(0, 1 << 15)), (RUN, r((1 << 15) - 200, 1 << 16))], "op:OR", RUN, 65536, npins=2),
    Pin("TestRunContainer.toBitmapOrArrayContainer/array", "TestRunContainer.java:2776-2781",
        [(RUN, r(0, 2048)), (BITMAP, FULL)], "op:AND", ARRAY, 2048,
        note="RunContainer.toBitmapOrArrayContainer(card) is the AB rule of Run AND Bitmap"),
    Pin("TestRunContainer.toBitmapOrArrayContainer/bitmap", "TestRunContainer.java:2785-2788",
        [(RUN, r(0, 8192)), (BITMAP, FULL)], "op:AND", BITMAP, 8192),
    Pin("TestRunContainer.charRangeRank", "TestRunContainer.java:2273-2281",
        [(RUN, r(16, 32)), (RUN, r(16, 32))], "op:AND", RUN, 16,
        note="the Run container built by add(16, 32) stays a Run (R AND R -> EFF keeps it)"),
    Pin("TestRunContainer.xor_array_largecase_runcontainer_best", "TestRunContainer.java:2876-2914",
        [(RUN, u(*[r(k * 100, k * 100 + 99) for k in range(60)])),
         (ARRAY, u(*[[k * 100 + 98, k * 100 + 99] for k in range(60)]))], "op:XOR", BITMAP, 5940, npins=2,
        note="inputs pinned Array / Run (:2889-2890); the result type is the one the comment at "
             ":2903-2904 says the code picks (a bitmap)"),
    Pin("TestRunContainer.xor_array_mediumcase", "TestRunContainer.java:2917-2962",
        [(RUN, u(*[[k * 10, k * 10 + 1, k * 10 + 2] for k in range(4096 // 6)])),
         (ARRAY, r(0, 10 * (4096 // 12), 10))], "op:XOR", ARRAY, 3 * (4096 // 6) - 4096 // 12, npins=2,
        note="inputs pinned (:2933-2934); result type per the comment at :2946-2949 (an array container)"),
    Pin("TestRunContainer.xor_array_smallcase", "TestRunContainer.java:2965-3002",
        [(RUN, u(*[r(k * 10, k * 10 + 5) for k in range(4096 // 3)])), (ARRAY, [1, 2, 3, 4, 5])],
        "op:XOR", None, 5 * (4096 // 3) - 3, npins=2,
        note="inputs pinned (:2980-2981); the result type is not asserted by the reference"),
    Pin("TestRunContainer.testLazyORFull", "TestRunContainer.java:3218-3227",
        [(RUN, r(0, 1 << 15)), (BITMAP, r(3210, 1 << 16))], "wide:FAST_OR", RUN, 65536),
    Pin("TestRunContainer.testLazyORFull2", "TestRunContainer.java:3229-3236",
        [(RUN, r(1024 - 200, 1 << 16)), (ARRAY, r(0, 1024))], "wide:PAR_OR", RUN, 65536,
        note="Run.lazyOR(Array) full; ParallelAggregation.or's clone + lazyIOR chain"),
    Pin("TestRunContainer.testLazyORFull3/lazyOR", "TestRunContainer.java:3238-3246",
        [(RUN, r(0, 1 << 15)), (RUN, r(1 << 15, 1 << 16))], "wide:FAST_OR", RUN, 65536),
    Pin("TestRunContainer.testLazyORFull3/lazyIOR", "TestRunContainer.java:3243-3247",
        [(RUN, r(0, 1 << 15)), (RUN, r(1 << 15, 1 << 16))], "wide:PAR_OR", RUN, 65536),
    # ------------------------------------------------------------------ TestBitmapContainer.java
    Pin("TestBitmapContainer.testLazyORFull/lazyor", "TestBitmapContainer.java:134-146",
        [(BITMAP, r(0, 1 << 15)), (BITMAP, r(3210, 1 << 16))], "wide:FAST_OR", RUN, 65536),
    Pin("TestBitmapContainer.testLazyORFull/ilazyor", "TestBitmapContainer.java:139-147",
        [(BITMAP, r(0, 1 << 15)), (BITMAP, r(3210, 1 << 16))], "wide:PAR_OR", RUN, 65536),
    Pin("TestBitmapContainer.testLazyORFull2/lazyor", "TestBitmapContainer.java:150-162",
        [(BITMAP, r(1024 - 200, 1 << 16)), (ARRAY, r(0, 1 << 10))], "wide:FAST_OR", RUN, 65536),
    Pin("TestBitmapContainer.testLazyORFull2/ilazyor", "TestBitmapContainer.java:155-163",
        [(BITMAP, r(1024 - 200, 1 << 16)), (ARRAY, r(0, 1 << 10))], "wide:PAR_OR", RUN, 65536),
    Pin("TestBitmapContainer.testLazyORFull3/lazyor", "TestBitmapContainer.java:166-178",
        [(BITMAP, r(0, 1 << 15)), (RUN, r(1 << 15, 1 << 16))], "wide:FAST_OR", RUN, 65536),
    Pin("TestBitmapContainer.testLazyORFull3/ilazyor", "TestBitmapContainer.java:171-179",
        [(BITMAP, r(0, 1 << 15)), (RUN, r(1 << 15, 1 << 16))], "wide:PAR_OR", RUN, 65536),
    Pin("TestBitmapContainer.orFullToRunContainer", "TestBitmapContainer.java:567-574",
        [(BITMAP, r(0, 1 << 15)), (BITMAP, r(1 << 15, 1 << 16))], "op:OR", RUN, 65536),
    Pin("TestBitmapContainer.orFullToRunContainer2", "TestBitmapContainer.java:576-583",
        [(BITMAP, r(0, 1 << 15)), (ARRAY, r(1 << 15, 1 << 16))], "op:OR", RUN, 65536,
        note="the Array operand holds 32768 values (non-canonical)"),
    Pin("TestBitmapContainer.orFullToRunContainer3/or", "TestBitmapContainer.java:585-593",
        [(BITMAP, r(0, 1 << 15)), (BITMAP, r(3210, 1 << 16))], "op:OR", RUN, 65536),
    Pin("TestBitmapContainer.orFullToRunContainer3/ior", "TestBitmapContainer.java:590-594",
        [(BITMAP, r(0, 1 << 15)), (BITMAP, r(3210, 1 << 16))], "inplace:OR", RUN, 65536),
    Pin("TestBitmapContainer.orFullToRunContainer4", "TestBitmapContainer.java:597-604",
        [(BITMAP, r(0, 1 << 15)), (RUN, r(3210, 1 << 16))], "inplace:OR", RUN, 65536),
    # ------------------------------------------------------------------ TestArrayContainer.java
    Pin("TestArrayContainer.orFullToRunContainer", "TestArrayContainer.java:109-116",
        [(ARRAY, r(0, 1 << 12)), (BITMAP, r(1 << 12, 1 << 16))], "op:OR", RUN, 65536),
    Pin("TestArrayContainer.orFullToRunContainer2", "TestArrayContainer.java:118-125",
        [(ARRAY, r(0, 1 << 15)), (ARRAY, r(1 << 15, 1 << 16))], "op:OR", RUN, 65536,
        note="two 32768-value Arrays (non-canonical)"),
    Pin("TestArrayContainer.testLazyORFull", "TestArrayContainer.java:210-219",
        [(ARRAY, r(0, 1 << 15)), (ARRAY, r(1 << 15, 1 << 16))], "wide:FAST_OR", RUN, 65536,
        note="two 32768-value Arrays (non-canonical)"),
    Pin("TestArrayContainer.testNextValue2", "TestArrayContainer.java:691-701",
        [(ARRAY, r(64, 129))], "build", ARRAY, 65),
    Pin("TestArrayContainer.testNextValueBetweenRuns", "TestArrayContainer.java:703-713",
        [(ARRAY, u(r(64, 129), r(256, 321)))], "build", ARRAY, 130),
    Pin("TestArrayContainer.testNextValue3", "TestArrayContainer.java:715-732",
        [(ARRAY, u(r(64, 129), r(200, 501), r(5000, 5201)))], "build", ARRAY, 567),
    Pin("TestArrayContainer.testPreviousValue1", "TestArrayContainer.java:734-744",
        [(ARRAY, r(64, 129))], "build", ARRAY, 65),
    Pin("TestArrayContainer.testPreviousValue2", "TestArrayContainer.java:746-755",
        [(ARRAY, u(r(64, 129), r(200, 501), r(5000, 5201)))], "build", ARRAY, 567),
]

# getSetOfRunContainers (TestRunContainer.java:81-153): pairs (Run, Array-or-Bitmap) of equal content;
# RunContainerArg_Array{AND,ANDNOT,OR,XOR} (:2294-2416) check b_k op r_l == b_k op b_l for all k, l.
# The loop bounds 655536 wrap at the char cast, so r3 / r4 hold the values below 65536.
RUN_ARG_SETS = [
    FULL,
    r(0, 4096),
    r(0, 65536, 2),
    r(0, 65536, 256),
    u(*[r(k, k + 256) for k in range(0, 65536 - 4096, 4096)]),
    r(0, 65535, 7),
    r(0, 65535, 11),
]
RUN_ARG_PINS = 4  # the four `instanceof BitmapContainer` lines (:2305, :2331, :2379, :2404)


def ab_type(vals) -> int:
    return ARRAY if len(vals) <= 4096 else BITMAP


def n_on_path_pins() -> int:
    return sum(p.npins for p in PINS) + RUN_ARG_PINS


def runs_of(vals: np.ndarray) -> np.ndarray:
    v = np.asarray(vals, dtype=np.int64)
    if len(v) == 0:
        return np.zeros((0, 2), np.uint16)
    brk = np.nonzero(np.diff(v) != 1)[0]
    starts = np.concatenate([[0], brk + 1])
    ends = np.concatenate([brk, [len(v) - 1]])
    return np.stack([v[starts], v[ends] - v[starts]], axis=1).astype(np.uint16)


def payload_of(t: int, vals) -> bytes:
    vals = np.asarray(vals, dtype=np.uint32)
    if t == ARRAY:
        return vals.astype(np.uint16).tobytes()
    if t == BITMAP:
        bits = np.zeros(65536, np.uint8)
        bits[vals] = 1
        return np.packbits(bits, bitorder="little").tobytes()
    return runs_of(vals).tobytes()


def one_container_soa(containers):
    """HostSoA of len(containers) one-container bitmaps (key 0) with the given types."""
    from roaringbitmap_amd.engine import HostSoA
    keys, types, cards, nruns, offs, chunks = [], [], [], [], [], []
    pos = 0
    for t, v in containers:
        data = payload_of(t, v)
        keys.append(0)
        types.append(t)
        cards.append(len(v))
        nruns.append(len(runs_of(v)) if t == RUN else 0)
        offs.append(pos)
        pad = (-len(data)) % 16
        chunks.append(data + b"\0" * pad)
        pos += len(data) + pad
    n = len(containers)
    return HostSoA(np.arange(n + 1, dtype=np.uint64), np.array(keys, np.uint16), np.array(types, np.uint8),
                   np.array(cards, np.uint32), np.array(nruns, np.uint16), np.array(offs, np.uint64),
                   np.frombuffer(b"".join(chunks) or b"\0" * 16, np.uint8).copy())


def oracle_bitmap(oracle, t: int, vals):
    """An oracle bitmap with ONE container of exactly type t at key 0 (non-canonical types allowed)."""
    data = np.frombuffer(payload_of(t, vals) or b"\0\0", np.uint8)
    v = np.asarray(vals)
    return oracle.from_soa([0], [t], [len(v)], [len(runs_of(v)) if t == RUN else 0], data, [0])

"""The reference's container-type pins (tests/type_pins.py) through the MI355X path: every pin whose
entry point the device serves (static and/or/xor/andNot, FastAggregation.or, ParallelAggregation.or,
in-place x1.or(x2) (rbgpu_pairwise_inplace), runOptimize (rbgpu_set_run_optimize), bitmapOf
construction) must give the pinned type and the oracle's bytes.  Pins with non-canonical inputs
(32768-value ArrayContainers) run with the canonical form of the same sets."""
import numpy as np
import pytest

from type_pins import PINS, RUN, RUN_ARG_SETS, TYPE_NAME, ab_type, one_container_soa, oracle_bitmap

pytestmark = pytest.mark.gpu
OPS = {"AND": 0, "OR": 1, "XOR": 2, "ANDNOT": 3}
DEVICE_PINS = [p for p in PINS if p.how.split(":")[0] in ("op", "wide", "build", "inplace", "runopt")]


def test_every_pin_runs_on_the_device():
    assert len(DEVICE_PINS) == len(PINS)


@pytest.mark.parametrize("pin", DEVICE_PINS, ids=[p.name for p in DEVICE_PINS])
def test_type_pin_on_device(ctx, oracle, pin):
    import roaringbitmap_amd as rb
    kind, _, what = pin.how.partition(":")
    inputs = pin.canonical_inputs()
    if kind == "build":
        out = ctx.upload_values([inputs[0][1]])
        want = oracle.RefBitmap.of(inputs[0][1]).serialize()
    elif kind == "runopt":
        s = ctx.upload_soa(one_container_soa(inputs))
        out, any_run = s.run_optimize()
        ref = oracle_bitmap(oracle, *inputs[0])
        assert bool(any_run[0]) == ref.run_optimize(), pin.cite
        want = ref.serialize()
    elif kind == "inplace":
        s = ctx.upload_soa(one_container_soa(inputs))
        refs = [oracle_bitmap(oracle, t, v) for t, v in inputs]
        out = ctx.pairwise_inplace(OPS[what], s, s, [0], [1])
        oracle.op_inplace(OPS[what], refs[0], refs[1])
        want = refs[0].serialize()
    else:
        s = ctx.upload_soa(one_container_soa(inputs))
        refs = [oracle_bitmap(oracle, t, v) for t, v in inputs]
        if kind == "op":
            out = ctx.pairwise(OPS[what], s, s, [0], [1])
            want = oracle.op(OPS[what], refs[0], refs[1]).serialize()
        else:
            out = ctx.wide(getattr(rb, what), s)
            want = oracle.wide(getattr(oracle, what), refs).serialize()
    h = out.download()
    assert out.serialize()[0] == want, pin.cite
    if pin.expect is not None:
        assert len(h.type) == 1 and int(h.type[0]) == pin.expect, \
            f"{pin.cite}: {[TYPE_NAME[int(t)] for t in h.type]} != {TYPE_NAME[pin.expect]}"
    if pin.card is not None:
        assert int(h.card.sum()) == pin.card, pin.cite


@pytest.mark.parametrize("opname", list(OPS))
def test_run_argument_equivalence_on_device(ctx, oracle, opname):
    """RunContainerArg_Array{AND,ANDNOT,OR,XOR} (TestRunContainer.java:2294-2416) on the device: b_k op
    r_l and b_k op b_l have the same content and each equals the oracle's bytes (Run operands of up to
    32768 runs take the > 8 KiB staging path)."""
    op = OPS[opname]
    n = len(RUN_ARG_SETS)
    conts = [(RUN, v) for v in RUN_ARG_SETS] + [(ab_type(v), v) for v in RUN_ARG_SETS]
    s = ctx.upload_soa(one_container_soa(conts))
    refs = [oracle_bitmap(oracle, t, v) for t, v in conts]
    a_idx = np.repeat(np.arange(n, 2 * n), n).astype(np.uint32)          # b_k
    b_run = np.tile(np.arange(n), n).astype(np.uint32)                   # r_l
    b_oth = b_run + n                                                    # b_l
    got_r = ctx.pairwise(op, s, s, a_idx, b_run)
    got_o = ctx.pairwise(op, s, s, a_idx, b_oth)
    br, bo = got_r.serialize(), got_o.serialize()
    hr, ho = got_r.download(), got_o.download()
    for i in range(n * n):
        assert br[i] == oracle.op(op, refs[a_idx[i]], refs[b_run[i]]).serialize(), (opname, i)
        assert bo[i] == oracle.op(op, refs[a_idx[i]], refs[b_oth[i]]).serialize(), (opname, i)
        assert np.array_equal(hr.values(i), ho.values(i)), (opname, i)

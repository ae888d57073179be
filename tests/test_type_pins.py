"""The oracle against the reference's own container-type assertions (tests/type_pins.py lists them with
their file:line): every on-path `instanceof` pin of TestContainer / TestRunContainer /
TestBitmapContainer / TestArrayContainer, plus the Run-argument equivalence loops of TestRunContainer."""
import numpy as np
import pytest

from type_pins import (PINS, RUN, RUN_ARG_SETS, TYPE_NAME, ab_type, n_on_path_pins, oracle_bitmap)

OPS = {"AND": 0, "OR": 1, "XOR": 2, "ANDNOT": 3}


def oracle_result(oracle, pin):
    """(type, card) of the one result container of the pin's entry point, or (None, 0) if empty."""
    R = oracle
    kind, _, what = pin.how.partition(":")
    if kind == "build":
        b = R.RefBitmap.of(pin.inputs[0][1])
    elif kind == "runopt":
        b = oracle_bitmap(R, *pin.inputs[0])
        b.run_optimize()
    elif kind == "op":
        b = R.op(OPS[what], oracle_bitmap(R, *pin.inputs[0]), oracle_bitmap(R, *pin.inputs[1]))
    elif kind == "inplace":
        b = oracle_bitmap(R, *pin.inputs[0])
        R.op_inplace(OPS[what], b, oracle_bitmap(R, *pin.inputs[1]))
    elif kind == "wide":
        b = R.wide(getattr(R, what), [oracle_bitmap(R, t, v) for t, v in pin.inputs])
    else:
        raise ValueError(pin.how)
    cs = b.containers()
    assert len(cs) <= 1
    return (cs[0][1], cs[0][2]) if cs else (None, 0)


def test_pin_inventory():
    # 54 of the 88 instanceof lines are on the set-algebra path (the rest: Container.not/inot, comments)
    assert n_on_path_pins() == 54
    assert len({p.name for p in PINS}) == len(PINS)


@pytest.mark.parametrize("pin", PINS, ids=[p.name for p in PINS])
def test_reference_type_pin(oracle, pin):
    t, c = oracle_result(oracle, pin)
    if pin.expect is not None:
        assert t == pin.expect, f"{pin.cite}: {TYPE_NAME.get(t)} != {TYPE_NAME[pin.expect]}"
    if pin.card is not None:
        assert c == pin.card, pin.cite


@pytest.mark.parametrize("pin", [p for p in PINS if p.how in ("build", "runopt") and p.inputs[0][0] != RUN],
                         ids=lambda p: p.name)
def test_host_construction_matches_pins(pin):
    """The product's host builders (bitmapOf, bitmapOf + runOptimize: engine.soa_from_values) make the
    container types these pins assert."""
    from roaringbitmap_amd.engine import soa_from_values
    h = soa_from_values([pin.inputs[0][1]], run_optimize=pin.how == "runopt")
    assert len(h.type) == 1 and int(h.type[0]) == pin.expect, pin.cite


@pytest.mark.parametrize("opname", list(OPS))
def test_run_argument_equivalence(oracle, opname):
    """RunContainerArg_Array{AND,ANDNOT,OR,XOR} (TestRunContainer.java:2294-2416): for every pair of
    getSetOfRunContainers (:81-153), b_k op r_l has the content of b_k op b_l."""
    R = oracle
    op = OPS[opname]
    runs = [oracle_bitmap(R, RUN, v) for v in RUN_ARG_SETS]
    others = [oracle_bitmap(R, ab_type(v), v) for v in RUN_ARG_SETS]
    for k in range(len(RUN_ARG_SETS)):
        for l in range(len(RUN_ARG_SETS)):
            a = R.op(op, others[k], runs[l]).to_array()
            b = R.op(op, others[k], others[l]).to_array()
            assert np.array_equal(a, b), (opname, k, l)

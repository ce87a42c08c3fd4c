"""Edge-function programs (TGO_EDGE_PROGRAM): the EdgeExpr DSL's postfix
compilation, and the oracle's restatement of the program (fr_set_edge_program, edge_fn 8)
pinned against an independent Python evaluation in Java arithmetic.

The check per entry: the oracle's combiner-less receive (fr_gather_lists) with the program
must equal the program evaluated here on the same entry's message (the receive with the
identity function) and weight (the receive with the program ``W``), in the same order.  CPU
only (the oracle and the host DSL); the device against the oracle: tests/test_gpu_edge_program.py.
"""
import math

import numpy as np
import pytest

import fulgora as fr
from titan_amd import _lib as L
from titan_amd import rmat_edges
from titan_amd.generic import EdgeExpr, M, MessageScope, W

IN, OUT, BOTH = L.SCOPE_IN_E, L.SCOPE_OUT_E, L.SCOPE_BOTH_E
I64_MIN, I64_MAX = -(1 << 63), (1 << 63) - 1


def wrap(x):
    return ((x - I64_MIN) % (1 << 64)) + I64_MIN


def java_long(op, a, b):
    if op == L.OP_ADD:
        return wrap(a + b)
    if op == L.OP_SUB:
        return wrap(a - b)
    if op == L.OP_MUL:
        return wrap(a * b)
    if op in (L.OP_DIV, L.OP_REM):
        if b == 0:
            raise ZeroDivisionError
        q = abs(a) // abs(b)
        q = q if (a < 0) == (b < 0) else -q
        return wrap(q) if op == L.OP_DIV else wrap(a - b * q)
    return min(a, b) if op == L.OP_MIN else max(a, b)


def java_double(op, a, b):
    if op == L.OP_ADD:
        return a + b
    if op == L.OP_SUB:
        return a - b
    if op == L.OP_MUL:
        return a * b
    if op == L.OP_DIV:
        if b == 0.0:
            return math.nan if a == 0.0 or a != a else math.copysign(math.inf, a) * math.copysign(1.0, b)
        return a / b
    if op == L.OP_REM:
        return math.nan if b == 0.0 or math.isinf(a) else math.fmod(a, b)
    if op == L.OP_MIN:
        if a != a:
            return a
        if a == 0.0 and b == 0.0 and math.copysign(1.0, b) < 0:
            return b
        return a if a <= b else b
    if a != a:
        return a
    if a == 0.0 and b == 0.0 and math.copysign(1.0, a) < 0:
        return b
    return a if a >= b else b


def java_eval(e: EdgeExpr, m, w, is_long):
    """The expression tree evaluated directly (no postfix program), Java semantics."""
    if e.op == L.OP_MSG:
        return m
    if e.op == L.OP_WEIGHT:
        return w
    if e.op == L.OP_CONST:
        return int(e.value) if is_long else float(e.value)
    a = java_eval(e.args[0], m, w, is_long)
    if e.op == L.OP_NEG:
        return wrap(-a) if is_long else -a
    if e.op == L.OP_ABS:
        if is_long:
            return wrap(-a) if a < 0 else a
        return 0.0 - a if a <= 0.0 else a
    b = java_eval(e.args[1], m, w, is_long)
    return java_long(e.op, a, b) if is_long else java_double(e.op, a, b)


LONG_EXPRS = [M + W, (M * 3 - W) % 7, (M / W).max(-5), abs(-M) * 2 + 1, M.min(W * 1000) - 4,
              M * 9223372036854775807 + W, -(M % (W + 1)) / 2, (M - W).max(W - M) * (M + 1)]
DOUBLE_EXPRS = [M + W, (M * 2.5 - W) / 3.0, (M % 1.5).min(W), abs(M) - W * 0.5, (-M).max(W / 7.0) * M,
                M / (W - W), (M * 0.0).min(-0.0)]


def test_compile_postfix_and_constants():
    ops, ic, fc = ((M * 2 + W).min(7) - abs(-M) % 3).compile()
    assert ops == [L.OP_MSG, L.OP_CONST | 0 << 8, L.OP_MUL, L.OP_WEIGHT, L.OP_ADD, L.OP_CONST | 1 << 8, L.OP_MIN,
                   L.OP_MSG, L.OP_NEG, L.OP_ABS, L.OP_CONST | 2 << 8, L.OP_REM, L.OP_SUB]
    assert ic == [2, 7, 3] and fc == [2.0, 7.0, 3.0]
    ops, ic, fc = (M / 2.5 + 2).compile()           # a non-integral constant: double messages only
    assert ic is None and fc == [2.5, 2.0]
    ops, ic, fc = (M + 2 + 2.0).compile()           # 2 and 2.0 are two constants (int vs float)
    assert len(fc) == 2
    assert (M + W) == (M + W) and hash(M + W) == hash(M + W) and (M + W) != (W + M)
    assert MessageScope.Local("inE", M + 1) == MessageScope.Local("inE", M + 1)
    with pytest.raises(ValueError):
        (M + (1 << 63)).compile()
    with pytest.raises(TypeError):
        M + "x"
    big = M
    for i in range(20):
        big = big + i
    with pytest.raises(ValueError):
        big.compile()                                # > 32 ops


@pytest.fixture(scope="module")
def oracle_graph():
    n = 1 << 8
    src, dst, w = rmat_edges(8, 8, seed=5, weights=True)
    return n, fr.OracleGraph.from_edges(n, src, dst, w)


def entry_lists(o, scope, vt, msg, has):
    fr.set_edge_program([L.OP_WEIGHT], [], [])
    off_w, ws = o.gather_lists(scope, vt, L.EDGE_PROGRAM, msg, has)
    off_m, ms = o.gather_lists(scope, vt, L.EDGE_IDENTITY, msg, has)
    assert np.array_equal(off_w, off_m)
    return off_m, ms, ws


@pytest.mark.parametrize("scope", [IN, OUT, BOTH])
def test_oracle_program_long_equals_java_evaluation(oracle_graph, scope):
    n, o = oracle_graph
    rng = np.random.default_rng(3)
    msg = rng.integers(-(1 << 62), 1 << 62, n)
    msg[:4] = [I64_MIN, I64_MAX, 0, -1]
    has = rng.random(n) < 0.7
    off, ms, ws = entry_lists(o, scope, L.VAL_INT64, msg, has)
    for e in LONG_EXPRS:
        ops, ic, fc = e.compile()
        fr.set_edge_program(ops, ic, fc)
        off2, got = o.gather_lists(scope, L.VAL_INT64, L.EDGE_PROGRAM, msg, has)
        assert np.array_equal(off2, off)
        exp = [java_eval(e, int(m), int(w), True) for m, w in zip(ms[:off[-1]], ws[:off[-1]])]
        assert [int(x) for x in got[:off[-1]]] == exp, e
        # with a combiner: the MIN over each vertex's stream
        got_c, gh = o.gather(scope, L.VAL_INT64, L.COMBINE_MIN, L.EDGE_PROGRAM, msg, has)
        for v in range(0, n, 17):
            seg = exp[off[v]:off[v + 1]]
            assert gh[v] == bool(seg) and (not seg or got_c[v] == min(seg)), (e, v)


@pytest.mark.parametrize("scope", [IN, BOTH])
def test_oracle_program_double_equals_java_evaluation(oracle_graph, scope):
    n, o = oracle_graph
    rng = np.random.default_rng(4)
    msg = rng.standard_normal(n) * 100
    msg[:5] = [0.0, -0.0, math.inf, -math.inf, math.nan]
    has = rng.random(n) < 0.7
    off, ms, ws = entry_lists(o, scope, L.VAL_FP64, msg, has)
    for e in DOUBLE_EXPRS:
        ops, ic, fc = e.compile()
        fr.set_edge_program(ops, ic, fc)
        _, got = o.gather_lists(scope, L.VAL_FP64, L.EDGE_PROGRAM, msg, has)
        exp = np.array([java_eval(e, float(m), float(w), False) for m, w in zip(ms[:off[-1]], ws[:off[-1]])])
        # bitwise, NaN payloads aside (signed zeros included)
        g = got[:off[-1]]
        assert np.array_equal(np.isnan(g), np.isnan(exp)), e
        ok = ~np.isnan(exp)
        assert np.array_equal(g[ok].view(np.int64), exp[ok].view(np.int64)), e


def test_oracle_program_division_by_zero_throws(oracle_graph):
    n, o = oracle_graph
    fr.set_edge_program(*(M / (W - W)).compile())
    with pytest.raises(RuntimeError):
        o.gather(IN, L.VAL_INT64, L.COMBINE_SUM, L.EDGE_PROGRAM, np.ones(n, np.int64), np.ones(n, bool))

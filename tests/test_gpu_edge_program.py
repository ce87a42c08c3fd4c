"""GPU: edge-function programs (TGO_EDGE_PROGRAM) — the device's per-entry
interpretation of an EdgeExpr against the oracle's restatement (fr_set_edge_program, pinned
against a Python evaluation in Java arithmetic by tests/test_edge_program.py).

Bars: int64 bit-exact (combined and per-entry lists); fp64 per-entry lists bitwise (NaN
payloads aside), fp64 MIN/MAX bitwise, fp64 SUM within 1e-12 relative (the device folds each
in-list in its own list order); errors as the reference's: a division by zero in long
arithmetic and a weight read on an edge without the property fail the program."""
import numpy as np
import pytest

import fulgora as fr
from test_edge_program import DOUBLE_EXPRS, LONG_EXPRS
from generic_programs import OracleEngine
from titan_amd import Engine, Schema, TitanException, rmat_edges
from titan_amd import _lib as L
from titan_amd.generic import M, W, GenericVertexProgram, MessageScope
from conftest import load_fixture

pytestmark = pytest.mark.gpu

OUT, IN, BOTH = L.SCOPE_OUT_E, L.SCOPE_IN_E, L.SCOPE_BOTH_E


@pytest.fixture(scope="module")
def graph():
    n = 1 << 11
    src, dst, w = rmat_edges(11, 8, seed=31, weights=True)
    return n, src, dst, w


def same_bits(a, b):
    return np.array_equal(np.isnan(a), np.isnan(b)) and np.array_equal(a[~np.isnan(a)].view(np.int64),
                                                                       b[~np.isnan(b)].view(np.int64))


@pytest.mark.parametrize("load_scope,scope", [(IN, IN), (OUT, OUT), (BOTH, BOTH), (BOTH, IN)])
def test_program_gather_matches_oracle(graph, load_scope, scope):
    n, src, dst, w = graph
    eng = Engine().load_edges(n, src, dst, load_scope, weight=w, apply_cap=False)
    o = fr.OracleGraph.from_edges(n, src, dst, w)
    assert np.array_equal(eng.vertex_ids(), o.vertex_ids())
    rng = np.random.default_rng(17)
    for vt, exprs in ((L.VAL_INT64, LONG_EXPRS), (L.VAL_FP64, DOUBLE_EXPRS)):
        msg = rng.integers(-(1 << 62), 1 << 62, n) if vt == L.VAL_INT64 else rng.standard_normal(n) * 100
        if vt == L.VAL_FP64:
            msg[:5] = [0.0, -0.0, np.inf, -np.inf, np.nan]
        has = rng.random(n) < 0.6
        for e in exprs:
            ops, ic, fc = e.compile()
            eng.set_edge_program(ops, ic, fc)
            fr.set_edge_program(ops, ic, fc)
            if vt == L.VAL_INT64 and e == (M / (W - W)):
                continue
            for comb in (L.COMBINE_SUM, L.COMBINE_MIN, L.COMBINE_MAX):
                # a MIN / MAX fold over a stream holding NaN depends on the stream's order (the
                # device folds list order, the oracle row order): those folds run NaN-free
                mc = msg
                if vt == L.VAL_FP64 and comb != L.COMBINE_SUM:
                    if e == (M / (W - W)):
                        continue
                    mc = np.where(np.isnan(msg), 0.5, msg)
                got, gh = eng.gather(scope, vt, comb, L.EDGE_PROGRAM, mc, has)
                exp, eh = o.gather(scope, vt, comb, L.EDGE_PROGRAM, mc, has)
                assert np.array_equal(gh, eh), (e, comb)
                if vt == L.VAL_INT64:
                    assert np.array_equal(got[gh], exp[eh]), (e, comb)
                elif comb != L.COMBINE_SUM:
                    assert same_bits(got[gh], exp[eh]), (e, comb)
                else:
                    np.testing.assert_allclose(got[gh], exp[eh], rtol=1e-12, atol=1e-300)
            if load_scope == BOTH and scope == BOTH:
                continue                          # lists: the scope-matched loads cover the order
            goff, gv = eng.gather_lists(scope, vt, L.EDGE_PROGRAM, msg, has)
            eoff, ev = o.gather_lists(scope, vt, L.EDGE_PROGRAM, msg, has)
            assert np.array_equal(goff, eoff), e
            if vt == L.VAL_INT64:
                assert np.array_equal(gv[:goff[-1]], ev[:eoff[-1]]), e
            else:
                assert same_bits(gv[:goff[-1]], ev[:eoff[-1]]), e


def test_program_menu_equivalence(graph):
    """M + W, M * W, M - W, M.min(W), M.max(W), M / W, M + 1 and M as programs give exactly the
    menu functions' results."""
    n, src, dst, w = graph
    eng = Engine().load_edges(n, src, dst, IN, weight=w, apply_cap=False)
    rng = np.random.default_rng(5)
    msg = rng.integers(-(1 << 40), 1 << 40, n)
    pairs = [(M + W, L.EDGE_ADD_WEIGHT), (M * W, L.EDGE_MUL_WEIGHT), (M - W, L.EDGE_SUB_WEIGHT),
             (M.min(W), L.EDGE_MIN_WEIGHT), (M.max(W), L.EDGE_MAX_WEIGHT), (M / W, L.EDGE_DIV_WEIGHT),
             (M + 1, L.EDGE_ADD_ONE)]
    for e, fn in pairs:
        eng.set_edge_program(*e.compile())
        a, ah = eng.gather(IN, L.VAL_INT64, L.COMBINE_SUM, L.EDGE_PROGRAM, msg)
        b, bh = eng.gather(IN, L.VAL_INT64, L.COMBINE_SUM, fn, msg)
        assert np.array_equal(ah, bh) and np.array_equal(a, b), e


def test_program_errors(graph):
    n, src, dst, w = graph
    eng = Engine().load_edges(n, src, dst, IN, weight=w, apply_cap=False)
    msg = np.ones(n, np.int64)
    with pytest.raises(TitanException) as e:
        eng.gather(IN, L.VAL_INT64, L.COMBINE_SUM, L.EDGE_PROGRAM, msg)          # no program set
    assert e.value.code == L.TGO_E_STATE
    eng.set_edge_program(*(M / (W - W)).compile())
    with pytest.raises(TitanException) as e:
        eng.gather(IN, L.VAL_INT64, L.COMBINE_SUM, L.EDGE_PROGRAM, msg)          # long / 0 throws
    assert e.value.code == L.TGO_E_PROGRAM
    got, gh = eng.gather(IN, L.VAL_FP64, L.COMBINE_MAX, L.EDGE_PROGRAM, msg.astype(np.float64))  # double: 1/0
    assert gh.any() and np.isposinf(got[gh]).all()
    eng.set_edge_program(*(M / 2.5).compile())
    with pytest.raises(TitanException) as e:
        eng.gather(IN, L.VAL_INT64, L.COMBINE_SUM, L.EDGE_PROGRAM, msg)          # no long constants
    assert e.value.code == L.TGO_E_INVALID
    bad = [[L.OP_ADD], [L.OP_MSG, L.OP_MSG], [L.OP_CONST | 3 << 8], [L.OP_MSG | 1 << 8], [99],
           [L.OP_MSG] * 9 + [L.OP_ADD] * 8, []]
    for ops in bad:
        with pytest.raises(TitanException) as e:
            eng.set_edge_program(ops, [1], [1.0])
        assert e.value.code == L.TGO_E_INVALID, ops
    plain = Engine().load_edges(n, src, dst, IN)
    plain.set_edge_program(*(M + 1).compile())                                   # no weight read: fine
    got, gh = plain.gather(IN, L.VAL_INT64, L.COMBINE_SUM, L.EDGE_PROGRAM, msg)
    ref, rh = plain.gather(IN, L.VAL_INT64, L.COMBINE_SUM, L.EDGE_ADD_ONE, msg)
    assert np.array_equal(got, ref) and np.array_equal(gh, rh)
    plain.set_edge_program(*(M + W).compile())
    with pytest.raises(TitanException) as e:
        plain.gather(IN, L.VAL_INT64, L.COMBINE_SUM, L.EDGE_PROGRAM, msg)        # no weight property loaded
    assert e.value.code == L.TGO_E_INVALID
    eng.set_edge_program(None)
    with pytest.raises(TitanException):
        eng.gather(IN, L.VAL_INT64, L.COMBINE_SUM, L.EDGE_PROGRAM, msg)


def test_program_weight_read_on_edge_without_property_fails():
    """GotG: `time` exists only on battled edges: a program that reads W fails there, one that
    does not runs."""
    rows, vids, sd, npz = load_fixture("gotg")
    eng = Engine().load_rows(rows, Schema.from_dict(sd), BOTH, weight_key=sd["property_keys"][0][0])
    n = eng.n
    eng.set_edge_program(*(M * 2 + W).compile())
    with pytest.raises(TitanException) as e:
        eng.gather(BOTH, L.VAL_INT64, L.COMBINE_SUM, L.EDGE_PROGRAM, np.zeros(n, np.int64))
    assert e.value.code == L.TGO_E_PROGRAM
    eng.set_edge_program(*(M * 2 - 1).compile())
    got, gh = eng.gather(BOTH, L.VAL_INT64, L.COMBINE_SUM, L.EDGE_PROGRAM, np.ones(n, np.int64))
    ref, rh = eng.gather(BOTH, L.VAL_INT64, L.COMBINE_SUM, L.EDGE_IDENTITY, np.ones(n, np.int64))
    assert np.array_equal(gh, rh) and np.array_equal(got, ref)                    # each message 2*1-1 = 1


class WeightedHops(GenericVertexProgram):
    """A k-superstep relaxation whose edge function is an EdgeExpr: dist' = min over in-entries
    of (2 * dist + w) % 1000003 — no menu function computes it."""
    value_type = L.VAL_INT64
    combiner = L.COMBINE_MIN
    compute_keys = ("d",)
    SCOPE = MessageScope.Local("inE", (M * 2 + W) % 1000003)

    def __init__(self, steps=4):
        self.steps = steps

    def getMessageScopes(self, memory):  # noqa: N802
        return [self.SCOPE]

    def execute(self, v, messenger, memory):
        if memory.isInitialIteration():
            d = v.ids % 97
            v.set_property("d", d)
            messenger.send(self.SCOPE, d)
            return
        cur, _ = v.property("d")
        got, has = messenger.receive(self.SCOPE)
        nd = np.where(has, np.minimum(got, cur), cur)
        v.set_property("d", nd)
        messenger.send(self.SCOPE, nd)

    def terminate(self, memory):
        return memory.getIteration() >= self.steps


def test_program_in_a_generic_vertex_program(graph):
    from titan_amd.generic import FulgoraMemory, run_generic
    n, src, dst, w = graph
    eng = Engine().load_edges(n, src, dst, IN, weight=w, apply_cap=False)
    o = OracleEngine(fr.OracleGraph.from_edges(n, src, dst, w))
    got = run_generic(eng, WeightedHops(), FulgoraMemory())
    exp = run_generic(o, WeightedHops(), FulgoraMemory())
    assert np.array_equal(got.ids, exp.ids)
    gd, gp = got.property("d")
    ed, ep = exp.property("d")
    assert np.array_equal(gp, ep) and np.array_equal(gd, ed)
    assert not np.array_equal(gd, got.ids % 97)                                   # the supersteps did something

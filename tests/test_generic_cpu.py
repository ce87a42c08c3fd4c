"""CPU: FulgoraMemory semantics, the oracle's generic message primitives, and Fulgora's
superstep loop (titan_amd/generic.py run_generic) driven through the oracle double.

References: FulgoraMemory.java:21-131 (memory), VertexMemoryHandler.java:77-117 (receive /
send), VertexState.java:55-89 (double-buffered messages, addMessage), FulgoraGraphComputer
.java:140-189 (loop order: setup, completeSubRound, execute, completeIteration,
completeSubRound, terminate, incrIteration, completeSubRound).
"""
import numpy as np
import pytest

import fulgora as fr
from generic_programs import ConnectedComponents, GenericPageRank, GlobalDegreeSum, OracleEngine
from titan_amd import FulgoraMemory, rmat_edges
from titan_amd.generic import run_generic

IN, OUT, BOTH = 1, 0, 2


def test_fulgora_memory_semantics():
    m = FulgoraMemory(["a", "b", "c"])
    assert m.isInitialIteration() and m.keys() == set()
    m.incr("a", 2)
    m.incr("a", 3)                          # accumulates in the current map
    with pytest.raises(KeyError):
        m.get("a")                          # reads go to the previous map
    m.completeSubRound()
    assert m.get("a") == 5
    m.and_("b", True)
    m.and_("b", False)
    m.or_("c", False)
    m.or_("c", True)
    m.completeSubRound()
    assert (m.get("b"), m.get("c")) == (False, True)
    m.incr("a", 1)                          # the current map is never cleared
    m.completeSubRound()
    assert m.get("a") == 6
    with pytest.raises(ValueError):
        m.set("zzz", 1)                     # providedKeyIsNotAMemoryComputeKey
    with pytest.raises(ValueError):
        m.set("a", None)
    m.incrIteration()
    m.incrIteration()
    m.complete()                            # complete() steps the iteration back (:73-76)
    assert m.getIteration() == 1


def python_gather(off, mid, adj, w, scope, vt, comb, fn, msg, has):
    """Plain restatement on the exported adjacency (OUT entries [off, mid), IN [mid, off+1))."""
    n = len(off) - 1
    out = np.zeros(n, np.int64 if vt == 0 else np.float64)
    oh = np.zeros(n, bool)
    for v in range(n):
        ranges = {OUT: [(off[v], mid[v])] if scope == IN else [], IN: [(mid[v], off[v + 1])] if scope == OUT else []}
        rr = ranges[OUT] + ranges[IN] if scope != BOTH else [(off[v], off[v + 1])]
        acc, any_ = None, False
        for b, e in rr:
            for k in range(b, e):
                u = adj[k]
                if not has[u]:
                    continue
                m = msg[u]
                x = w[k] if fn >= 2 else 0
                if fn == 1:
                    m = m + 1
                elif fn == 2:
                    m = m + x
                elif fn == 3:
                    m = m * x
                elif fn == 4:
                    m = m - x
                elif fn == 5:
                    m = min(m, x)
                elif fn == 6:
                    m = max(m, x)
                elif fn == 7:                      # Java: long / truncates toward zero
                    m = (abs(int(m)) // abs(int(x))) * (1 if (m < 0) == (x < 0) else -1) if vt == 0 else m / x
                if vt == 0:
                    m = np.int64(m)
                if not any_:
                    acc, any_ = m, True
                elif comb == 0:
                    acc = acc + m
                elif comb == 1:
                    acc = min(acc, m)
                else:
                    acc = max(acc, m)
        if any_:
            out[v], oh[v] = acc, True
    return out, oh


@pytest.mark.parametrize("scope", [IN, OUT, BOTH])
@pytest.mark.parametrize("vt,comb,fn", [(0, 0, 0), (0, 1, 2), (0, 2, 1), (1, 0, 3), (1, 1, 0), (1, 0, 2),
                                        (0, 0, 4), (0, 1, 5), (0, 2, 6), (0, 0, 7), (1, 0, 4), (1, 1, 5),
                                        (1, 2, 6), (1, 0, 7)])
def test_oracle_gather_matches_plain_restatement(scope, vt, comb, fn):
    scale = 7
    n = 1 << scale
    src, dst, w = rmat_edges(scale, 4, seed=12, weights=True)
    o = fr.OracleGraph.from_edges(n, src, dst, w)
    off, mid, adj, ww = o.export(weighted=True)
    rng = np.random.default_rng(3)
    msg = rng.integers(-1000, 1000, n) if vt == 0 else rng.standard_normal(n)
    has = rng.random(n) < 0.7
    got = o.gather(scope, vt, comb, fn, msg, has)
    exp = python_gather(off, mid, adj, ww, scope, vt, comb, fn, msg, has)
    assert np.array_equal(got[1], exp[1])
    if vt == 0:
        assert np.array_equal(got[0], exp[0])
    else:
        np.testing.assert_allclose(got[0], exp[0], rtol=1e-12, atol=1e-12)


def test_oracle_combine_global_folds_in_send_order():
    t = np.array([3, 1, 3, 3, 7, 1], np.int64)
    v = np.array([0.1, 2.0, 0.2, 0.3, 5.0, -1.0])
    out, has = fr.combine_global(8, 1, 0, t, v)
    assert has.tolist() == [False, True, False, True, False, False, False, True]
    assert out[3] == (0.1 + 0.2) + 0.3 and out[1] == 2.0 + -1.0
    out, _ = fr.combine_global(8, 0, 2, t, np.array([4, 9, -2, 8, 1, 11], np.int64))
    assert (out[3], out[1], out[7]) == (8, 11, 1)


def components(n, src, dst):
    parent = np.arange(n)

    def find(x):
        while parent[x] != x:
            parent[x] = parent[parent[x]]
            x = parent[x]
        return x
    for a, b in zip(src, dst):
        ra, rb = find(a), find(b)
        if ra != rb:
            parent[max(ra, rb)] = min(ra, rb)
    return np.array([find(i) for i in range(n)])


def test_connected_components_through_the_oracle_loop():
    scale = 9
    n = 1 << scale
    src, dst, _ = rmat_edges(scale, 2, seed=4)
    o = fr.OracleGraph.from_edges(n, src, dst)
    ids = o.vertex_ids()
    mem = FulgoraMemory(ConnectedComponents.memory_compute_keys)
    verts = run_generic(OracleEngine(o), ConnectedComponents(), mem)
    cc, present = verts.property("cc")
    assert present.all()
    root = components(n, src, dst)
    # label = smallest Titan id of the component; ids grow with the dense index here
    assert np.array_equal(cc, ids[root])
    assert mem.get("any") is True and mem.get("changes") > 0


@pytest.mark.parametrize("iters", [1, 2, 7])
def test_generic_pagerank_equals_the_native_restatement(iters):
    scale = 8
    n = 1 << scale
    src, dst, _ = rmat_edges(scale, 8, seed=6)
    o = fr.OracleGraph.from_edges(n, src, dst)
    mem = FulgoraMemory()
    verts = run_generic(OracleEngine(o), GenericPageRank(0.85, n, iters), mem)
    pr, present = verts.property("pr")
    opr, it = o.pagerank(0.85, n, iters)
    assert present.all()
    np.testing.assert_allclose(pr, opr, rtol=1e-12)
    mem.complete()
    assert mem.getIteration() == it == iters


def test_global_scope_program_through_the_oracle_loop():
    scale = 8
    n = 1 << scale
    src, dst, w = rmat_edges(scale, 8, seed=9, weights=True)
    o = fr.OracleGraph.from_edges(n, src, dst, w)
    ids = o.vertex_ids()
    hubs = ids[[5, 77, 200]]
    mem = FulgoraMemory(GlobalDegreeSum.memory_compute_keys)
    verts = run_generic(OracleEngine(o), GlobalDegreeSum(hubs), mem)
    inbox, has = verts.property("inbox")
    # weighted in-degree by the inE scope: a receiver walks its OUT entries
    wdeg = np.bincount(src, weights=w, minlength=n).astype(np.int64)
    exp = {int(h): 0 for h in hubs}
    for i in range(n):
        exp[int(hubs[ids[i] % len(hubs)])] += int(wdeg[i])
    pos = {int(v): i for i, v in enumerate(ids)}
    assert has.sum() == 3
    for h, s in exp.items():
        assert inbox[pos[h]] == s
    assert mem.get("total") == int(wdeg.sum()) and mem.get("best") == max(exp.values())


def python_lists(off, mid, adj, w, scope, vt, fn, msg, has):
    """Per-vertex message streams on the exported adjacency (OUT entries first, in stored
    order = column order for an edge-list graph of one label)."""
    n = len(off) - 1
    o2 = np.zeros(n + 1, np.int64)
    vals = []
    for v in range(n):
        rr = {IN: [(off[v], mid[v])], OUT: [(mid[v], off[v + 1])], BOTH: [(off[v], off[v + 1])]}[scope]
        for b, e in rr:
            for k in range(b, e):
                u = adj[k]
                if has[u]:
                    m = python_gather(np.array([0, 1]), np.array([1]), np.array([0]), np.array([w[k]]), IN, vt, 0, fn,
                                      np.array([msg[u]]), np.array([True]))[0][0]
                    vals.append(m)
        o2[v + 1] = len(vals)
    return o2, np.array(vals, np.int64 if vt == 0 else np.float64)


@pytest.mark.parametrize("scope", [IN, OUT, BOTH])
@pytest.mark.parametrize("vt,fn", [(0, 0), (0, 4), (1, 2), (1, 7)])
def test_oracle_gather_lists_are_the_streams_in_column_order(scope, vt, fn):
    """fr_gather_lists: no combiner — each vertex's stream as VertexMemoryHandler.receiveMessages
    yields it (VertexMemoryHandler.java:83-92): the row's entries in column order, null
    messages filtered, edgeFct applied."""
    scale = 6
    n = 1 << scale
    src, dst, w = rmat_edges(scale, 4, seed=14, weights=True)
    o = fr.OracleGraph.from_edges(n, src, dst, w)
    off, mid, adj, ww = o.export(weighted=True)
    rng = np.random.default_rng(5)
    msg = rng.integers(-1000, 1000, n) if vt == 0 else rng.standard_normal(n)
    has = rng.random(n) < 0.7
    got_off, got = o.gather_lists(scope, vt, fn, msg, has)
    exp_off, exp = python_lists(off, mid, adj, ww, scope, vt, fn, msg, has)
    assert np.array_equal(got_off, exp_off)
    if vt == 0:
        assert np.array_equal(got, exp)
    else:
        np.testing.assert_allclose(got, exp, rtol=1e-15)
    # folded with SUM the streams give the combined receive
    comb, ch = o.gather(scope, vt, 0, fn, msg, has)
    from titan_amd.generic import MessageLists
    red, rh = MessageLists(got_off, got).reduce(np.add)
    assert np.array_equal(rh, ch)
    assert np.allclose(red, comb, rtol=1e-12)


def test_oracle_integer_division_by_zero_fails():
    n = 4
    src, dst, w = np.array([0, 1], np.int32), np.array([1, 2], np.int32), np.array([3, 0], np.int32)
    o = fr.OracleGraph.from_edges(n, src, dst, w)
    with pytest.raises(RuntimeError):
        o.gather(IN, 0, 0, 7, np.ones(n, np.int64), np.ones(n, bool))
    out, has = o.gather(IN, 1, 0, 7, np.ones(n), np.ones(n, bool))          # double: IEEE infinity
    assert has[1] and np.isinf(out[1])


def test_combiner_less_program_through_the_oracle_loop():
    """A program without a combiner reads message streams (MessageLists): the first and the
    last message of each vertex and their count — order-sensitive, so the stream order matters."""
    from generic_programs import FirstLastCount
    scale = 7
    n = 1 << scale
    src, dst, w = rmat_edges(scale, 4, seed=22, weights=True)
    o = fr.OracleGraph.from_edges(n, src, dst, w)
    mem = FulgoraMemory()
    verts = run_generic(OracleEngine(o), FirstLastCount(), mem)
    first, fp = verts.property("first")
    cnt, _ = verts.property("count")
    off, mid, adj, ww = o.export(weighted=True)
    ids = o.vertex_ids()
    for v in range(n):
        ins = [int(ids[adj[k]] % 1000) - int(ww[k]) for k in range(off[v], mid[v])]    # inE: walk OUT entries, sub_weight
        assert cnt[v] == len(ins)
        assert fp[v] == bool(ins)
        if ins:
            assert first[v] == ins[0] and verts.property("last")[0][v] == ins[-1]


def test_global_scope_without_combiner_delivers_single_messages_only():
    from generic_programs import GlobalNoCombiner
    scale = 6
    n = 1 << scale
    src, dst, _ = rmat_edges(scale, 4, seed=23)
    o = fr.OracleGraph.from_edges(n, src, dst)
    ids = o.vertex_ids()
    verts = run_generic(OracleEngine(o), GlobalNoCombiner(ids, unique=True), FulgoraMemory())
    inbox, has = verts.property("inbox")
    assert has.sum() == n and np.array_equal(inbox, np.arange(n)[::-1] * 3)
    from titan_amd import TitanException
    with pytest.raises(TitanException):               # two messages meet at one target: ThrowingCombiner
        run_generic(OracleEngine(o), GlobalNoCombiner(ids, unique=False), FulgoraMemory())

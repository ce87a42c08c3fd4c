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
                if fn == 1:
                    m = m + 1
                elif fn == 2:
                    m = m + w[k]
                elif fn == 3:
                    m = m * w[k]
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
@pytest.mark.parametrize("vt,comb,fn", [(0, 0, 0), (0, 1, 2), (0, 2, 1), (1, 0, 3), (1, 1, 0), (1, 0, 2)])
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

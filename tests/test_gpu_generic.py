"""GPU: generic vertex programs.  The device's message combining
(tgo_gather, tgo_combine_global) against the oracle's restatement (fr_gather,
fr_combine_global), and whole vectorised programs run through the computer mirror against
the same programs driven through the oracle double.

Bars: int64 results and MIN/MAX bit-exact; fp64 SUM of a Local scope within 1e-12 relative
(the device folds each in-list in its own list order); Global fp64 SUM bit-exact (both fold
in send order); programs: int64 exact, PageRank within 1e-6 L1 of the native oracle.
"""
import numpy as np
import pytest

import fulgora as fr
from conftest import load_fixture
from generic_programs import (ConnectedComponents, FirstLastCount, GenericPageRank, GlobalDegreeSum, GlobalNoCombiner,
                              OracleEngine)
from titan_amd import (ComputeKeyMapReduce, Engine, ExecutionException, GpuGraph, Schema, TitanException,
                       TitanGraphComputer, rmat_edges)
from titan_amd import _lib as L

pytestmark = pytest.mark.gpu

OUT, IN, BOTH = L.SCOPE_OUT_E, L.SCOPE_IN_E, L.SCOPE_BOTH_E


def reorder(ids_from, values, ids_to):
    pos = {int(v): i for i, v in enumerate(ids_from)}
    return np.array([values[pos[int(v)]] for v in ids_to])


@pytest.fixture(scope="module")
def weighted_rmat():
    scale = 11
    n = 1 << scale
    src, dst, w = rmat_edges(scale, 8, seed=31, weights=True)
    return n, src, dst, w


@pytest.mark.parametrize("load_scope,scope", [(IN, IN), (OUT, OUT), (BOTH, BOTH), (BOTH, IN), (BOTH, OUT)])
def test_local_gather_matches_oracle(weighted_rmat, load_scope, scope):
    n, src, dst, w = weighted_rmat
    eng = Engine().load_edges(n, src, dst, load_scope, weight=w, apply_cap=False)
    o = fr.OracleGraph.from_edges(n, src, dst, w)
    ids = eng.vertex_ids()
    assert np.array_equal(ids, o.vertex_ids())
    rng = np.random.default_rng(7)
    for vt in (L.VAL_INT64, L.VAL_FP64):
        msg = rng.integers(-(1 << 40), 1 << 40, n) if vt == L.VAL_INT64 else rng.standard_normal(n)
        has = rng.random(n) < 0.6
        for comb in (L.COMBINE_SUM, L.COMBINE_MIN, L.COMBINE_MAX):
            for fn in (L.EDGE_IDENTITY, L.EDGE_ADD_ONE, L.EDGE_ADD_WEIGHT, L.EDGE_MUL_WEIGHT, L.EDGE_SUB_WEIGHT,
                       L.EDGE_MIN_WEIGHT, L.EDGE_MAX_WEIGHT, L.EDGE_DIV_WEIGHT):
                got, gh = eng.gather(scope, vt, comb, fn, msg, has)
                exp, eh = o.gather(scope, vt, comb, fn, msg, has)
                assert np.array_equal(gh, eh), (vt, comb, fn)
                if vt == L.VAL_INT64 or comb != L.COMBINE_SUM:
                    assert np.array_equal(got[gh], exp[eh]), (vt, comb, fn)
                else:
                    np.testing.assert_allclose(got[gh], exp[eh], rtol=1e-12, atol=1e-300)
                    again, _ = eng.gather(scope, vt, comb, fn, msg, has)
                    assert np.array_equal(got, again)            # fixed fold order


def test_gather_all_present_and_scope_checks(weighted_rmat):
    n, src, dst, w = weighted_rmat
    eng = Engine().load_edges(n, src, dst, IN, weight=w)
    o = fr.OracleGraph.from_edges(n, src, dst, w, hard_limit=100000)
    msg = np.arange(n, dtype=np.int64)
    got, gh = eng.gather(IN, L.VAL_INT64, L.COMBINE_MAX, L.EDGE_IDENTITY, msg)       # has = NULL: all present
    exp, eh = o.gather(IN, 0, 2, 0, msg, np.ones(n, bool))
    assert np.array_equal(gh, eh) and np.array_equal(got[gh], exp[eh])
    with pytest.raises(TitanException) as e:
        eng.gather(OUT, L.VAL_INT64, L.COMBINE_SUM, L.EDGE_IDENTITY, msg)            # not the preloaded slice
    assert e.value.code == L.TGO_E_INVALID
    plain = Engine().load_edges(n, src, dst, IN)
    with pytest.raises(TitanException):
        plain.gather(IN, L.VAL_INT64, L.COMBINE_SUM, L.EDGE_ADD_WEIGHT, msg)         # no weight property loaded


def test_weight_function_over_an_edge_without_the_property_fails():
    """GotG: `time` exists only on battled edges; reading it elsewhere throws in the
    reference (edge.value()), here TGO_E_PROGRAM."""
    rows, vids, sd, npz = load_fixture("gotg")
    eng = Engine().load_rows(rows, Schema.from_dict(sd), BOTH, weight_key=sd["property_keys"][0][0])
    n = eng.n
    with pytest.raises(TitanException) as e:
        eng.gather(BOTH, L.VAL_INT64, L.COMBINE_SUM, L.EDGE_ADD_WEIGHT, np.zeros(n, np.int64))
    assert e.value.code == L.TGO_E_PROGRAM


def test_global_combine_matches_oracle(weighted_rmat):
    n, src, dst, w = weighted_rmat
    eng = Engine().load_edges(n, src, dst, BOTH)
    rng = np.random.default_rng(11)
    m = 200000
    targets = rng.integers(0, n, m)
    targets[::7] = rng.integers(0, 16, len(targets[::7]))           # a few hot targets
    for vt in (L.VAL_INT64, L.VAL_FP64):
        vals = rng.integers(-(1 << 50), 1 << 50, m) if vt == L.VAL_INT64 else rng.standard_normal(m)
        for comb in (L.COMBINE_SUM, L.COMBINE_MIN, L.COMBINE_MAX):
            got, gh = eng.combine_global(vt, comb, targets, vals)
            exp, eh = fr.combine_global(n, vt, comb, targets, vals)
            assert np.array_equal(gh, eh)
            assert np.array_equal(got[gh], exp[eh]), (vt, comb)       # same (send) order: bit-exact
    got, gh = eng.combine_global(L.VAL_INT64, L.COMBINE_SUM, np.zeros(0, np.int64), np.zeros(0, np.int64))
    assert not gh.any()
    with pytest.raises(TitanException):
        eng.combine_global(L.VAL_INT64, L.COMBINE_SUM, np.array([n]), np.array([1]))
    ids = eng.vertex_ids()
    assert np.array_equal(eng.dense_ids(ids[[3, 0, 9]]), [3, 0, 9])
    assert eng.dense_ids(np.array([-5]))[0] == -1


def run_both(graph_args, program_factory, oracle, weight_keys=None, mr_key=None):
    graph = GpuGraph(**graph_args)
    computer = graph.compute()
    if weight_keys:
        computer.weight_keys = weight_keys
    computer.program(program_factory())
    if mr_key:
        computer.mapReduce(ComputeKeyMapReduce(*mr_key))
    result = computer.submit().get()
    from titan_amd import FulgoraMemory
    from titan_amd.generic import run_generic
    p = program_factory()
    mem = FulgoraMemory(p.memory_compute_keys)
    verts = run_generic(OracleEngine(oracle), p, mem)
    mem.complete()
    return result, verts, mem


def test_connected_components_program(weighted_rmat):
    n, src, dst, w = weighted_rmat
    o = fr.OracleGraph.from_edges(n, src, dst)
    result, verts, mem = run_both({"edges": (n, src, dst, None)}, ConnectedComponents, o, mr_key=("cc", "components"))
    ids, (cc, present) = result.vertex_properties["cc"][0], result.vertex_properties["cc"][1]
    assert present.all()
    assert np.array_equal(reorder(ids, cc, verts.ids), verts.property("cc")[0])
    assert result.memory().getIteration() == mem.getIteration()
    assert result.memory().get("changes") == mem.get("changes")
    kv = {x.getKey(): x.getValue() for x in result.memory().get("components")}
    assert len(kv) == n and all(kv[int(i)] == int(c) for i, c in zip(ids, cc))


def test_generic_pagerank_program(weighted_rmat):
    n, src, dst, w = weighted_rmat
    o = fr.OracleGraph.from_edges(n, src, dst)
    result, verts, mem = run_both({"edges": (n, src, dst, None)}, lambda: GenericPageRank(0.85, n, 10), o)
    ids, (pr, present) = result.vertex_properties["pr"]
    opr, it = o.pagerank(0.85, n, 10)
    assert present.all() and result.memory().getIteration() == it
    assert np.abs(reorder(ids, pr, o.vertex_ids()) - opr).sum() <= 1e-6
    np.testing.assert_allclose(reorder(ids, pr, verts.ids), verts.property("pr")[0], rtol=1e-12)


def test_global_scope_program(weighted_rmat):
    n, src, dst, w = weighted_rmat
    o = fr.OracleGraph.from_edges(n, src, dst, w)
    ids = o.vertex_ids()
    hubs = ids[[1, 500, 1999]]
    result, verts, mem = run_both({"edges": (n, src, dst, w)}, lambda: GlobalDegreeSum(hubs), o,
                                  weight_keys={"w": 1})
    gids, (inbox, has) = result.vertex_properties["inbox"]
    assert np.array_equal(reorder(gids, has, verts.ids), verts.property("inbox")[1])
    assert np.array_equal(reorder(gids, inbox, verts.ids)[verts.property("inbox")[1]],
                          verts.property("inbox")[0][verts.property("inbox")[1]])
    assert result.memory().get("total") == mem.get("total")
    assert result.memory().get("best") == mem.get("best")


def test_components_over_vertex_cuts():
    """TitanPartitionGraphTest's vertex cuts (:380-435): canonical-id folding keeps the
    generic program equal to the oracle's per-row combine."""
    rows, vids, sd, npz = load_fixture("partition_groups")
    o = fr.OracleGraph.from_rows(rows, fr.OracleSchema(sd["edge_types"], [tuple(x) for x in sd["property_keys"]]),
                                 BOTH)
    result, verts, mem = run_both({"rows": rows, "schema": sd}, ConnectedComponents, o)
    ids, (cc, present) = result.vertex_properties["cc"]
    assert np.array_equal(reorder(ids, cc, verts.ids), verts.property("cc")[0])


def test_generic_program_write_back():
    """PERSIST / LOCALTX of a generic program's element compute keys (FulgoraGraphComputer.java:
    248-305): one SINGLE-cardinality entry per vertex holding a value, byte-exact against the
    oracle's EdgeSerializer restatement — a typed Long key and a generic (Object) key, read
    back through the store (PERSIST) or the local transaction (LOCALTX)."""
    rows, vids, sd, npz = load_fixture("gotg")
    cc_key = (7000 << 6) | 5
    graph = GpuGraph(rows, sd, property_keys={"cc": (cc_key, L.DT_LONG)})
    computer = graph.compute()
    computer.resultMode(TitanGraphComputer.ResultMode.PERSIST)
    computer.program(ConnectedComponents())
    res = computer.submit().get()
    ids, (cc, present) = res.vertex_properties["cc"]
    assert res.graph() is graph and present.all()
    for vid, c in zip(ids, cc):
        assert graph.read_property(int(vid), cc_key, L.DT_LONG) == int(c)
    # the device rows equal the oracle's encoder, relation ids base + running index
    eng = Engine().load_rows(rows, Schema.from_dict(sd), BOTH)
    base = 1 << 30
    got = eng.result_rows_values(cc_key, L.DT_LONG, L.VAL_INT64, reorder(ids, cc, eng.vertex_ids()),
                                 np.ones(eng.n, bool), base)
    lib = fr.load()
    want = [fr.encode_property(cc_key, L.DT_LONG, int(c), base + i)
            for i, c in enumerate(reorder(ids, cc, eng.vertex_ids()))]
    for r in range(got.nrows):
        b = bytes(got.data[got.byte_begin[r]:got.byte_begin[r + 1]])
        lv = int(got.limit_valpos[r])
        assert (b, lv & 0x7FFFFFFF) == want[r] and got.keys[r] == lib.fr_key_of(int(eng.vertex_ids()[r]), 5)
    # generic key (no schema): LOCALTX leaves the store alone; fp64 values
    g2 = GpuGraph(rows, sd)
    c2 = g2.compute()
    c2.resultMode(TitanGraphComputer.ResultMode.LOCALTX)
    c2.program(GenericPageRank(0.85, eng.n, 4))
    res = c2.submit().get()
    key, dt = g2.property_key("pr")
    assert dt == L.DT_OBJECT
    ids, (pr, _) = res.vertex_properties["pr"]
    assert g2.read_property(int(ids[0]), key, L.DT_OBJECT) is None
    assert [res.graph().read_property(int(v), key, L.DT_OBJECT) for v in ids] == [float(x) for x in pr]
    got = eng.result_rows_values(key, L.DT_OBJECT, L.VAL_FP64, np.full(eng.n, 0.25), np.arange(eng.n) % 2 == 0, 9)
    assert got.nrows == (eng.n + 1) // 2
    assert bytes(got.data[:got.byte_begin[1]]) == fr.encode_property_generic(key, L.DT_DOUBLE, 0.25, 9)[0]
    with pytest.raises(TitanException):                     # an Integer key holds int values only
        eng.result_rows_values(cc_key, L.DT_INTEGER, L.VAL_INT64, np.full(eng.n, 1 << 40), np.ones(eng.n, bool), 9)


def float_weight_rows():
    """A weighted power-law graph whose weight is a Float property (values -3..250)."""
    import edgestore as es
    scale = 9
    n = 1 << scale
    src, dst, w = rmat_edges(scale, 8, seed=91, weights=True)
    knows = es.user_edge_label(1)
    fkey = es.user_property_key(3)
    sd = {"edge_types": [{"type_id": knows, "multiplicity": 0}], "property_keys": [[fkey, 5]]}
    osch = fr.OracleSchema(sd["edge_types"], [(fkey, 5)])
    spec = es.GraphSpec(n=n, edges=[(int(a), int(b), knows, [(fkey, int(x) - 4)]) for a, b, x in zip(src, dst, w)])
    rows, vids = es.build_rows(spec, osch)
    return rows, vids, sd, osch, fkey, n


@pytest.mark.parametrize("host_decode", [False, True])
def test_float_weights_in_generic_edge_functions(host_decode, monkeypatch):
    """A Float weight (FloatSerializer bits): generic fp64 edge functions read it widened to
    double, int64 messages are refused, and ShortestDistance (edge.<Integer>value) fails as
    its ClassCastException does — through the device and the host decoder (the host decoder
    once left the column typed Integer)."""
    if host_decode:
        monkeypatch.setenv("TGO_HOST_DECODE", "1")
    rows, vids, sd, osch, fkey, n = float_weight_rows()
    eng = Engine().load_rows(rows, Schema.from_dict(sd), IN, weight_key=fkey)
    o = fr.OracleGraph.from_rows(rows, osch, IN, weight_key=fkey)
    rng = np.random.default_rng(2)
    msg = rng.standard_normal(eng.n)
    has = rng.random(eng.n) < 0.8
    for fn in (L.EDGE_ADD_WEIGHT, L.EDGE_MUL_WEIGHT, L.EDGE_SUB_WEIGHT, L.EDGE_MIN_WEIGHT, L.EDGE_MAX_WEIGHT,
               L.EDGE_DIV_WEIGHT):
        got, gh = eng.gather(IN, L.VAL_FP64, L.COMBINE_MAX, fn, msg, has)
        exp, eh = o.gather(IN, 1, 2, fn, msg, has)
        assert np.array_equal(gh, eh) and np.array_equal(got[gh], exp[eh]), fn
    with pytest.raises(TitanException) as e:
        eng.gather(IN, L.VAL_INT64, L.COMBINE_SUM, L.EDGE_ADD_WEIGHT, np.zeros(eng.n, np.int64))
    assert e.value.code == L.TGO_E_INVALID
    with pytest.raises(TitanException) as e:
        eng.sssp(int(vids[0]), 5, IN)
    assert e.value.code == L.TGO_E_UNSUPPORTED
    with pytest.raises(RuntimeError):
        o.shortest_distance(int(vids[0]), 5, IN, weighted=True)


def wide_weight_rows(dt, where, order="ASC"):
    """A power-law graph whose weight is a Long (4) or Double (6) property, in the remaining
    properties or a MULTI label's sort key (ASC / DESC), with values past 32 bits (Long: about
    +-4e11; Double: integral values up to 2^41, not representable as a Float)."""
    import edgestore as es
    scale = 9
    n = 1 << scale
    src, dst, w = rmat_edges(scale, 8, seed=93, weights=True)
    knows = es.user_edge_label(1)
    key = es.user_property_key(3)
    et = {"type_id": knows, "multiplicity": 0}
    if where == "sort_key":
        et.update({"sort_key": [key], "order": order})
    sd = {"edge_types": [et], "property_keys": [[key, dt]]}
    osch = fr.OracleSchema(sd["edge_types"], [(key, dt)])
    vals = (w.astype(np.int64) - 100) * 3_000_000_007 + 11
    spec = es.GraphSpec(n=n, edges=[(int(a), int(b), knows, [(key, int(x))]) for a, b, x in zip(src, dst, vals)])
    rows, vids = es.build_rows(spec, osch)
    return rows, vids, sd, osch, key


@pytest.mark.parametrize("dt", [4, 6])
@pytest.mark.parametrize("where,order", [("remaining", "ASC"), ("sort_key", "ASC"), ("sort_key", "DESC")])
@pytest.mark.parametrize("host_decode", [False, True])
def test_long_double_weights_in_generic_edge_functions(dt, where, order, host_decode, monkeypatch):
    """Long and Double weight keys (row loads; the weight column holds each
    entry's staged position into a 64-bit value table).  fp64 messages with every weight edge
    function and int64 messages with a Long weight (Java long arithmetic) equal the oracle's
    gathers (exact combiners) and streams; a Double weight refuses int64 messages, and
    ShortestDistance (edge.<Integer>value) fails as its ClassCastException does — through the
    device decoder and the host decoder (TGO_HOST_DECODE=1) alike."""
    if host_decode:
        monkeypatch.setenv("TGO_HOST_DECODE", "1")
    rows, vids, sd, osch, key = wide_weight_rows(dt, where, order)
    eng = Engine().load_rows(rows, Schema.from_dict(sd), IN, weight_key=key)
    o = fr.OracleGraph.from_rows(rows, osch, IN, weight_key=key)
    ids = o.vertex_ids()
    assert np.array_equal(np.sort(eng.vertex_ids()), np.sort(ids))
    rng = np.random.default_rng(5)
    msg = rng.standard_normal(eng.n) * 1e3
    has = rng.random(eng.n) < 0.8
    fns = (L.EDGE_ADD_WEIGHT, L.EDGE_MUL_WEIGHT, L.EDGE_SUB_WEIGHT, L.EDGE_MIN_WEIGHT, L.EDGE_MAX_WEIGHT,
           L.EDGE_DIV_WEIGHT)
    for fn in fns:
        for comb in (L.COMBINE_MIN, L.COMBINE_MAX):
            got, gh = eng.gather(IN, L.VAL_FP64, comb, fn, reorder(ids, msg, eng.vertex_ids()),
                                 reorder(ids, has, eng.vertex_ids()))
            exp, eh = o.gather(IN, 1, comb, fn, msg, has)
            got, gh = reorder(eng.vertex_ids(), got, ids), reorder(eng.vertex_ids(), gh, ids)
            assert np.array_equal(gh, eh) and np.array_equal(got[gh], exp[eh]), (fn, comb)
    off, vals = eng.gather_lists(IN, L.VAL_FP64, L.EDGE_ADD_WEIGHT, reorder(ids, msg, eng.vertex_ids()),
                                 reorder(ids, has, eng.vertex_ids()))
    ooff, ovals = o.gather_lists(IN, 1, L.EDGE_ADD_WEIGHT, msg, has)
    assert off[-1] == ooff[-1] and np.array_equal(np.sort(vals), np.sort(ovals))
    imsg = rng.integers(-(1 << 40), 1 << 40, eng.n)
    if dt == 4:
        for fn in fns[:-1]:
            for comb in (L.COMBINE_SUM, L.COMBINE_MIN):
                got, gh = eng.gather(IN, L.VAL_INT64, comb, fn, reorder(ids, imsg, eng.vertex_ids()),
                                     reorder(ids, has, eng.vertex_ids()))
                exp, eh = o.gather(IN, 0, comb, fn, imsg, has)
                got, gh = reorder(eng.vertex_ids(), got, ids), reorder(eng.vertex_ids(), gh, ids)
                assert np.array_equal(gh, eh) and np.array_equal(got[gh], exp[eh]), (fn, comb)
    else:
        with pytest.raises(TitanException) as e:
            eng.gather(IN, L.VAL_INT64, L.COMBINE_SUM, L.EDGE_ADD_WEIGHT, np.zeros(eng.n, np.int64))
        assert e.value.code == L.TGO_E_INVALID
    with pytest.raises(TitanException) as e:
        eng.sssp(int(vids[0]), 5, IN)
    assert e.value.code == L.TGO_E_UNSUPPORTED


def test_integer_division_by_zero_fails_the_program():
    n = 64
    src, dst, w = np.array([0, 1, 2], np.int32), np.array([1, 2, 3], np.int32), np.array([3, 0, 5], np.int32)
    eng = Engine().load_edges(n, src, dst, IN, weight=w)
    with pytest.raises(TitanException) as e:
        eng.gather(IN, L.VAL_INT64, L.COMBINE_SUM, L.EDGE_DIV_WEIGHT, np.ones(n, np.int64))
    assert e.value.code == L.TGO_E_PROGRAM
    out, has = eng.gather(IN, L.VAL_FP64, L.COMBINE_SUM, L.EDGE_DIV_WEIGHT, np.ones(n))
    assert has[1] and np.isinf(out[1]) and out[0] == 1.0 / 3


@pytest.mark.parametrize("column_order", [False, True])
@pytest.mark.parametrize("load_scope,scope", [(IN, IN), (OUT, OUT), (BOTH, BOTH), (BOTH, IN)])
def test_gather_lists_match_oracle_streams(weighted_rmat, load_scope, scope, column_order):
    """Combiner-less receive (tgo_gather_lists) over an edge list: every vertex's stream equal
    to the oracle's (fr_gather_lists), element by element.  For an edge list the (direction,
    neighbour) order IS the column order, so both loads must match."""
    n, src, dst, w = weighted_rmat
    eng = Engine().load_edges(n, src, dst, load_scope, weight=w, apply_cap=False, column_order=column_order)
    o = fr.OracleGraph.from_edges(n, src, dst, w)
    rng = np.random.default_rng(17)
    for vt, fn in ((L.VAL_INT64, L.EDGE_IDENTITY), (L.VAL_INT64, L.EDGE_SUB_WEIGHT), (L.VAL_FP64, L.EDGE_MUL_WEIGHT)):
        msg = rng.integers(-(1 << 40), 1 << 40, n) if vt == L.VAL_INT64 else rng.standard_normal(n)
        has = rng.random(n) < 0.6
        off, vals = eng.gather_lists(scope, vt, fn, msg, has)
        ooff, ovals = o.gather_lists(scope, vt, fn, msg, has)
        assert np.array_equal(off, ooff)
        assert np.array_equal(vals, ovals), (vt, fn)


def test_gather_lists_in_column_order_on_edgestore_rows():
    """GraphOfTheGods rows (several labels: the column order interleaves labels and
    directions): with TGO_LOAD_COLUMN_ORDER every stream is in the reference's order."""
    rows, vids, sd, npz = load_fixture("gotg")
    osch = fr.OracleSchema(sd["edge_types"], [tuple(x) for x in sd["property_keys"]])
    o = fr.OracleGraph.from_rows(rows, osch, BOTH)
    eng = Engine().load_rows(rows, Schema.from_dict(sd), BOTH, column_order=True)
    assert np.array_equal(eng.vertex_ids(), o.vertex_ids())
    msg = np.arange(eng.n, dtype=np.int64) * 10
    for scope in (IN, OUT, BOTH):
        off, vals = eng.gather_lists(scope, L.VAL_INT64, L.EDGE_ADD_ONE, msg, np.ones(eng.n, bool))
        ooff, ovals = o.gather_lists(scope, 0, 1, msg, np.ones(eng.n, bool))
        assert np.array_equal(off, ooff) and np.array_equal(vals, ovals), scope


def test_combiner_less_programs(weighted_rmat):
    n, src, dst, w = weighted_rmat
    o = fr.OracleGraph.from_edges(n, src, dst, w)
    result, verts, mem = run_both({"edges": (n, src, dst, w)}, FirstLastCount, o, weight_keys={"w": 1})
    for key in ("first", "last", "count"):
        ids, (vals, present) = result.vertex_properties[key]
        assert np.array_equal(reorder(ids, present, verts.ids), verts.property(key)[1]), key
        ok = verts.property(key)[1]
        assert np.array_equal(reorder(ids, vals, verts.ids)[ok], verts.property(key)[0][ok]), key
    ids = o.vertex_ids()
    result, verts, mem = run_both({"edges": (n, src, dst, None)}, lambda: GlobalNoCombiner(ids, True), o)
    gids, (inbox, has) = result.vertex_properties["inbox"]
    assert has.all() and np.array_equal(reorder(gids, inbox, verts.ids), verts.property("inbox")[0])
    graph = GpuGraph(edges=(n, src, dst, None))
    c = graph.compute()
    c.program(GlobalNoCombiner(ids, False))
    with pytest.raises(ExecutionException):
        c.submit().get()


def test_generic_program_failure_surfaces_as_execution_exception():
    rows, vids, sd, npz = load_fixture("gotg")
    graph = GpuGraph(rows, sd)
    computer = graph.compute()
    computer.weight_keys = {"w": sd["property_keys"][0][0]}
    computer.program(GlobalDegreeSum(np.array(vids[:2])))      # add_weight over edges without `time`
    with pytest.raises(ExecutionException):
        computer.submit().get()

"""GPU parity: the HIP engine (through the C-ABI) against the reference's known answers and
against the CPU oracle on identical inputs.

Bars (BASELINE.json north_star): BFS levels, reachability and integer distances bit-exact;
PageRank within 1e-6 L1.
"""
import numpy as np
import pytest

import fulgora as fr
from conftest import load_fixture
from titan_amd import (DegreeCounter, DegreeMapper, Engine, ExecutionException, GpuGraph, PageRankMapReduce,
                       PageRankVertexProgram, Schema, ShortestDistanceMapReduce, ShortestDistanceVertexProgram,
                       TitanException, TitanGraphComputer, pick_roots, rmat_edges)
from titan_amd import _lib as L

pytestmark = pytest.mark.gpu

OUT, IN, BOTH = L.SCOPE_OUT_E, L.SCOPE_IN_E, L.SCOPE_BOTH_E
ABSENT = L.DIST_ABSENT
PR_L1_TOL = 1e-6      # north_star: PageRank within 1e-6 L1


def engine_from_fixture(name, scope, weight_key=0, hard_limit=100000, batch_rows=None):
    rows, vids, sd, npz = load_fixture(name)
    eng = Engine(hard_query_limit=hard_limit).load_rows(rows, Schema.from_dict(sd), scope, weight_key=weight_key,
                                                       batch_rows=batch_rows)
    return eng, rows, vids, sd, npz


def oracle_from_fixture(name, scope, weight_key=0, hard_limit=100000):
    rows, vids, sd, npz = load_fixture(name)
    return fr.OracleGraph.from_rows(rows, fr.OracleSchema(sd["edge_types"], [tuple(x) for x in sd["property_keys"]]),
                                    scope, weight_key=weight_key, hard_limit=hard_limit)


def reorder(ids_from, values, ids_to):
    pos = {int(v): i for i, v in enumerate(ids_from)}
    return np.array([values[pos[int(v)]] for v in ids_to])


# ----------------------------------------------------------------------------- GraphOfTheGods
@pytest.mark.parametrize("scope,seed_name,key", [(IN, "saturn", "bfs_in_saturn"), (OUT, "jupiter", "bfs_out_jupiter"),
                                                 (BOTH, "jupiter", "bfs_both_jupiter")])
@pytest.mark.parametrize("batch", [None, 3])
def test_gotg_bfs(scope, seed_name, key, batch):
    eng, rows, vids, sd, npz = engine_from_fixture("gotg", scope, batch_rows=batch)
    names = list(npz["names"])
    d = eng.bfs(int(vids[names.index(seed_name)]), 12, scope)
    d = reorder(eng.vertex_ids(), d, vids)
    assert np.array_equal(np.where(d == ABSENT, -1, d), npz[key])
    st = eng.stats()
    assert st["num_vertices"] == 12 and st["ghost_vertices"] == 1 and st["skipped_rows"] == 1


def test_gotg_degree_counter_through_computer():
    rows, vids, sd, npz = load_fixture("gotg")
    graph = GpuGraph(rows, sd)
    computer = graph.compute()
    computer.resultMode(TitanGraphComputer.ResultMode.NONE)
    computer.workers(4)
    computer.program(DegreeCounter(1))
    computer.mapReduce(DegreeMapper())
    result = computer.submit().get()
    degrees = result.memory().get(DegreeMapper.DEGREE_RESULT)
    assert len(degrees) == 12
    assert [degrees[int(v)] for v in vids] == list(npz["degree1"])
    assert result.memory().getIteration() == 1


# ----------------------------------------------------------------------------- OLAPTest
def test_pagerank_tree():
    rows, vids, sd, npz = load_fixture("pagerank_tree")
    graph = GpuGraph(rows, sd)
    computer = graph.compute()
    computer.workers(4)
    numV = int(npz["num_v"])
    computer.program(PageRankVertexProgram.build().iterations(10).vertexCount(numV).dampingFactor(0.85).create(graph))
    computer.mapReduce(PageRankMapReduce.build().create())
    result = computer.submit().get()
    ranks = list(result.memory().get(PageRankMapReduce.DEFAULT_MEMORY_KEY))
    assert len(ranks) == numV
    got = dict((kv.getKey(), kv.getValue()) for kv in ranks)
    pr = np.array([got[int(v)] for v in vids])
    exp = npz["expected_pr"]
    assert abs(pr.sum() - exp.sum()) < 0.001                  # OLAPTest.java:561
    np.testing.assert_allclose(pr, exp, rtol=1e-12)           # closed form per vertex
    o = oracle_from_fixture("pagerank_tree", IN)
    opr, _ = o.pagerank(0.85, numV, 10)
    opr = reorder(o.vertex_ids(), opr, vids)
    assert np.abs(pr - opr).sum() <= PR_L1_TOL


def test_sssp_tree_weighted():
    rows, vids, sd, npz = load_fixture("sssp_tree")
    wk = int(npz["weight_key"])
    graph = GpuGraph(rows, sd)
    computer = graph.compute()
    computer.weight_keys = {"distance": wk}
    seed = int(vids[int(npz["seed_index"])])
    computer.program(ShortestDistanceVertexProgram.build().seed(seed).maxDepth(int(npz["max_depth"])).create(graph))
    computer.mapReduce(ShortestDistanceMapReduce.build().create())
    result = computer.submit().get()
    dist = {kv.getKey(): kv.getValue() for kv in result.memory().get(ShortestDistanceMapReduce.DEFAULT_MEMORY_KEY)}
    assert len(dist) == len(vids)                              # OLAPTest.java:605
    assert [dist[int(v)] for v in vids] == list(npz["expected_dist"])


@pytest.mark.parametrize("depth", [0, 1, 3, 7])
def test_sssp_tree_hop_bound_matches_oracle(depth):
    rows, vids, sd, npz = load_fixture("sssp_tree")
    wk = int(npz["weight_key"])
    eng = Engine().load_rows(rows, Schema.from_dict(sd), IN, weight_key=wk)
    seed = int(vids[0])
    d = eng.sssp(seed, depth, IN)
    o = oracle_from_fixture("sssp_tree", IN, weight_key=wk)
    od, it = o.shortest_distance(seed, depth, IN, weighted=True)
    assert np.array_equal(d, reorder(o.vertex_ids(), od, eng.vertex_ids()))


@pytest.mark.parametrize("name,length,key", [("degree_random", 1, "degree1"), ("degree_random100", 2, "degree2")])
def test_degree_counter(name, length, key):
    eng, rows, vids, sd, npz = engine_from_fixture(name, IN)
    d = reorder(eng.vertex_ids(), eng.walkcount(length), vids)
    assert np.array_equal(d, npz[key])


def test_exception_propagates_to_caller():
    # OLAPTest.vertexProgramExceptionPropagatesToCaller: failure => ExecutionException from get()
    rows, vids, sd, npz = load_fixture("gotg")
    graph = GpuGraph(rows, sd)
    computer = graph.compute()
    computer.weight_keys = {"time": sd["property_keys"][0][0]}
    jupiter = int(vids[list(npz["names"]).index("jupiter")])
    # `time` exists only on `battled` edges: traversing any other edge reads a missing key
    computer.program(ShortestDistanceVertexProgram.build().seed(jupiter).maxDepth(5).weightProperty("time")
                     .scope("bothE").create(graph))
    with pytest.raises(ExecutionException):
        computer.submit().get()


# ----------------------------------------------------------------------------- RMAT vs oracle
def numpy_adjacency(n, src, dst, w=None):
    """Reference-independent dense adjacency: per row OUT entries then IN entries, each
    sorted by (neighbour, edge index) — the column order of a MULTI label."""
    m = len(src)
    eidx = np.arange(m)
    o_ord = np.lexsort((eidx, dst, src))
    i_ord = np.lexsort((eidx, src, dst))
    outdeg = np.bincount(src, minlength=n)
    indeg = np.bincount(dst, minlength=n)
    off = np.zeros(n + 1, np.int64)
    off[1:] = np.cumsum(outdeg + indeg)
    mid = off[:-1] + outdeg
    adj = np.empty(2 * m, np.int32)
    ww = np.empty(2 * m, np.int32) if w is not None else None
    o_start = np.zeros(n + 1, np.int64); o_start[1:] = np.cumsum(outdeg)
    i_start = np.zeros(n + 1, np.int64); i_start[1:] = np.cumsum(indeg)
    so, si = src[o_ord], dst[i_ord]
    pos_o = off[so] + (np.arange(m) - o_start[so])
    pos_i = mid[si] + (np.arange(m) - i_start[si])
    adj[pos_o] = dst[o_ord]
    adj[pos_i] = src[i_ord]
    if w is not None:
        ww[pos_o] = w[o_ord]
        ww[pos_i] = w[i_ord]
    return off, mid, adj, ww


@pytest.fixture(scope="module")
def rmat12():
    scale = 12
    src, dst, w = rmat_edges(scale, 16, seed=0x54495441, weights=True)
    n = 1 << scale
    ids = (np.arange(n, dtype=np.int64) + 1) << 3
    off, mid, adj, ww = numpy_adjacency(n, src, dst, w)
    oracle = fr.OracleGraph.from_adjacency(ids, off, mid, adj, ww)
    roots = pick_roots(n, src, dst, 6, seed=7)
    return n, src, dst, w, ids, oracle, roots


@pytest.mark.parametrize("scope", [BOTH, IN, OUT])
def test_rmat_bfs_bit_exact(rmat12, scope):
    n, src, dst, w, ids, oracle, roots = rmat12
    eng = Engine().load_edges(n, src, dst, scope)
    for r in roots:
        d = eng.bfs(int(r), n, scope, seed_is_dense=True, stats=True)
        od, _ = oracle.shortest_distance(int(ids[r]), n, scope)
        assert np.array_equal(d, od)
        st = eng.stats()
        assert st["reached"] == int((od != ABSENT).sum())
    # k-hop bound
    d = eng.bfs(int(roots[0]), 2, scope, seed_is_dense=True)
    od, _ = oracle.shortest_distance(int(ids[roots[0]]), 2, scope)
    assert np.array_equal(d, od)


@pytest.mark.parametrize("scope", [BOTH, IN, OUT])
@pytest.mark.parametrize("nseeds", [1, 5, 64])
def test_rmat_multi_source_bfs_bit_exact(rmat12, scope, nseeds):
    """64 ShortestDistance programs at once: every seed's result equals its own run."""
    n, src, dst, w, ids, oracle, roots = rmat12
    eng = Engine().load_edges(n, src, dst, scope)
    seeds = pick_roots(n, src, dst, nseeds, seed=13)
    d = eng.bfs_multi(seeds, n, scope, seed_is_dense=True, stats=True)
    r, e = eng.multi_stats(nseeds)
    for i, s in enumerate(seeds):
        od, _ = oracle.shortest_distance(int(ids[s]), n, scope)
        assert np.array_equal(d[i], od), i
        assert r[i] == int((od != ABSENT).sum())
    # hop bound applies to every source
    d2 = eng.bfs_multi(seeds[:3], 2, scope, seed_is_dense=True)
    for i, s in enumerate(seeds[:3]):
        assert np.array_equal(d2[i], oracle.shortest_distance(int(ids[s]), 2, scope)[0])


@pytest.mark.parametrize("split", [0.0, -1.0, 0.3, 1.0])
def test_multi_source_split_budget_is_policy_only(rmat12, split):
    """the source split's push budget (tgo_set_tuning TGO_TUNE_MS_SPLIT; 0 = pull
    every source, -1 = the default 0.5 %, 0.3 / 1.0 = most or all sources pushed at the first
    pull level) changes the traversal plan, never a level: every seed equals the oracle."""
    n, src, dst, w, ids, oracle, roots = rmat12
    eng = Engine().load_edges(n, src, dst, BOTH).set_tuning(L.TUNE_MS_SPLIT, split)
    seeds = pick_roots(n, src, dst, 64, seed=17)
    d = eng.bfs_multi(seeds, n, BOTH, seed_is_dense=True, stats=True)
    r, _ = eng.multi_stats(64)
    for i, s in enumerate(seeds):
        od, _ = oracle.shortest_distance(int(ids[s]), n, BOTH)
        assert np.array_equal(d[i], od), (split, i)
        assert r[i] == int((od != ABSENT).sum())
    with pytest.raises(TitanException):
        eng.set_tuning(L.TUNE_MS_SPLIT, 1.5)
    with pytest.raises(TitanException):
        eng.set_tuning(99, 0.0)


_MS_SWEEPS = """
import hashlib
from titan_amd import Engine, pick_roots, rmat_edges
from titan_amd import _lib as L
n = 1 << 14
src, dst, _ = rmat_edges(14, 16, seed=5)
h = hashlib.sha256()
for scope in (L.SCOPE_BOTH_E, L.SCOPE_IN_E, L.SCOPE_OUT_E):
    eng = Engine().load_edges(n, src, dst, scope, apply_cap=False)
    for split in (-1.0, 0.3, 1.0):
        eng.set_tuning(L.TUNE_MS_SPLIT, split)
        for seed in (3, 4):
            d = eng.bfs_multi(pick_roots(n, src, dst, 64, seed=seed), n, scope, seed_is_dense=True)
            h.update(d.tobytes())
print(h.hexdigest())
"""


def _ms_sweeps(**env):
    import os
    import subprocess
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    p = subprocess.run([sys.executable, "-c", _MS_SWEEPS], cwd=root, env=dict(os.environ, TGO_TRACE="1", **env),
                       capture_output=True, text=True, timeout=240)
    assert p.returncode == 0, p.stderr[-2000:]
    return p.stdout.strip().splitlines()[-1], p.stderr


def test_multi_source_settle_sums_and_ranged_push():
    """Two sweep-plan paths the parity tests alone would not pin, in fresh processes (their
    switches are read once per process): (1) the source split after a push level reads the
    per-source push entries that level's settle summed (bit-sliced over the fresh masks);
    TGO_MS_SRCENT_CHECK=1 recomputes them with ms_source_entries at every such split and fails the
    sweep on any difference; (2) the target-ranged push (TGO_MS_PUSH_RANGE = log2 of the range,
    here 256-vertex ranges for every push level) gives the same levels as the queue-order push."""
    plain, _ = _ms_sweeps(TGO_MS_PUSH_RANGE="0")
    checked, err = _ms_sweeps(TGO_MS_PUSH_RANGE="0", TGO_MS_SRCENT_CHECK="1")
    assert "settle per-source entries checked" in err
    ranged, _ = _ms_sweeps(TGO_MS_PUSH_RANGE="8", TGO_MS_PUSH_RANGE_MIN="1", TGO_MS_SRCENT_CHECK="1")
    assert plain == checked == ranged


@pytest.mark.parametrize("env", [{"TGO_MS_LONG": "4"}, {"TGO_MS_LONG": "2"}, {"TGO_MS_LONG": "8"},
                                 {"TGO_MS_RAMP": "1"}, {"TGO_MS_STEP": "4"}, {"TGO_MS_STEP": "16", "TGO_MS_LONG": "4"},
                                 {"TGO_MS_COOP": "8"}, {"TGO_MS_COOP": "1000"}, {"TGO_MS_PUSH_PROBE": "0"},
                                 {"TGO_MS_PUSH_LIGHT": "0"}])
def test_multi_source_pull_shapes_give_the_same_levels(env):
    """The pull's walk shapes (long-list trip 64 / 128 / 256 / 512 entries, a 64-entry first trip,
    4 / 8 / 16 entries per short-list round trip, the wave-cooperative threshold) and the push's
    probe / reached-mask read only change how much is read before a walk stops: every sweep
    equals the default's, level for level (fresh processes: the switches are read once)."""
    if "base" not in _MS_BASE:
        _MS_BASE["base"] = _ms_sweeps()[0]
    other, _ = _ms_sweeps(**env)
    assert other == _MS_BASE["base"], env


_MS_BASE = {}


@pytest.mark.parametrize("scope", [BOTH, IN, OUT])
@pytest.mark.parametrize("cold,split", [(0, -1.0), (1, -1.0), (300, -1.0), (300, 0.0), (1000, 0.3), (64, 1.0)])
def test_multi_source_cold_split_level(rmat12, scope, cold, split):
    """The first pull level split at a hot head (TGO_TUNE_MS_COLD: hot walk + blocked cold pass +
    finish; values > 1 set the head and segment size so RMAT-12 has cold entries) with the source
    split on / off / forced: every seed equals the oracle and the plain sweep."""
    n, src, dst, w, ids, oracle, roots = rmat12
    eng = Engine().load_edges(n, src, dst, scope).set_tuning(L.TUNE_MS_SPLIT, split)
    seeds = pick_roots(n, src, dst, 64, seed=23)
    plain = eng.set_tuning(L.TUNE_MS_COLD, 0).bfs_multi(seeds, n, scope, seed_is_dense=True)
    d = eng.set_tuning(L.TUNE_MS_COLD, cold).bfs_multi(seeds, n, scope, seed_is_dense=True, stats=True)
    r, _ = eng.multi_stats(64)
    assert np.array_equal(d, plain)
    for i, s in enumerate(seeds):
        od, _ = oracle.shortest_distance(int(ids[s]), n, scope)
        assert np.array_equal(d[i], od), (cold, i)
        assert r[i] == int((od != ABSENT).sum())
    # the layout is rebuilt for another head and reused; a repeated sweep is identical
    assert np.array_equal(eng.bfs_multi(seeds, n, scope, seed_is_dense=True), d)
    with pytest.raises(TitanException):
        eng.set_tuning(L.TUNE_MS_COLD, 2.5)


def test_multi_source_duplicate_and_gotg_seeds():
    eng, rows, vids, sd, npz = engine_from_fixture("gotg", BOTH)
    names = list(npz["names"])
    seeds = [int(vids[names.index("jupiter")]), int(vids[names.index("saturn")]), int(vids[names.index("jupiter")])]
    d = eng.bfs_multi(seeds, 12, BOTH)
    single = eng.bfs(seeds[0], 12, BOTH)
    assert np.array_equal(d[0], single) and np.array_equal(d[2], single)
    assert np.array_equal(d[1], eng.bfs(seeds[1], 12, BOTH))


def test_rmat_bfs_deterministic(rmat12):
    n, src, dst, w, ids, oracle, roots = rmat12
    eng = Engine().load_edges(n, src, dst, BOTH)
    a = eng.bfs(int(roots[1]), n, BOTH, seed_is_dense=True)
    b = eng.bfs(int(roots[1]), n, BOTH, seed_is_dense=True)
    assert np.array_equal(a, b)


@pytest.mark.parametrize("depth", [2, 5, 64])
def test_rmat_sssp_weighted_bit_exact(rmat12, depth):
    n, src, dst, w, ids, oracle, roots = rmat12
    eng = Engine().load_edges(n, src, dst, IN, weight=w)
    for r in roots[:3]:
        d = eng.sssp(int(r), depth, IN, seed_is_dense=True)
        od, _ = oracle.shortest_distance(int(ids[r]), depth, IN, weighted=True)
        assert np.array_equal(d, od)


@pytest.mark.parametrize("scope", [OUT, IN, BOTH])
@pytest.mark.parametrize("delta", [0, 1, 37, 1 << 40])
def test_rmat_sssp_delta_equals_converged(rmat12, scope, delta):
    """Delta-stepping (any bucket width, incl. one bucket = Bellman-Ford and width 1 =
    Dijkstra-like) gives the converged distances of the reference program bit-exactly."""
    n, src, dst, w, ids, oracle, roots = rmat12
    eng = Engine().load_edges(n, src, dst, scope, weight=w)
    for r in roots[:3]:
        d = eng.sssp(int(r), n, scope, mode=L.SSSP_DELTA, seed_is_dense=True, stats=True, delta=delta)
        od, _ = oracle.shortest_distance(int(ids[r]), n, scope, weighted=True)
        assert np.array_equal(d, od)
        st = eng.stats()
        assert st["reached"] == int((od != ABSENT).sum())
        assert (st["relaxed_entries"] > 0) == (st["reached"] > 1)   # a seed with no push entries reaches nobody


@pytest.mark.parametrize("scope", [OUT, IN])
@pytest.mark.parametrize("delta", [0, 9, 37, 200])
@pytest.mark.parametrize("bins,cap,done,pull", [(1, 0, 0, 0), (1, 0, 1, 0), (1, 16, 1, 0), (1, 1024, 0, 0), (0, 0, 0, 0),
                                                (1, 0, 0, 0.001), (1, 16, 1, 0.001), (1, 0, 1, 0.02)])
def test_rmat_sssp_delta_piles(rmat12, scope, delta, bins, cap, done, pull):
    """The binned loop (next bucket extracted from its pile of improved vertices; with and
    without the done-target filter; finished buckets' heavy entries pushed or pulled), the same
    loop with piles so small that buckets overflow into the bitmap scan, and the bitmap-scan
    loop all give the oracle's converged distances bit for bit."""
    n, src, dst, w, ids, oracle, roots = rmat12
    eng = Engine().load_edges(n, src, dst, scope, weight=w)
    eng.set_tuning(L.TUNE_DS_BINS, bins).set_tuning(L.TUNE_DS_PILE_CAP, cap).set_tuning(L.TUNE_DS_DONE, done)
    eng.set_tuning(L.TUNE_DS_PULL, pull)
    for r in roots[:3]:
        d = eng.sssp(int(r), n, scope, mode=L.SSSP_DELTA, seed_is_dense=True, stats=True, delta=delta)
        od, _ = oracle.shortest_distance(int(ids[r]), n, scope, weighted=True)
        assert np.array_equal(d, od)
        assert eng.stats()["reached"] == int((od != ABSENT).sum())


@pytest.mark.parametrize("scope", [OUT, IN])
@pytest.mark.parametrize("delta", [0, 9, 200])
@pytest.mark.parametrize("cap", [0, 16])
def test_rmat_sssp_delta_small_steps(rmat12, scope, delta, cap):
    """The binned loop with its tiny steps run in one block (TGO_TUNE_DS_SMALL, delta_loop.hip
    ds_small_steps, queue buffer on the device) and the grid kernels taking over at the first
    step that is not small — RMAT-12's steps are mostly small; cap 16 overflows piles into the
    bitmap scan, which always goes to the grid — gives the oracle's distances bit for bit."""
    n, src, dst, w, ids, oracle, roots = rmat12
    eng = Engine().load_edges(n, src, dst, scope, weight=w)
    eng.set_tuning(L.TUNE_DS_BINS, 1).set_tuning(L.TUNE_DS_PILE_CAP, cap).set_tuning(L.TUNE_DS_SMALL, 1)
    for r in roots[:3]:
        d = eng.sssp(int(r), n, scope, mode=L.SSSP_DELTA, seed_is_dense=True, stats=True, delta=delta)
        od, _ = oracle.shortest_distance(int(ids[r]), n, scope, weighted=True)
        assert np.array_equal(d, od)
        assert eng.stats()["reached"] == int((od != ABSENT).sum())


def test_rmat_sssp_delta_zero_weights(rmat12):
    """Zero-weight edges (ties inside a bucket, re-relaxation at equal distance)."""
    n, src, dst, w, ids, _, roots = rmat12
    w0 = (w % 3).astype(np.int32)
    off, mid, adj, ww = numpy_adjacency(n, src, dst, w0)
    oracle = fr.OracleGraph.from_adjacency(ids, off, mid, adj, ww)
    eng = Engine().load_edges(n, src, dst, OUT, weight=w0)
    for pull in (0, 0.001):
        eng.set_tuning(L.TUNE_DS_PULL, pull)
        for r in roots[:2]:
            d = eng.sssp(int(r), n, OUT, mode=L.SSSP_DELTA, seed_is_dense=True, delta=2)
            assert np.array_equal(d, oracle.shortest_distance(int(ids[r]), n, OUT, weighted=True)[0])


@pytest.mark.parametrize("scope", [OUT, IN])
@pytest.mark.parametrize("done,pull,small", [(0, 0, 0), (1, 0, 0), (0, 0.001, 0), (1, 0.001, 0), (1, 1.0, 0),
                                             (0, 0, 1)])
def test_sssp_delta_bucket_merge(scope, done, pull, small):
    """A bucket merge in the binned loop (delta 10): s -10-> a, s -35-> z, a -10-> y, z -4-> c,
    y -10-> c.  When bucket 1 (a) finishes, pile 2 is empty and pile 3 holds z, so the loop
    jumps to bucket 3 while a's heavy entry puts y (20) into the near queue: buckets 2..3 merge.
    z's light entry gives c 39; y's heavy entry, relaxed at the merged range's finish, must
    still lower c to 30 — with the done filter and the pull form, whose members are final only
    after a single bucket (the merged range once marked c done)."""
    n = 5
    src = np.array([0, 0, 1, 2, 3], np.int64)
    dst = np.array([1, 2, 3, 4, 4], np.int64)
    w = np.array([10, 35, 10, 4, 10], np.int32)
    if scope == IN:                        # an inE scope's messages travel against the edges
        src, dst = dst, src
    ids = (np.arange(n, dtype=np.int64) + 1) << 3
    off, mid, adj, ww = numpy_adjacency(n, src, dst, w)
    oracle = fr.OracleGraph.from_adjacency(ids, off, mid, adj, ww)
    od = oracle.shortest_distance(int(ids[0]), n, scope, weighted=True)[0]
    assert list(od) == [0, 10, 35, 20, 30]
    eng = Engine().load_edges(n, src, dst, scope, weight=w)
    eng.set_tuning(L.TUNE_DS_BINS, 1).set_tuning(L.TUNE_DS_DONE, done).set_tuning(L.TUNE_DS_PULL, pull)
    eng.set_tuning(L.TUNE_DS_SMALL, small)
    d = eng.sssp(0, n, scope, mode=L.SSSP_DELTA, seed_is_dense=True, delta=10)
    assert np.array_equal(d, od), (d, od)


def test_sssp_tree_delta():
    rows, vids, sd, npz = load_fixture("sssp_tree")
    wk = int(npz["weight_key"])
    eng = Engine().load_rows(rows, Schema.from_dict(sd), IN, weight_key=wk)
    seed = int(vids[int(npz["seed_index"])])
    d = reorder(eng.vertex_ids(), eng.sssp(seed, 100, IN, mode=L.SSSP_DELTA), vids)
    assert list(d) == list(npz["expected_dist"])
    # unknown seed: nobody gets a distance
    assert -1 not in set(int(v) for v in vids)
    assert (eng.sssp(-1, 100, IN, mode=L.SSSP_DELTA) == ABSENT).all()


@pytest.mark.parametrize("iters", [0, 1, 2, 5, 20])
def test_rmat_pagerank_l1(rmat12, iters):
    n, src, dst, w, ids, oracle, roots = rmat12
    eng = Engine().load_edges(n, src, dst, IN)
    pr = eng.pagerank(0.85, n, iters)
    opr, it = oracle.pagerank(0.85, n, iters)
    assert it == iters
    if iters == 0:
        assert np.isnan(pr).all() and np.isnan(opr).all()
        return
    assert np.abs(pr - opr).sum() <= PR_L1_TOL
    pr2 = eng.pagerank(0.85, n, iters)
    assert np.array_equal(pr, pr2)                             # fixed reduction order


@pytest.mark.parametrize("k", [1, 2, 3, 6])
def test_rmat_walkcount_exact(rmat12, k):
    n, src, dst, w, ids, oracle, roots = rmat12
    eng = Engine().load_edges(n, src, dst, IN)
    d = eng.walkcount(k)
    od, _ = oracle.degree_counter(k)
    assert np.array_equal(d, od)                               # includes int32 wrap at k=6


def test_rmat_cap_parity(rmat12):
    """QueryContainer hard limit: rows cut in column order; pull lists are no longer
    transposes, so BFS/SSSP push over an explicit transpose."""
    n, src, dst, w, ids, _, roots = rmat12
    limit = 40
    off, mid, adj, ww = numpy_adjacency(n, src, dst, w)
    # apply the cap to the reference-independent rows: keep the first `limit` entries
    keep = np.zeros(len(adj), bool)
    for v in range(n):
        keep[off[v]:min(off[v + 1], off[v] + limit)] = True
    noff = np.zeros(n + 1, np.int64)
    cnt = np.array([keep[off[v]:off[v + 1]].sum() for v in range(n)])
    noff[1:] = np.cumsum(cnt)
    nmid = noff[:-1] + np.minimum(mid - off[:-1], cnt)
    oracle = fr.OracleGraph.from_adjacency(ids, noff, nmid, adj[keep], ww[keep])
    eng = Engine(hard_query_limit=limit).load_edges(n, src, dst, IN, weight=w)
    assert eng.stats()["truncated_results"] == int(((off[1:] - off[:-1]) >= limit).sum())
    pr = eng.pagerank(0.85, n, 10)
    opr, _ = oracle.pagerank(0.85, n, 10)
    fin = np.isfinite(opr)
    assert np.array_equal(np.isfinite(pr), fin)
    assert np.abs(pr[fin] - opr[fin]).sum() <= PR_L1_TOL
    assert np.array_equal(eng.walkcount(3), oracle.degree_counter(3)[0])
    for r in roots[:3]:
        assert np.array_equal(eng.bfs(int(r), n, IN, seed_is_dense=True), oracle.shortest_distance(int(ids[r]), n, IN)[0])
        assert np.array_equal(eng.sssp(int(r), 6, IN, seed_is_dense=True),
                              oracle.shortest_distance(int(ids[r]), 6, IN, weighted=True)[0])


def test_rmat_rows_path_matches_oracle():
    """Full path: byte-exact edgestore rows -> device decode -> traversal."""
    import edgestore as es
    scale = 9
    src, dst, _ = rmat_edges(scale, 8, seed=99)
    n = 1 << scale
    knows = es.user_edge_label(1)
    sd = {"edge_types": [{"type_id": knows, "multiplicity": 0}], "property_keys": []}
    osch = fr.OracleSchema(sd["edge_types"], [])
    spec = es.GraphSpec(n=n, edges=[(int(a), int(b), knows, []) for a, b in zip(src, dst)])
    rows, vids = es.build_rows(spec, osch)
    for scope in (BOTH, IN):
        o = fr.OracleGraph.from_rows(rows, osch, scope, hard_limit=30)
        eng = Engine(hard_query_limit=30).load_rows(rows, Schema.from_dict(sd), scope, batch_rows=100)
        assert np.array_equal(eng.vertex_ids(), o.vertex_ids())
        assert eng.stats()["truncated_results"] == o.stats.truncated_results
        for r in vids[:4]:
            assert np.array_equal(eng.bfs(int(r), n, scope), o.shortest_distance(int(r), n, scope)[0])
        if scope == IN:
            pr = eng.pagerank(0.85, n, 8)
            opr = o.pagerank(0.85, n, 8)[0]
            fin = np.isfinite(opr)
            assert np.array_equal(np.isfinite(pr), fin)
            assert np.abs(pr[fin] - opr[fin]).sum() <= PR_L1_TOL
            assert np.array_equal(eng.walkcount(2), o.degree_counter(2)[0])


def test_errors_are_reported():
    eng = Engine()
    with pytest.raises(TitanException) as e:
        eng.bfs(0, 3, BOTH)
    assert e.value.code == L.TGO_E_STATE
    src = np.array([0, 1], np.int32)
    dst = np.array([1, 5], np.int32)
    with pytest.raises(TitanException) as e:
        eng.load_edges(3, src, dst, BOTH)
    assert e.value.code == L.TGO_E_INVALID
    eng.load_edges(6, src, dst, BOTH)
    with pytest.raises(TitanException):
        eng.pagerank(0.85, 6, 3)            # PageRank needs a single-direction preload
    with pytest.raises(TitanException):
        eng.bfs(0, 3, IN)                   # scope differs from the preloaded one


# ----------------------------------------------------------------------------- vertex cuts
def test_partition_groups_degree_and_bfs():
    """TitanPartitionGraphTest.testVertexPartitionOlap (:395-435) on the device: DegreeCounter
    gives the group degree at each vertex cut and 1 for every person."""
    eng, rows, vids, sd, npz = engine_from_fixture("partition_groups", IN)
    o = oracle_from_fixture("partition_groups", IN)
    st = eng.stats()
    assert st["partitioned_vertices"] == o.stats.partitioned_vertices == 3
    assert st["partition_rows"] == o.stats.partition_rows
    assert st["ghost_partition_rows"] == o.stats.ghost_partition_rows > 0
    assert sorted(eng.vertex_ids().tolist()) == sorted(int(v) for v in vids)
    assert np.array_equal(reorder(eng.vertex_ids(), eng.walkcount(1), vids), npz["degree1"])
    with pytest.raises(TitanException) as ei:            # no combiner: ThrowingCombiner (FulgoraUtil.java:80-91)
        eng.pagerank(0.85, len(vids), 3)
    assert ei.value.code == L.TGO_E_PROGRAM
    eb, _, _, _, _ = engine_from_fixture("partition_groups", BOTH)
    g0 = int(vids[int(npz["group_index"][0])])
    d = reorder(eb.vertex_ids(), eb.bfs(g0, 10, BOTH), vids)
    assert np.array_equal(np.where(d == ABSENT, -1, d), npz["bfs_both_group0"])


def test_partitioned_hubs_match_oracle():
    """Random weighted graph whose hubs are vertex cuts (edges spread over representative rows,
    each row capped on its own): every program bit-exact against the oracle's Fulgora restatement."""
    import random
    import edgestore as es
    rnd = random.Random(5)
    knows = es.user_edge_label(1)
    wkey = es.user_property_key(1)
    sd = {"edge_types": [{"type_id": knows, "multiplicity": 0, "signature": [wkey]}], "property_keys": [[wkey, 3]]}
    osch = fr.OracleSchema(sd["edge_types"], [tuple(x) for x in sd["property_keys"]])
    n = 600
    edges = [(rnd.randrange(n), rnd.randrange(n), knows, [(wkey, rnd.randint(1, 20))]) for _ in range(6000)]
    for hub in (0, 1, 2):
        edges += [(hub, rnd.randrange(n), knows, [(wkey, rnd.randint(1, 20))]) for _ in range(150)]
        edges += [(rnd.randrange(n), hub, knows, [(wkey, rnd.randint(1, 20))]) for _ in range(150)]
    rows, vids = es.build_rows(es.GraphSpec(n=n, edges=edges, partitioned=[0, 1, 2, 3, 9]), osch)
    for scope in (IN, OUT, BOTH):
        o = fr.OracleGraph.from_rows(rows, osch, scope, hard_limit=12, weight_key=wkey)
        eng = Engine(hard_query_limit=12).load_rows(rows, Schema.from_dict(sd), scope, weight_key=wkey, batch_rows=64)
        ids = eng.vertex_ids()
        assert np.array_equal(ids, o.vertex_ids())
        st = eng.stats()
        assert (st["partitioned_vertices"], st["partition_rows"], st["truncated_results"]) == \
            (o.stats.partitioned_vertices, o.stats.partition_rows, o.stats.truncated_results)
        for r in (0, 3, 17):
            seed = int(vids[r])
            assert np.array_equal(eng.bfs(seed, n, scope), o.shortest_distance(seed, n, scope)[0])
            for depth in (3, n):
                assert np.array_equal(eng.sssp(seed, depth, scope),
                                      o.shortest_distance(seed, depth, scope, weighted=True)[0])
            conv = o.shortest_distance(seed, n, scope, weighted=True)[0]
            assert np.array_equal(eng.sssp(seed, n, scope, mode=L.SSSP_DELTA), conv)
        if scope == IN:
            assert np.array_equal(eng.walkcount(3), o.degree_counter(3)[0])
        if scope != BOTH:
            with pytest.raises(TitanException):
                eng.pagerank(0.85, n, 4)
            with pytest.raises(RuntimeError):
                o.pagerank(0.85, n, 4)


@pytest.mark.parametrize("win", [0, 2])
@pytest.mark.parametrize("tile", ["4096", "8192", "16384"])
@pytest.mark.parametrize("iters", [2, 20])
@pytest.mark.parametrize("hot,seg", [(64, 256), (1000, 100), (4096, 512)])
def test_rmat_pagerank_cache_blocked(rmat12, iters, hot, seg, tile, win, monkeypatch):
    """The cache-blocked PageRank gather (hot CSR + XCD-pinned cold segments, engine.hpp
    ColdBlocks) forced onto a small graph with tiny hot sets / segments (many segments, so
    every XCD has several), with each hot tile size (gather_hot_pf / gather_hot_big), without
    and with the LDS window pass over the hottest hot / win sources (lds_window): oracle bar,
    bitwise reproducible, within rounding of the plain CSR-adaptive gather.  hot >= n means
    nothing is cold (plain path)."""
    n, src, dst, w, ids, oracle, roots = rmat12
    monkeypatch.setenv("TGO_PR_HOT", str(hot))
    monkeypatch.setenv("TGO_PR_SEG", str(seg))
    monkeypatch.setenv("TGO_PR_WIN", str(hot // win if win else 0))
    monkeypatch.setenv("TGO_PR_HOT_TILE", tile)
    eng = Engine().load_edges(n, src, dst, IN)
    pr = eng.pagerank(0.85, n, iters)
    opr, _ = oracle.pagerank(0.85, n, iters)
    assert np.abs(pr - opr).sum() <= PR_L1_TOL
    assert np.array_equal(pr, eng.pagerank(0.85, n, iters))
    # the persistent software-pipelined hot pass (gather_hot_pipe) sums the same tiles in the
    # same order: bitwise equal
    monkeypatch.setenv("TGO_PR_HOT_PIPE", "1")
    assert np.array_equal(pr, Engine().load_edges(n, src, dst, IN).pagerank(0.85, n, iters))
    monkeypatch.delenv("TGO_PR_HOT_PIPE")
    monkeypatch.setenv("TGO_PR_BLOCKED", "0")
    plain = Engine().load_edges(n, src, dst, IN).pagerank(0.85, n, iters)
    assert np.abs(pr - plain).sum() <= 1e-12


@pytest.mark.parametrize("hot", [64, 1000, 3000])
def test_rmat_pagerank_source_split_bitwise(rmat12, hot, monkeypatch):
    """The fixed-point hot pass split over S ranges of the hot sources (TGO_PR_FX_SPLIT = S
    launches, the row sums carried between them): the same exact 128-bit sums, so the ranks are
    bitwise equal for S = 1, 2, 3 and 5, and within the oracle bar."""
    n, src, dst, w, ids, oracle, roots = rmat12
    monkeypatch.setenv("TGO_PR_HOT", str(hot))
    monkeypatch.setenv("TGO_PR_SEG", "256")
    ranks = {}
    for split in (1, 2, 3, 5):
        monkeypatch.setenv("TGO_PR_FX_SPLIT", str(split))
        ranks[split] = Engine().load_edges(n, src, dst, IN).pagerank(0.85, n, 20)
    opr, _ = oracle.pagerank(0.85, n, 20)
    assert np.abs(ranks[1] - opr).sum() <= PR_L1_TOL
    for split in (2, 3, 5):
        assert np.array_equal(ranks[split], ranks[1]), split


def hub_graph(n, hub, k_in, k_out, seed=11):
    """A random background plus a hub receiving `k_in` and sending `k_out` edges."""
    rng = np.random.default_rng(seed)
    src = np.concatenate([rng.integers(0, n, k_in), np.full(k_out, hub), rng.integers(0, n, 200000)]).astype(np.int32)
    dst = np.concatenate([np.full(k_in, hub), rng.integers(0, n, k_out), rng.integers(0, n, 200000)]).astype(np.int32)
    return src, dst


KTILE = 4096     # CSR-adaptive tile (engine.hpp kTile): rows longer than this are split in chunks


@pytest.mark.parametrize("blocked,tile,pipe,win", [("0", "4096", "0", 0), ("1", "4096", "0", 0), ("1", "8192", "0", 0),
                                                   ("1", "16384", "0", 0), ("1", "4096", "1", 0), ("1", "16384", "1", 0),
                                                   ("1", "4096", "0", 8192), ("1", "8192", "0", 512)])
def test_pagerank_long_rows(monkeypatch, blocked, tile, pipe, win):
    """A hub whose in-list spans many tiles: 80 000 entries = ~20 chunks of kTile through
    gather_chunks + finalize_long; cache-blocked with 1024 hot sources and 4096-source cold
    segments, its cold run per segment (~10 000 entries) is cut into several kTile pieces;
    the larger hot tiles cut the hub's hot run into 8192 / 16384-entry chunks (packed words
    with the top bit set).  With an LDS window of 8192 sources (16 384 hot) the hub's ~20 000
    window entries are one long window row, summed by a whole workgroup.  All within 1e-6 L1
    of the oracle and bitwise reproducible."""
    monkeypatch.setenv("TGO_PR_BLOCKED", blocked)
    monkeypatch.setenv("TGO_PR_HOT_TILE", tile)
    monkeypatch.setenv("TGO_PR_HOT_PIPE", pipe)
    monkeypatch.setenv("TGO_PR_HOT", "16384" if win > 1024 else "1024")
    monkeypatch.setenv("TGO_PR_SEG", "4096")
    monkeypatch.setenv("TGO_PR_WIN", str(win))
    n = 1 << 15
    src, dst = hub_graph(n, 7, 80000, 0)
    assert (dst == 7).sum() > 2 * 8 * KTILE
    ids = (np.arange(n, dtype=np.int64) + 1) << 3
    off, mid, adj, ww = numpy_adjacency(n, src, dst, None)
    oracle = fr.OracleGraph.from_adjacency(ids, off, mid, adj, ww)
    eng = Engine(hard_query_limit=1 << 30).load_edges(n, src, dst, IN)
    pr = eng.pagerank(0.85, n, 6)
    opr, _ = oracle.pagerank(0.85, n, 6)
    fin = np.isfinite(opr)
    assert np.array_equal(np.isfinite(pr), fin)
    assert np.abs(pr[fin] - opr[fin]).sum() <= PR_L1_TOL
    assert np.array_equal(pr, eng.pagerank(0.85, n, 6))


def test_walkcount_long_rows():
    """DegreeCounter gathers over OUT lists: an out-hub of 50 000 entries (> 12 tiles) plus an
    in-hub, exact (with Java int wrap) against the oracle."""
    n = 1 << 14
    src, dst = hub_graph(n, 3, 30000, 50000, seed=4)
    ids = (np.arange(n, dtype=np.int64) + 1) << 3
    off, mid, adj, ww = numpy_adjacency(n, src, dst, None)
    oracle = fr.OracleGraph.from_adjacency(ids, off, mid, adj, ww)
    eng = Engine(hard_query_limit=1 << 30).load_edges(n, src, dst, IN)
    assert (src == 3).sum() > 12 * KTILE
    for k in (1, 2, 4):
        assert np.array_equal(eng.walkcount(k), oracle.degree_counter(k)[0])


# ----------------------------------------------------------------------------- typed scopes
def two_label_rows(n=400, seed=21):
    """Rows of a graph with two MULTI labels: `knows` (weighted) and `likes`; a few hubs carry
    more than the small hard limit used below."""
    import random
    import edgestore as es
    rnd = random.Random(seed)
    knows, likes = es.user_edge_label(1), es.user_edge_label(2)
    wkey = es.user_property_key(1)
    sd = {"edge_types": [{"type_id": knows, "multiplicity": 0, "signature": [wkey]},
                         {"type_id": likes, "multiplicity": 0, "signature": [wkey]}],
          "property_keys": [[wkey, 3]]}
    osch = fr.OracleSchema(sd["edge_types"], [tuple(x) for x in sd["property_keys"]])
    edges = []
    for _ in range(4000):
        a, b = rnd.randrange(n), rnd.randrange(n)
        edges.append((a, b, knows if rnd.random() < 0.5 else likes, [(wkey, rnd.randint(1, 9))]))
    for hub in (0, 1):
        edges += [(rnd.randrange(n), hub, knows, [(wkey, rnd.randint(1, 9))]) for _ in range(60)]
        edges += [(hub, rnd.randrange(n), likes, [(wkey, rnd.randint(1, 9))]) for _ in range(60)]
    rows, vids = es.build_rows(es.GraphSpec(n=n, edges=edges), osch)
    return rows, vids, sd, osch, knows, likes, wkey


@pytest.mark.parametrize("scope", [IN, OUT, BOTH])
def test_typed_scope_is_fitted_and_sees_only_its_label(scope):
    """__.inE("knows") etc.: a typed scope sees only that label's entries and is never capped,
    even past the hard limit (BasicVertexCentricQueryBuilder.java:469-474,710-711); the same
    scope untyped is cut at the limit (QueryContainer.java:122)."""
    rows, vids, sd, osch, knows, likes, wkey = two_label_rows()
    limit = 12
    n = len(vids)
    o = fr.OracleGraph.from_rows(rows, osch, scope, hard_limit=limit, labels=[knows], weight_key=wkey)
    eng = Engine(hard_query_limit=limit).load_rows(rows, Schema.from_dict(sd), scope, labels=[knows],
                                                   weight_key=wkey, batch_rows=64)
    assert eng.stats()["truncated_results"] == o.stats.truncated_results == 0
    untyped = fr.OracleGraph.from_rows(rows, osch, scope, hard_limit=limit, weight_key=wkey)
    if scope != BOTH:
        assert untyped.stats.truncated_results > 0
    # only `knows` entries: the typed entry count is that label's share
    off, mid, adj, _ = o.export()
    st = eng.stats()
    assert st["out_entries"] + st["in_entries"] == len(adj)
    for r in (0, 1, 5, 77):
        seed = int(vids[r])
        assert np.array_equal(eng.bfs(seed, n, scope), o.shortest_distance(seed, n, scope)[0])
        assert np.array_equal(eng.sssp(seed, 4, scope), o.shortest_distance(seed, 4, scope, weighted=True)[0])
    if scope == IN:
        assert np.array_equal(eng.walkcount(3), o.degree_counter(3)[0])
    if scope != BOTH:
        pr = eng.pagerank(0.85, n, 8)
        opr = o.pagerank(0.85, n, 8)[0]
        fin = np.isfinite(opr)
        assert np.array_equal(np.isfinite(pr), fin)
        assert np.abs(pr[fin] - opr[fin]).sum() <= PR_L1_TOL


def zero_edge_count_rows(n=2000, hubs=(0, 1, 2), k_in=40, k_out=3, seed=31):
    """Rows where the column-order cut leaves vertices NO OUT entry while their neighbours still
    read them (What's weak 1).  Two MULTI labels, `knows` (lower type id, so first in
    column order; IDHandler.java:103-108) and `likes`.  Each hub receives k_in > limit `knows`
    edges and sends k_out `likes` edges only: its row's user-edge slice is cut inside the `knows`
    IN entries (ColumnValueStore.java:47-69 at QueryContainer's limit, :28,122), so its edgeCount
    is 0 (PageRankVertexProgram.java:80-83), while each `likes` target's short row keeps the IN
    entry and gathers the hub's contribution PR / 0 = +inf (:84-88)."""
    import random
    import edgestore as es
    rnd = random.Random(seed)
    knows, likes = es.user_edge_label(1), es.user_edge_label(2)
    sd = {"edge_types": [{"type_id": knows, "multiplicity": 0}, {"type_id": likes, "multiplicity": 0}],
          "property_keys": []}
    osch = fr.OracleSchema(sd["edge_types"], [])
    edges = []
    for _ in range(2 * n):
        a, b = rnd.randrange(len(hubs), n), rnd.randrange(len(hubs), n)
        edges.append((a, b, knows if rnd.random() < 0.5 else likes, []))
    for h in hubs:
        edges += [(rnd.randrange(len(hubs), n), h, knows, []) for _ in range(k_in)]
        edges += [(h, rnd.randrange(len(hubs), n), likes, []) for _ in range(k_out)]
    rows, vids = es.build_rows(es.GraphSpec(n=n, edges=edges), osch)
    return rows, vids, sd, osch


def assert_pagerank_like_oracle(pr, opr):
    """Java double semantics: the same +inf / NaN positions, finite ranks within 1e-6 L1."""
    assert np.array_equal(np.isnan(pr), np.isnan(opr))
    assert np.array_equal(np.isposinf(pr), np.isposinf(opr)) and np.array_equal(np.isneginf(pr), np.isneginf(opr))
    fin = np.isfinite(opr)
    assert np.abs(pr[fin] - opr[fin]).sum() <= PR_L1_TOL


@pytest.mark.parametrize("split", ["1", "2"])
@pytest.mark.parametrize("cold_fx", ["1", "0"])
def test_pagerank_infinite_contribution_after_cut(split, cold_fx, monkeypatch):
    """The fixed-point PageRank passes (spmv.hip gather_hot_fx / cold_fx) cannot hold +inf:
    a message outside their exact range flags the layout and the program re-runs on the plain
    fp64 gather, so the +inf a zero-edgeCount vertex sends spreads exactly as Java doubles do.
    Forced onto the cache-blocked layout with a tiny hot set; through tgo_load_rows."""
    monkeypatch.setenv("TGO_PR_HOT", "64")
    monkeypatch.setenv("TGO_PR_SEG", "128")
    monkeypatch.setenv("TGO_PR_FX_SPLIT", split)
    monkeypatch.setenv("TGO_PR_FX_COLD", cold_fx)
    rows, vids, sd, osch = zero_edge_count_rows()
    limit, n = 24, len(vids)
    o = fr.OracleGraph.from_rows(rows, osch, IN, hard_limit=limit)
    eng = Engine(hard_query_limit=limit).load_rows(rows, Schema.from_dict(sd), IN, batch_rows=64)
    assert eng.stats()["truncated_results"] == o.stats.truncated_results >= 3
    for iters in (2, 3, 8):
        opr = o.pagerank(0.85, n, iters)[0]
        assert np.isposinf(opr).sum() >= 3 and np.isfinite(opr).sum() > n // 2    # the fixture reaches the case
        pr = eng.pagerank(0.85, n, iters)
        assert_pagerank_like_oracle(pr, opr)
        assert eng.stats()["exact_reruns"] == 1
        assert np.array_equal(pr, eng.pagerank(0.85, n, iters), equal_nan=True)
    # the slot form of the blocked layout (TGO_PR_FX=0) sums doubles itself: no re-run, same ranks
    monkeypatch.setenv("TGO_PR_FX", "0")
    slot = Engine(hard_query_limit=limit).load_rows(rows, Schema.from_dict(sd), IN, batch_rows=64)
    sp = slot.pagerank(0.85, n, 8)
    assert slot.stats()["exact_reruns"] == 0
    assert_pagerank_like_oracle(sp, o.pagerank(0.85, n, 8)[0])
    fin = np.isfinite(sp)
    assert np.array_equal(fin, np.isfinite(pr)) and np.abs(sp[fin] - pr[fin]).sum() <= 1e-12


def test_pagerank_out_of_range_parameters(rmat12, monkeypatch):
    """vertexCount is a user parameter (PageRankVertexProgram.java:54): N = 0 makes every rank
    +inf (1/0 in Java doubles), N = 2^60 puts every contribution below the fixed-point form's
    2^-53 floor.  Both re-run on the fp64 gather and match the oracle."""
    monkeypatch.setenv("TGO_PR_HOT", "512")
    monkeypatch.setenv("TGO_PR_SEG", "256")
    n, src, dst, w, ids, oracle, roots = rmat12
    eng = Engine().load_edges(n, src, dst, IN)
    pr = eng.pagerank(0.85, 0, 6)
    assert eng.stats()["exact_reruns"] == 1 and np.isposinf(pr).all()
    assert_pagerank_like_oracle(pr, oracle.pagerank(0.85, 0, 6)[0])
    big = 1 << 60
    pr = eng.pagerank(0.85, big, 6)
    assert eng.stats()["exact_reruns"] == 1
    opr = oracle.pagerank(0.85, big, 6)[0]
    assert np.allclose(pr, opr, rtol=1e-12, atol=0)
    pr = eng.pagerank(0.85, n, 6)                      # back in range: the fixed-point passes
    assert eng.stats()["exact_reruns"] == 0
    assert np.abs(pr - oracle.pagerank(0.85, n, 6)[0]).sum() <= PR_L1_TOL
    # a damping factor above 1 (the reference takes any alpha, PageRankVertexProgram.java:86)
    # grows the ranks past the split words' exact range (|v| < 2^11, spmv.hip fx_hl) within the
    # run: the emission guard flags the first contribution out of range and the program re-runs
    pr = eng.pagerank(3.0, 1, 16)
    opr = oracle.pagerank(3.0, 1, 16)[0]
    assert eng.stats()["exact_reruns"] == 1 and np.abs(opr).max() > 2.0 ** 20
    assert np.allclose(pr, opr, rtol=1e-12, atol=0)


def test_rows_with_sort_key_weights_and_string_properties():
    """Codec breadth through the device load: a MULTI label whose sort key is
    (String, Float, weight) in DESC order, a String + Double signature and String / Date /
    Character remaining properties; SSSP distances bit-exact against the oracle in every scope,
    cap on (EdgeSerializer.java:130-152,311-313; StringSerializer, FloatSerializer, ...)."""
    import random
    import edgestore as es
    lib = fr.load()
    knows = es.user_edge_label(1)
    w, ks, kf, kd, kdt, kc = (lib.fr_schema_id(0, c) for c in (1, 2, 3, 4, 5, 6))
    pkeys = [(w, 3), (ks, 10), (kf, 5), (kd, 6), (kdt, 8), (kc, 9)]
    sd = {"edge_types": [{"type_id": knows, "multiplicity": 0, "sort_key": [ks, kf, w], "signature": [ks, kd],
                          "order": "DESC"}],
          "property_keys": [list(p) for p in pkeys]}
    osch = fr.OracleSchema(sd["edge_types"], pkeys)
    scale = 9
    src, dst, _ = rmat_edges(scale, 8, seed=5)
    n = 1 << scale
    rnd = random.Random(11)
    edges = []
    for a, b in zip(src, dst):
        props = [(w, rnd.randint(1, 40)), (ks, rnd.choice([0, 7, -31, 123456])), (kf, rnd.randint(-9, 9)),
                 (kd, rnd.randint(-5, 5)), (kdt, rnd.randint(0, 1 << 40)), (kc, rnd.randint(1, 0xFFFF))]
        edges.append((int(a), int(b), knows, [p for p in props if rnd.random() > 0.05 or p[0] == w]))
    rows, vids = es.build_rows(es.GraphSpec(n=n, edges=edges), osch)
    for scope in (IN, OUT, BOTH):
        o = fr.OracleGraph.from_rows(rows, osch, scope, hard_limit=40, weight_key=w)
        eng = Engine(hard_query_limit=40).load_rows(rows, Schema.from_dict(sd), scope, weight_key=w, batch_rows=100)
        assert eng.stats()["truncated_results"] == o.stats.truncated_results
        for r in vids[:3]:
            assert np.array_equal(eng.sssp(int(r), 5, scope), o.shortest_distance(int(r), 5, scope, weighted=True)[0])
            assert np.array_equal(eng.sssp(int(r), n, scope, mode=L.SSSP_DELTA),
                                  o.shortest_distance(int(r), n, scope, weighted=True)[0])

"""GPU parity at the benchmarked sizes (BASELINE.json configs[1] and configs[2]).

Small graphs pin semantics (test_gpu_parity.py); these tests check the HIP engine against the
CPU oracle on the very graphs bench.py measures:

* configs[1] — RMAT scale 20 (ef 16), single-source BFS, through the edgestore path:
  byte-exact rows (tgo_synth_rows) -> tgo_load_rows in work blocks of the reference's
  readBatchSize (FulgoraGraphComputer.java:76-81) -> device decode + CSR -> tgo_bfs.
  inE at the real 100 000-entry preload cap (QueryContainer.java:28,122; RMAT-20 hubs hold
  up to ~138 K entries, so rows ARE cut) and bothE (fitted, uncapped).  Oracle: its own row
  decoder (fr_load_rows) + Fulgora superstep restatement.
* configs[2] — RMAT scale 24: the 64-source multi-source BFS sweep against 64 single-source
  runs and against the oracle for two seeds; PageRank(20) on the capped inE graph within
  1e-6 L1 of the oracle, with the same truncated-row count on both sides.
* configs[4] on one GPU — the bench's weighted RMAT-24 inE graph: delta-stepping SSSP from two
  of the bench's roots and hop-bounded maxDepth 3, bit-exact against the oracle.

Sized so each test finishes in well under two minutes on the GPU box (oracle threads = 16,
the box's CPU share).
"""
import ctypes as C

import numpy as np
import pytest

import fulgora as fr
from titan_amd import Engine, pick_roots, rmat_edges, synth_rows
from titan_amd import _lib as L

pytestmark = pytest.mark.gpu

IN, BOTH = L.SCOPE_IN_E, L.SCOPE_BOTH_E
THREADS = 16
PR_L1_TOL = 1e-6
READ_BATCH = 10 * 1024           # FulgoraGraphComputer readBatchSize = 10 x storage.buffer-size


@pytest.fixture(scope="module")
def rmat20_rows():
    import edgestore as es
    scale = 20
    n = 1 << scale
    src, dst, _ = rmat_edges(scale, 16, seed=0x54495441)
    knows = es.user_edge_label(1)
    rows = synth_rows(n, src, dst, None, label_id=knows, threads=THREADS)
    sd = {"edge_types": [{"type_id": knows, "multiplicity": 0}], "property_keys": []}
    roots = pick_roots(n, src, dst, 4, seed=7)
    vid = np.array([es.vertex_id(int(r)) for r in roots], np.int64)
    return n, rows, sd, vid


@pytest.mark.parametrize("scope", [IN, BOTH])
def test_config2_rmat20_rows_bfs_bit_exact(rmat20_rows, scope):
    from titan_amd import Schema
    n, rows, sd, seeds = rmat20_rows
    osch = fr.OracleSchema(sd["edge_types"], [])
    o = fr.OracleGraph.from_rows(rows, osch, scope, hard_limit=100000).resolve(THREADS)
    eng = Engine(host_threads=THREADS).load_rows(rows, Schema.from_dict(sd), scope, batch_rows=READ_BATCH)
    assert np.array_equal(eng.vertex_ids(), o.vertex_ids())
    st = eng.stats()
    assert st["num_vertices"] == n
    assert st["truncated_results"] == o.stats.truncated_results
    if scope == IN:
        assert st["truncated_results"] > 0          # the real cap is exercised at this scale
    else:
        assert st["truncated_results"] == 0        # bothE is fitted: no limit
    for s in seeds:
        d = eng.bfs(int(s), n, scope, stats=True)
        od, it = o.shortest_distance(int(s), n, scope, threads=THREADS)
        assert it == n
        assert np.array_equal(d, od)
        assert eng.stats()["reached"] == int((od != L.DIST_ABSENT).sum())


@pytest.fixture(scope="module")
def rmat24():
    scale = 24
    n = 1 << scale
    src, dst, w = rmat_edges(scale, 16, seed=0x54495441, weights=True)     # bench.py's graph and weights
    roots = pick_roots(n, src, dst, 64, seed=7)
    return n, src, dst, roots, w


@pytest.fixture(scope="module")
def oracle24_in_capped(rmat24):
    """The oracle's inE graph at the real 100 000-entry cap, with the bench's weights (PageRank
    ignores them): shared by the PageRank and SSSP tests."""
    n, src, dst, roots, w = rmat24
    return fr.OracleGraph.from_edges(n, src, dst, w, hard_limit=100000).resolve(THREADS)


def test_config3_rmat24_msbfs_sweep(rmat24):
    """All 64 seeds of the bench's sweep equal their single-source runs; two equal the oracle."""
    n, src, dst, roots, _ = rmat24
    eng = Engine(host_threads=THREADS).load_edges(n, src, dst, BOTH, apply_cap=False)
    eng.bfs_multi(roots, n, BOTH, seed_is_dense=True, stats=True, fetch=False)
    reached, entries = eng.multi_stats(len(roots))
    ms = np.empty(n, np.int64)
    for i, r in enumerate(roots):
        assert eng.lib.tgo_copy_multi_distances(eng.ctx, i, L.ptr(ms, C.c_int64)) == 0
        single = eng.bfs(int(r), n, BOTH, seed_is_dense=True, stats=True)
        assert np.array_equal(ms, single), i
        assert reached[i] == eng.stats()["reached"]
        assert entries[i] == eng.stats()["reached_entries"]
    keep = {int(roots[0]): eng.bfs(int(roots[0]), n, BOTH, seed_is_dense=True),
            int(roots[37]): eng.bfs(int(roots[37]), n, BOTH, seed_is_dense=True)}
    del eng
    o = fr.OracleGraph.from_edges(n, src, dst).resolve(THREADS)
    for r, d in keep.items():
        od, _ = o.shortest_distance(int((r + 1) << 3), n, BOTH, threads=THREADS)
        assert np.array_equal(d, od), r


def test_config3_rmat24_pagerank_capped(rmat24, oracle24_in_capped):
    """PageRank(20) on the capped inE graph (25 rows cut at 100 000 entries)."""
    n, src, dst, roots, _ = rmat24
    eng = Engine(host_threads=THREADS).load_edges(n, src, dst, IN, apply_cap=True)
    pr = eng.pagerank(0.85, n, 20)
    assert np.array_equal(pr, eng.pagerank(0.85, n, 20))             # fixed reduction order
    st = eng.stats()
    d_in = eng.bfs(int(roots[1]), n, IN, seed_is_dense=True)
    del eng
    o = oracle24_in_capped
    assert st["truncated_results"] == o.stats.truncated_results > 0
    opr, it = o.pagerank(0.85, n, 20, threads=THREADS)
    assert it == 20
    fin = np.isfinite(opr)
    assert np.array_equal(np.isfinite(pr), fin)
    assert np.abs(pr[fin] - opr[fin]).sum() <= PR_L1_TOL
    od, _ = o.shortest_distance(int((int(roots[1]) + 1) << 3), n, IN, threads=THREADS)
    assert np.array_equal(d_in, od)


def test_config5_rmat24_weighted_sssp(rmat24, oracle24_in_capped):
    """configs[4] at the size bench.py measures it: weighted inE ShortestDistance (int32 weights
    1 + splitmix64 mod 255, the 100 000 cap on) from the first two of the bench's SSSP roots
    (roots whose reach is the giant component).  Delta-stepping gives the converged distances,
    bit-exact against the oracle's Jacobi supersteps run to their fixpoint
    (ShortestDistanceVertexProgram.java:96-130); hop-bounded maxDepth 3 gives the reference's
    3-superstep distances exactly.  Reached counts equal; relaxed/reached stays near 1."""
    n, src, dst, roots, w = rmat24
    eng = Engine(host_threads=THREADS).load_edges(n, src, dst, IN, weight=w, apply_cap=True)
    picked = []
    for r in roots:
        d = eng.sssp(int(r), n, IN, mode=L.SSSP_DELTA, seed_is_dense=True, stats=True)
        st = eng.stats()
        if st["reached"] * 4 < n:                 # bench.py sssp_leg: the giant component only
            continue
        assert st["relaxed_entries"] <= 1.5 * st["reached_entries"]
        picked.append((int(r), d, st["reached"]))
        if len(picked) == 2:
            break
    assert len(picked) == 2
    hop3 = eng.sssp(picked[0][0], 3, IN, mode=L.SSSP_HOP_BOUNDED, seed_is_dense=True, stats=True)
    hop3_reached = eng.stats()["reached"]
    eng.set_tuning(L.TUNE_DS_SMALL, 1)            # tiny steps in one block: the same distances
    for r, d, _ in picked:
        assert np.array_equal(eng.sssp(r, n, IN, mode=L.SSSP_DELTA, seed_is_dense=True), d), r
    del eng
    o = oracle24_in_capped
    for r, d, reached in picked:
        od, it = o.shortest_distance((r + 1) << 3, n, IN, weighted=True, threads=THREADS)
        assert it == n
        assert np.array_equal(d, od), r
        assert reached == int((od != L.DIST_ABSENT).sum())
    od3, it = o.shortest_distance((picked[0][0] + 1) << 3, 3, IN, weighted=True, threads=THREADS)
    assert it == 3
    assert np.array_equal(hop3, od3)
    assert hop3_reached == int((od3 != L.DIST_ABSENT).sum())


def test_wide_bitmap_single_source_bfs():
    """More vertices than one launch grid has threads (2^26 vertices = 1 M bitmap words,
    the capped grids cover 524 288): every per-level bitmap clear must reach the whole array.
    At RMAT-27 the one-thread-per-word level_prep left the next-frontier tail stale and 24 of
    the 64 single-source runs differed from the sweep (profiles/r03d_scale27_one_gpu.json).
    Single-source direction-optimizing BFS == multi-source sweep == hop-bounded Jacobi."""
    scale = 26
    n = 1 << scale
    src, dst, _ = rmat_edges(scale, 2, seed=0x54495441)
    roots = [int(r) for r in pick_roots(n, src, dst, 4, seed=7)]
    eng = Engine(host_threads=16).load_edges(n, src, dst, L.SCOPE_BOTH_E, apply_cap=False)
    del src, dst
    eng.bfs_multi(roots, n, L.SCOPE_BOTH_E, seed_is_dense=True, fetch=False)
    ms = np.empty(n, np.int64)
    for i, r in enumerate(roots):
        eng.lib.tgo_copy_multi_distances(eng.ctx, i, L.ptr(ms, C.c_int64))
        bf = eng.bfs(r, n, L.SCOPE_BOTH_E, seed_is_dense=True)
        assert np.array_equal(ms, bf), (i, int(np.sum(ms != bf)))
        if i == 0:
            hb = eng.sssp(r, 64, L.SCOPE_BOTH_E, mode=L.SSSP_HOP_BOUNDED, seed_is_dense=True)
            assert np.array_equal(hb, bf)


@pytest.mark.parametrize("world", [2, 4])
def test_config5_rmat24_weighted_sssp_partitioned(rmat24, world):
    """configs[4] partitioned: the bench's weighted, capped RMAT-24 inE graph over `world`
    ranks (equal ranges, degree-grouped global layout, one device, ranks as threads with the
    drivers' collectives in-process) — the native loop bench.py times at N > 1
    (tgo_part_sssp_run) gives delta-stepping distances equal to the one-GPU engine's bit for bit
    (that engine is oracle-pinned in test_config5_rmat24_weighted_sssp) for both roots, reached
    counts global, every rank through the same phases; the Python driver agrees on one root."""
    from test_gpu_distributed import Ranks
    from titan_amd.distributed import NativeExchange, distributed_sssp, distributed_sssp_native
    n, src, dst, roots, w = rmat24
    one = Engine(host_threads=THREADS).load_edges(n, src, dst, IN, weight=w, apply_cap=True)
    picked = []
    for r in roots:
        d = one.sssp(int(r), n, IN, mode=L.SSSP_DELTA, seed_is_dense=True, stats=True)
        if one.stats()["reached"] * 4 >= n:                  # the giant component, as bench.py
            picked.append((int(r), d, one.stats()["reached"]))
        if len(picked) == 2:
            break
    del one
    ranks = Ranks(world, n, src, dst, IN, weight=w, layout=True, apply_cap=True)
    xs = NativeExchange.local_group(world)
    for r, d, reached in picked:
        res = ranks.run(lambda be, comm: distributed_sssp_native(be, r, xs[comm.rank]))
        assert np.array_equal(np.concatenate([x[0] for x in res]), d), r
        assert all(x[1][0] == reached for x in res)
        assert len({x[2] for x in res}) == 1
    r, d, reached = picked[0]
    res = ranks.run(lambda be, comm: distributed_sssp(be, r, 0, comm=comm))
    assert np.array_equal(np.concatenate([x[0] for x in res]), d), r
    assert all(x[1][0] == reached for x in res)


@pytest.fixture(scope="module")
def rmat24_one_gpu(rmat24):
    """One-GPU results on the bench's RMAT-24 graphs (each pinned to the oracle by the config
    tests above): bothE BFS / the multi-source sweep, capped inE PageRank(20), weighted capped
    inE delta-stepping SSSP.  Engines are dropped: only the arrays stay."""
    n, src, dst, roots, w = rmat24
    seeds = [int(r) for r in roots[:8]]
    eb = Engine(host_threads=THREADS).load_edges(n, src, dst, BOTH, apply_cap=False)
    eb.bfs_multi(seeds, n, BOTH, seed_is_dense=True, fetch=False)
    ms = []
    for i in range(len(seeds)):
        d = np.empty(n, np.int64)
        eb.lib.tgo_copy_multi_distances(eb.ctx, i, L.ptr(d, C.c_int64))
        ms.append(d)
    del eb
    ep = Engine(host_threads=THREADS).load_edges(n, src, dst, IN, apply_cap=True)
    pr = ep.pagerank(0.85, n, 20)
    del ep
    es = Engine(host_threads=THREADS).load_edges(n, src, dst, IN, weight=w, apply_cap=True)
    for r in roots:
        d = es.sssp(int(r), n, IN, mode=L.SSSP_DELTA, seed_is_dense=True, stats=True)
        if es.stats()["reached"] * 4 >= n:
            sssp = (int(r), d)
            break
    del es
    return seeds, ms, pr, sssp


@pytest.mark.parametrize("world", [8, 6])
def test_rmat24_every_native_loop_at_world(rmat24, rmat24_one_gpu, world):
    """world 8 (north_star's node) and a non-power-of-two world 6 (edge-
    balanced slot ranges, as bench.py partitions) on the bench's RMAT-24 graphs, every native
    partitioned loop over an in-process exchange group on one device: the 8-source sweep and
    single-source BFS (bothE), PageRank(20) in both exchanges (capped inE: the hot-first blocked
    layout, 8 / 6 peers' ghost sets) and weighted delta SSSP (capped inE: the W-slice pair
    exchange) — BFS / SSSP bit-exact and PageRank within 1e-6 L1 of the one-GPU results."""
    from test_gpu_distributed import Ranks
    from titan_amd.distributed import (NativeExchange, PR_EXCHANGE_ALLGATHER, PR_EXCHANGE_GHOST, SlotPartition,
                                       distributed_bfs_native, distributed_msbfs_native, distributed_pagerank_native,
                                       distributed_sssp_native, word_weights)
    n, src, dst, roots, w = rmat24
    seeds, ms, pr_one, (sroot, sd_one) = rmat24_one_gpu
    part = None if world == 8 else SlotPartition.balanced(word_weights(src, dst, 0, n), world)
    ns = n if part is None else part.n_slots
    slot = (lambda v: int(v)) if part is None else (lambda v: int(part.to_slots(np.asarray([v]))[0]))

    def cut(per_rank):
        if part is None:
            return np.concatenate(per_rank)
        return np.concatenate([part.slot_results(r, x) for r, x in enumerate(per_rank)])
    xs = NativeExchange.local_group(world)
    ranks = Ranks(world, n, src, dst, BOTH, layout=True, device_counts=True, part=part)
    res = ranks.run(lambda be, comm: (distributed_msbfs_native(be, [slot(s) for s in seeds], ns, xs[comm.rank]),
                                      [be.ms_levels(i) for i in range(len(seeds))]))
    for i in range(len(seeds)):
        assert np.array_equal(cut([r[1][i] for r in res]), ms[i]), i
        assert all(r[0][0][i] == int((ms[i] != L.DIST_ABSENT).sum()) for r in res)
    res = ranks.run(lambda be, comm: distributed_bfs_native(be, slot(seeds[0]), ns, xs[comm.rank]))
    assert np.array_equal(cut([r[0] for r in res]), ms[0])
    del ranks
    ranks = Ranks(world, n, src, dst, IN, layout=True, apply_cap=True, part=part)
    for mode in (PR_EXCHANGE_ALLGATHER, PR_EXCHANGE_GHOST):
        res = ranks.run(lambda be, comm: distributed_pagerank_native(be, 0.85, n, 20, xs[comm.rank], mode=mode))
        got = cut([r[0] for r in res])
        assert np.abs(got - pr_one).sum() <= PR_L1_TOL, mode
    del ranks
    ranks = Ranks(world, n, src, dst, IN, weight=w, layout=True, apply_cap=True, part=part)
    res = ranks.run(lambda be, comm: distributed_sssp_native(be, slot(sroot), xs[comm.rank]))
    assert np.array_equal(cut([r[0] for r in res]), sd_one)
    assert len({r[2] for r in res}) == 1

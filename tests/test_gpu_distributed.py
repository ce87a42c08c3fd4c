"""GPU: the partitioned (multi-GPU) path — the REAL drivers of titan_amd/distributed.py
(distributed_bfs / distributed_msbfs / distributed_sssp / distributed_pagerank) over the HIP
local steps (HipPartBackend, titan_gpu_olap_part.h).  The 1-GPU box has one device, so the
ranks run in ONE process: every rank is a thread with its own Engine (ctx, partition, HIP
stream), and titan_amd.distributed.InProcessGroup performs the drivers' all-to-all /
all-gather / all-reduce as thread rendezvous with torch ops on the device.  Results must equal
the oracle bit-for-bit (BFS / SSSP levels and distances) or within 1e-6 L1 (PageRank).
"""
import numpy as np
import pytest
import torch

import fulgora as fr
from titan_amd import Engine, rmat_edges
from titan_amd import _lib as L
from titan_amd.distributed import (HipPartBackend, InProcessGroup, SlotPartition, distributed_bfs,
                                   distributed_msbfs, distributed_pagerank, distributed_sssp, exchange_stream,
                                   local_layout, pagerank_layout, partition_range, word_weights)
from titan_amd.engine import TitanException

pytestmark = pytest.mark.gpu
ABSENT = L.DIST_ABSENT


class Ranks:
    """One Engine + HipPartBackend + HIP stream per simulated rank; run() drives a function
    on every rank's thread with that rank's communicator."""

    def __init__(self, world, n, src, dst, scope, weight=None, layout=False, apply_cap=False, hard_limit=100000,
                 device_counts=False, part=None):
        # part (SlotPartition): edge-balanced ranges — the engines see slot ids over n_slots
        if part is not None:
            src, dst, n = part.to_slots(src), part.to_slots(dst), part.n_slots
        rng = (lambda r: part.slot_range(r)) if part is not None else (lambda r: partition_range(n, world, r))
        lay = None
        if layout:
            lay = np.concatenate([local_layout(src, dst, n, *rng(r)) for r in range(world)])
            assert np.array_equal(np.sort(lay), np.arange(n))
        self.world, self.streams, self.backends = world, [], []
        for r in range(world):
            lo, hi = rng(r)
            s = torch.cuda.Stream()
            with torch.cuda.stream(s):
                eng = Engine(stream=s.cuda_stream, hard_query_limit=hard_limit).load_partition(
                    n, lo, hi, src, dst, scope, weight=weight, apply_cap=apply_cap, layout=lay)
                self.backends.append(HipPartBackend(eng, n, lo, hi, device_counts=device_counts))
            self.streams.append(s)

    def run(self, fn):
        def body(rank, comm):
            torch.cuda.set_stream(self.streams[rank])
            return fn(self.backends[rank], comm)
        return InProcessGroup(self.world).run(body)


@pytest.mark.parametrize("layout", [False, True])
@pytest.mark.parametrize("world,scope", [(2, L.SCOPE_IN_E), (4, L.SCOPE_OUT_E), (4, L.SCOPE_BOTH_E)])
def test_partitioned_delta_stepping(world, scope, layout):
    scale = 12
    n = 1 << scale
    src, dst, w = rmat_edges(scale, 16, seed=35, weights=True)
    ranks = Ranks(world, n, src, dst, scope, weight=w, layout=layout)
    og = fr.OracleGraph.from_edges(n, src, dst, w)
    ids = (np.arange(n, dtype=np.int64) + 1) << 3
    for seed in (int(src[0]), int(dst[9])):
        od, _ = og.shortest_distance(int(ids[seed]), n, scope, weighted=True)
        for delta in (0, 1, 1 << 40):
            res = ranks.run(lambda be, comm: distributed_sssp(be, seed, delta, comm=comm))
            d = np.concatenate([x[0] for x in res])
            assert np.array_equal(d, od), (seed, delta)
            assert all(x[1][0] == int((od != ABSENT).sum()) for x in res)
            assert len({x[2] for x in res}) == 1                  # every rank ran the same phases


@pytest.mark.parametrize("layout", [False, True])
@pytest.mark.parametrize("world,scope", [(2, L.SCOPE_IN_E), (4, L.SCOPE_IN_E), (3, L.SCOPE_OUT_E)])
def test_partitioned_delta_stepping_capped(world, scope, layout):
    """Capped single-direction scopes (QueryContainer.java:28,122 at a small limit): a vertex
    pushes to v only if it survived in v's cut pull list, and v may live on another rank — the
    partition load builds its push rows from the global cut (the one-GPU load's explicit
    transpose).  Weighted delta-stepping equals the oracle's converged distances bit for bit.
    (Found at RMAT-24 with the real 100 000 cap: a hub's own IN list, cut after its OUT
    entries, missed pushes its receivers' uncut OUT lists hold.)"""
    scale = 12
    n = 1 << scale
    limit = 40
    src, dst, w = rmat_edges(scale, 16, seed=39, weights=True)
    if world == 3:
        n = 3 * 1408                                  # 64-aligned equal thirds past the RMAT range
    ranks = Ranks(world, n, src, dst, scope, weight=w, layout=layout, apply_cap=True, hard_limit=limit)
    og = fr.OracleGraph.from_edges(n, src, dst, w, hard_limit=limit)
    assert sum(be.e.stats()["truncated_results"] for be in ranks.backends) == og.stats.truncated_results > 0
    ids = (np.arange(n, dtype=np.int64) + 1) << 3
    deg = np.bincount(src, minlength=n) + np.bincount(dst, minlength=n)
    for seed in (int(np.argmax(deg)), int(src[3]), int(dst[11])):
        od, _ = og.shortest_distance(int(ids[seed]), n, scope, weighted=True)
        res = ranks.run(lambda be, comm: distributed_sssp(be, seed, 0, comm=comm))
        assert np.array_equal(np.concatenate([x[0] for x in res]), od), seed
        assert all(x[1][0] == int((od != ABSENT).sum()) for x in res)


@pytest.mark.parametrize("device_counts", [False, True])
@pytest.mark.parametrize("layout", [False, True])
@pytest.mark.parametrize("world", [2, 4])
def test_partitioned_multi_source_bfs(world, layout, device_counts):
    scale = 12
    n = 1 << scale
    src, dst, _ = rmat_edges(scale, 16, seed=33)
    ranks = Ranks(world, n, src, dst, L.SCOPE_BOTH_E, layout=layout, device_counts=device_counts)
    nfixed = [0] * world
    for r, be in enumerate(ranks.backends):                   # count the fixed-capacity exchanges
        def counted(*a, _f=be.ms_pack_fixed, _r=r):
            nfixed[_r] += 1
            return _f(*a)
        be.ms_pack_fixed = counted
    og = fr.OracleGraph.from_edges(n, src, dst)
    ids = (np.arange(n, dtype=np.int64) + 1) << 3
    rng = np.random.default_rng(5)
    seeds = [int(s) for s in rng.choice(n, 40, replace=False)] + [int(src[0])]
    expect = [og.shortest_distance(int(ids[s]), n, 2)[0] for s in seeds]
    # mixed levels with the default sparse exchange (fixed capacity), sized pairs (fixed=0),
    # whole-slice all-to-all; always push in each form; always pull
    for ms_alpha, sparse, fixed in ((12.0, True, None), (12.0, True, 0), (12.0, False, None), (1e9, True, None),
                                    (1e9, True, 0), (1e9, False, None), (1e-9, True, None)):
        def body(be, comm):
            r, e, lv = distributed_msbfs(be, seeds, n, ms_alpha=ms_alpha, sparse_exchange=sparse,
                                         fixed_exchange_bytes=fixed, comm=comm)
            return r, [be.ms_levels(i) for i in range(len(seeds))]
        res = ranks.run(body)
        for i, od in enumerate(expect):
            assert np.array_equal(np.concatenate([x[1][i] for x in res]), od), (ms_alpha, sparse, fixed, i)
            assert all(x[0][i] == int((od != ABSENT).sum()) for x in res)
    assert min(nfixed) > 0                                     # the fixed-capacity exchange ran on every rank


@pytest.mark.parametrize("layout", [False, True])
@pytest.mark.parametrize("world", [2, 4])
def test_partitioned_bfs_and_plain_pagerank(world, layout):
    scale = 12
    n = 1 << scale
    src, dst, _ = rmat_edges(scale, 16, seed=31)
    ranks = Ranks(world, n, src, dst, L.SCOPE_BOTH_E, layout=layout)
    og = fr.OracleGraph.from_edges(n, src, dst)
    ids = (np.arange(n, dtype=np.int64) + 1) << 3
    for seed in (int(src[0]), int(dst[9]), int(src[100])):
        od, _ = og.shortest_distance(int(ids[seed]), n, 2)
        for alpha in (15.0, 1e9):
            res = ranks.run(lambda be, comm: distributed_bfs(be, seed, n, alpha=alpha, comm=comm))
            assert np.array_equal(np.concatenate([x[0] for x in res]), od)
            assert all(x[1][0] == int((od != ABSENT).sum()) for x in res)
    # PageRank on the same partitions (the in-lists of a bothE load) with the plain
    # rank-major all-gather: a bothE load is never cache-blocked (tgo_part_pr_blocked)
    iters = 10
    assert set(ranks.run(lambda be, comm: pagerank_layout(be, comm=comm))) == {(0, n // world)}
    res = ranks.run(lambda be, comm: distributed_pagerank(be, 0.85, n, iters, comm=comm))
    pr = np.concatenate(res)
    opr, _ = og.pagerank(0.85, n, iters)
    fin = np.isfinite(opr)
    assert np.array_equal(np.isfinite(pr), fin)
    assert np.abs(pr[fin] - opr[fin]).sum() <= 1e-6


@pytest.mark.parametrize("overlap", [True, False])
@pytest.mark.parametrize("layout", [False, True])
@pytest.mark.parametrize("world", [1, 2, 4])
def test_partitioned_pagerank(world, layout, overlap, monkeypatch):
    """distributed_pagerank over inE lists: the plain all-gather and the cache-blocked
    hot-first gathered layout (tgo_part_pr_blocked; small hot set / segments so every rank
    has hot rows, cold pieces in several segments and entry-less rows past the span)."""
    monkeypatch.setenv("TGO_PR_HOT", "512")
    monkeypatch.setenv("TGO_PR_SEG", "256")
    scale = 12
    n = 1 << scale
    src, dst, _ = rmat_edges(scale, 16, seed=37)
    ranks = Ranks(world, n, src, dst, L.SCOPE_IN_E, layout=layout)
    og = fr.OracleGraph.from_edges(n, src, dst)
    lays = ranks.run(lambda be, comm: pagerank_layout(be, comm=comm))
    assert len(set(lays)) == 1
    hot, span = lays[0]
    assert hot == max(64, 512 // world // 64 * 64)
    if layout:
        assert span < n // world                               # entry-less rows are not exchanged
    for iters in (2, 10):
        opr, _ = og.pagerank(0.85, n, iters)
        fin = np.isfinite(opr)
        res = ranks.run(lambda be, comm: distributed_pagerank(be, 0.85, n, iters, layout=(hot, span), overlap=overlap,
                                                              comm=comm))
        pr = np.concatenate(res)
        assert np.array_equal(np.isfinite(pr), fin)
        assert np.abs(pr[fin] - opr[fin]).sum() <= 1e-6
    be = ranks.backends[0]
    with pytest.raises(TitanException):                        # rank property only after the last step
        be.pr_begin(0.85, n, 5, be.tensor(be.n_local, torch.float64))
        be.pr_end(True)


@pytest.mark.parametrize("world", [2, 4])
def test_partitioned_pagerank_capped(world, monkeypatch):
    """The bench loads partitioned PageRank with the preload cap on: rows cut at the hard
    limit in column order (QueryContainer.java:28,122), the same cut as one GPU and the oracle."""
    monkeypatch.setenv("TGO_PR_HOT", "512")
    monkeypatch.setenv("TGO_PR_SEG", "256")
    scale = 12
    n = 1 << scale
    limit = 40
    src, dst, _ = rmat_edges(scale, 16, seed=43)
    ranks = Ranks(world, n, src, dst, L.SCOPE_IN_E, layout=True, apply_cap=True, hard_limit=limit)
    og = fr.OracleGraph.from_edges(n, src, dst, hard_limit=limit)
    trunc = sum(be.e.stats()["truncated_results"] for be in ranks.backends)
    assert trunc == og.stats.truncated_results > 0
    for iters in (3, 20):
        res = ranks.run(lambda be, comm: distributed_pagerank(be, 0.85, n, iters, comm=comm))
        pr = np.concatenate(res)
        opr, _ = og.pagerank(0.85, n, iters)
        fin = np.isfinite(opr)
        assert np.array_equal(np.isfinite(pr), fin)
        assert np.abs(pr[fin] - opr[fin]).sum() <= 1e-6
    one = Engine(hard_query_limit=limit).load_edges(n, src, dst, L.SCOPE_IN_E, apply_cap=True)
    assert one.stats()["truncated_results"] == trunc


def test_fixed_exchange_overflow_fails_the_sweep():
    """A fixed-capacity pack whose owner receives more pairs than `cap` fails tgo_part_ms_end
    (the dropped pairs would give wrong levels); the flag does not leak into the next sweep."""
    scale = 10
    n = 1 << scale
    src, dst, _ = rmat_edges(scale, 16, seed=47)
    st = exchange_stream()
    be = HipPartBackend(Engine(stream=st).load_partition(n, 0, n, src, dst, L.SCOPE_BOTH_E, apply_cap=False),
                        n, 0, n)
    deg = np.bincount(src, minlength=n) + np.bincount(dst, minlength=n)
    seed = int(np.argmax(deg))
    fr_ = be.tensor(n, torch.int64)
    cand = be.tensor(n, torch.int64)
    send = be.tensor(2 * n + 2, torch.int64)
    be.ms_begin([seed], fr_)
    be.ms_push(0, fr_, cand)
    be.ms_pack_fixed(cand, send, 1, 1)                   # the hub's neighbours do not fit one pair
    with pytest.raises(TitanException, match="capacity"):
        be.ms_end(1)
    og = fr.OracleGraph.from_edges(n, src, dst)
    r, _, _ = distributed_msbfs_world1(be, [seed], n)
    od, _ = og.shortest_distance(int((seed + 1) << 3), n, 2)
    assert np.array_equal(be.ms_levels(0), od)
    assert r[0] == int((od != ABSENT).sum())


def distributed_msbfs_world1(be, seeds, n):
    return InProcessGroup(1).run(lambda rank, comm: distributed_msbfs(be, seeds, n, comm=comm))[0]


def test_partition_load_drops_the_last_programs_results():
    """a partition load frees the scratch a finished program's results live in,
    so tgo_result_rows must refuse afterwards instead of reading freed device memory."""
    scale = 10
    n = 1 << scale
    src, dst, _ = rmat_edges(scale, 16, seed=53)
    eng = Engine(stream=exchange_stream()).load_edges(n, src, dst, L.SCOPE_IN_E)
    eng.bfs(int(src[0]), n, L.SCOPE_IN_E, seed_is_dense=True)
    assert eng.result_rows(L.RESULT_DISTANCE, [(900 << 6) | 5], [L.DT_LONG], 1 << 20).nrows > 0
    eng.load_partition(n, 0, n, src, dst, L.SCOPE_BOTH_E, apply_cap=False)
    with pytest.raises(TitanException) as ei:
        eng.result_rows(L.RESULT_DISTANCE, [(900 << 6) | 5], [L.DT_LONG], 1 << 20)
    assert ei.value.code == L.TGO_E_STATE


def test_drivers_on_a_real_world1_group(monkeypatch):
    """The real drivers on a one-rank RCCL group (TorchComm over backend "nccl"): device-
    resident level counts (tgo_part_device_counts) for BFS / multi-source BFS, and the
    cache-blocked PageRank exchange with the hot all-gather overlapping the cold phase."""
    import socket
    import torch.distributed as dist
    monkeypatch.setenv("TGO_PR_HOT", "512")
    monkeypatch.setenv("TGO_PR_SEG", "256")
    sock = socket.socket()
    sock.bind(("127.0.0.1", 0))
    port = sock.getsockname()[1]
    sock.close()
    dist.init_process_group("nccl", init_method=f"tcp://127.0.0.1:{port}", rank=0, world_size=1,
                            device_id=torch.device("cuda", 0))
    try:
        scale = 12
        n = 1 << scale
        src, dst, _ = rmat_edges(scale, 16, seed=41)
        lay = local_layout(src, dst, n, 0, n)
        st = exchange_stream()
        bfs_be = HipPartBackend(Engine(stream=st).load_partition(n, 0, n, src, dst, L.SCOPE_BOTH_E, apply_cap=False,
                                                                  layout=lay), n, 0, n, device_counts=True)
        og = fr.OracleGraph.from_edges(n, src, dst)
        ids = (np.arange(n, dtype=np.int64) + 1) << 3
        seeds = [int(src[0]), int(dst[7]), int(src[300])]
        for seed in seeds:
            od, _ = og.shortest_distance(int(ids[seed]), n, 2)
            d, reached, _ = distributed_bfs(bfs_be, seed, n)
            assert np.array_equal(d, od)
            assert reached[0] == int((od != ABSENT).sum())
        # default (fixed-capacity exchange on small sparse levels), sized pairs only, push only
        for alpha, fixed in ((12.0, None), (12.0, 0), (1e9, None), (1e9, 0)):
            r, _, _ = distributed_msbfs(bfs_be, seeds, n, ms_alpha=alpha, fixed_exchange_bytes=fixed)
            for i, seed in enumerate(seeds):
                od, _ = og.shortest_distance(int(ids[seed]), n, 2)
                assert np.array_equal(bfs_be.ms_levels(i), od)
                assert r[i] == int((od != ABSENT).sum())
        pr_be = HipPartBackend(Engine(stream=st).load_partition(n, 0, n, src, dst, L.SCOPE_IN_E, apply_cap=False,
                                                                 layout=lay), n, 0, n)
        hot, span = pagerank_layout(pr_be)
        assert hot == 512 and span < n
        pr = distributed_pagerank(pr_be, 0.85, n, 10, layout=(hot, span))
        opr, _ = og.pagerank(0.85, n, 10)
        fin = np.isfinite(opr)
        assert np.array_equal(np.isfinite(pr), fin)
        assert np.abs(pr[fin] - opr[fin]).sum() <= 1e-6
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 4])
def test_edge_balanced_partition_drivers(world, monkeypatch):
    """Edge-balanced ranges (SlotPartition, what bench.py's partitioned path runs): unequal
    64-aligned caller ranges in equal exchange slots, the real drivers over the HIP local
    steps — BFS / multi-source BFS / delta SSSP bit-exact and capped cache-blocked PageRank
    within 1e-6 L1 of the oracle, results mapped back to caller ids."""
    scale = 12
    n = 1 << scale
    src, dst, w = rmat_edges(scale, 16, seed=43, weights=True)
    part = SlotPartition.balanced(word_weights(src, dst, 0, n), world)
    assert part.n_slots > n                                   # unequal ranges: padded slots
    og = fr.OracleGraph.from_edges(n, src, dst, w)
    ids = (np.arange(n, dtype=np.int64) + 1) << 3
    roots = [int(src[0]), int(dst[9]), int(src[100])]
    rs = [int(x) for x in part.to_slots(np.asarray(roots))]
    ns = part.n_slots
    cut = lambda res, k: np.concatenate([part.slot_results(r, x[k]) for r, x in enumerate(res)])  # noqa: E731
    ranks = Ranks(world, n, src, dst, L.SCOPE_BOTH_E, layout=True, device_counts=True, part=part)
    res = ranks.run(lambda be, comm: distributed_bfs(be, rs[0], ns, comm=comm))
    od, _ = og.shortest_distance(int(ids[roots[0]]), n, 2)
    assert np.array_equal(cut(res, 0), od)

    def ms(be, comm):
        r, _, _ = distributed_msbfs(be, rs, ns, comm=comm)
        return [be.ms_levels(i) for i in range(len(rs))], r
    res = ranks.run(ms)
    for i, root in enumerate(roots):
        o, _ = og.shortest_distance(int(ids[root]), n, 2)
        assert np.array_equal(np.concatenate([part.slot_results(r, x[0][i]) for r, x in enumerate(res)]), o)
        assert res[0][1][i] == int((o != ABSENT).sum())
    hard = 40
    monkeypatch.setenv("TGO_PR_HOT", "512")
    monkeypatch.setenv("TGO_PR_SEG", "256")
    pr_ranks = Ranks(world, n, src, dst, L.SCOPE_IN_E, layout=True, apply_cap=True, hard_limit=hard, part=part)

    def pr(be, comm):
        lay = pagerank_layout(be, comm=comm)
        return (distributed_pagerank(be, 0.85, n, 12, layout=lay, comm=comm), lay)
    res = pr_ranks.run(pr)
    assert res[0][1][0] > 0                                   # the blocked hot-first layout ran
    opr, _ = fr.OracleGraph.from_edges(n, src, dst, hard_limit=hard).pagerank(0.85, n, 12)
    got = cut(res, 0)
    fin = np.isfinite(opr)
    assert np.array_equal(np.isfinite(got), fin) and np.abs(got[fin] - opr[fin]).sum() <= 1e-6
    w_ranks = Ranks(world, n, src, dst, L.SCOPE_IN_E, weight=w, layout=True, part=part)
    res = w_ranks.run(lambda be, comm: distributed_sssp(be, rs[1], 0, comm=comm))
    osd, _ = og.shortest_distance(int(ids[roots[1]]), n, L.SCOPE_IN_E, weighted=True)
    assert np.array_equal(cut(res, 0), osd)


@pytest.mark.parametrize("world,fixed,split", [(1, None, -1.0), (2, None, -1.0), (2, 0, -1.0), (4, None, -1.0),
                                               (4, 0, -1.0), (1, None, 0.0), (2, None, 0.3), (4, 0, 0.3),
                                               (4, None, 0.0)])
def test_native_msbfs_driver(world, fixed, split):
    """tgo_part_msbfs_run: the partitioned multi-source sweep as ONE native call (C++ level
    loop, collectives through an in-process exchange group of thread ranks on this device):
    every seed's levels equal the oracle's, reached counts global, and the result equals the
    Python driver's.  fixed=0 forces the sized-pairs exchange on every sparse level; split sets
    the source-split budget (tgo_set_tuning; -1 the default, 0 no split, 0.3 a forced split)."""
    from titan_amd.distributed import NativeExchange, distributed_msbfs_native
    scale = 12
    n = 1 << scale
    src, dst, _ = rmat_edges(scale, 16, seed=33)
    ranks = Ranks(world, n, src, dst, L.SCOPE_BOTH_E, layout=True, device_counts=True)
    for be in ranks.backends:
        be.e.set_tuning(L.TUNE_MS_SPLIT, split)
    og = fr.OracleGraph.from_edges(n, src, dst)
    ids = (np.arange(n, dtype=np.int64) + 1) << 3
    rng = np.random.default_rng(9)
    seeds = [int(s) for s in rng.choice(n, 63, replace=False)] + [int(src[0])]
    xs = NativeExchange.local_group(world)

    def body(be, comm):
        r, e, lv = distributed_msbfs_native(be, seeds, n, xs[comm.rank], fixed_exchange_bytes=fixed)
        return r, e, lv, [be.ms_levels(i) for i in range(len(seeds))]
    res = ranks.run(body)
    for i, s in enumerate(seeds):
        od, _ = og.shortest_distance(int(ids[s]), n, 2)
        assert np.array_equal(np.concatenate([x[3][i] for x in res]), od), i
        assert all(x[0][i] == int((od != ABSENT).sum()) for x in res)
    assert len({x[2] for x in res}) == 1
    # the Python driver on the same partitions gives the same counts and levels
    py = ranks.run(lambda be, comm: distributed_msbfs(be, seeds, n, comm=comm, fixed_exchange_bytes=fixed))
    assert all(np.array_equal(a[0], b[0]) and np.array_equal(a[1], b[1]) for a, b in zip(res, py))
    # device counts of the Python driver's backends were restored by the native call
    res2 = ranks.run(body)
    assert all(np.array_equal(a[0], b[0]) for a, b in zip(res, res2))
    # dense levels refresh only the ghost masks by default (TGO_TUNE_MS_GHOST); the all-gather
    # of every rank's masks gives the same sweep
    for be in ranks.backends:
        be.e.set_tuning(L.TUNE_MS_GHOST, 0)
    res3 = ranks.run(body)
    assert all(np.array_equal(a[0], b[0]) and all(np.array_equal(p, q) for p, q in zip(a[3], b[3]))
               for a, b in zip(res, res3))
    for be in ranks.backends:
        be.e.set_tuning(L.TUNE_MS_GHOST, 1)


def test_native_msbfs_rccl_world1():
    """The RCCL exchange (one rank): unique id shared over the driver's communicator, the
    sweep through ncclAllGather / ncclAllToAll paths, equal to the oracle."""
    from titan_amd.distributed import NativeExchange, distributed_msbfs_native
    scale = 11
    n = 1 << scale
    src, dst, _ = rmat_edges(scale, 16, seed=35)
    st = torch.cuda.Stream()
    with torch.cuda.stream(st):
        be = HipPartBackend(Engine(stream=st.cuda_stream).load_partition(n, 0, n, src, dst, L.SCOPE_BOTH_E,
                                                                         apply_cap=False), n, 0, n)
        x = NativeExchange.rccl(0, comm=InProcessGroup(1).comm(0))
        seeds = [int(src[0]), int(dst[1]), int(src[7])]
        r, e, lv = distributed_msbfs_native(be, seeds, n, x)
        og = fr.OracleGraph.from_edges(n, src, dst)
        ids = (np.arange(n, dtype=np.int64) + 1) << 3
        for i, s in enumerate(seeds):
            od, _ = og.shortest_distance(int(ids[s]), n, 2)
            assert np.array_equal(be.ms_levels(i), od)
            assert r[i] == int((od != ABSENT).sum())
        del x


def test_native_msbfs_rejects_a_mismatched_exchange():
    from titan_amd.distributed import NativeExchange, distributed_msbfs_native
    scale = 10
    n = 1 << scale
    src, dst, _ = rmat_edges(scale, 16, seed=3)
    st = torch.cuda.Stream()
    with torch.cuda.stream(st):
        be = HipPartBackend(Engine(stream=st.cuda_stream).load_partition(n, 0, n, src, dst, L.SCOPE_BOTH_E,
                                                                         apply_cap=False), n, 0, n)
        xs = NativeExchange.local_group(2)          # world 2 against a one-rank partition
        with pytest.raises(TitanException):
            distributed_msbfs_native(be, [int(src[0])], n, xs[0])


@pytest.mark.parametrize("world", [1, 2, 4])
def test_native_bfs_sssp_pagerank_drivers(world, monkeypatch):
    """tgo_part_bfs_run / tgo_part_sssp_run / tgo_part_pagerank_run: each partitioned program
    as ONE native call over an in-process exchange group — BFS and capped weighted SSSP
    bit-exact against the oracle and equal to the Python drivers, capped cache-blocked
    PageRank within 1e-6 L1 of the oracle and bitwise equal across the all-gather and the
    ghost exchange (which moves fewer bytes whenever there is more than one rank)."""
    from titan_amd.distributed import (NativeExchange, PR_EXCHANGE_ALLGATHER, PR_EXCHANGE_GHOST, distributed_bfs_native,
                                       distributed_pagerank_native, distributed_sssp_native)
    monkeypatch.setenv("TGO_PR_HOT", "512")
    monkeypatch.setenv("TGO_PR_SEG", "256")
    scale = 12
    n = 1 << scale
    src, dst, w = rmat_edges(scale, 16, seed=57, weights=True)
    ids = (np.arange(n, dtype=np.int64) + 1) << 3
    og = fr.OracleGraph.from_edges(n, src, dst)
    seeds = [int(src[0]), int(dst[5]), int(src[900])]
    bfs = Ranks(world, n, src, dst, L.SCOPE_BOTH_E, layout=True, device_counts=True)
    xs = NativeExchange.local_group(world)
    for seed in seeds:
        od, _ = og.shortest_distance(int(ids[seed]), n, 2)
        for alpha in (15.0, 1e9):
            res = bfs.run(lambda be, comm: distributed_bfs_native(be, seed, n, xs[comm.rank], alpha=alpha))
            assert np.array_equal(np.concatenate([x[0] for x in res]), od), (seed, alpha)
            assert all(x[1][0] == int((od != ABSENT).sum()) for x in res)
            py = bfs.run(lambda be, comm: distributed_bfs(be, seed, n, alpha=alpha, comm=comm))
            assert res[0][2] == py[0][2]                      # same levels
    limit = 40
    sp = Ranks(world, n, src, dst, L.SCOPE_IN_E, weight=w, layout=True, apply_cap=True, hard_limit=limit)
    ogc = fr.OracleGraph.from_edges(n, src, dst, w, hard_limit=limit)
    for seed in seeds:
        od, _ = ogc.shortest_distance(int(ids[seed]), n, L.SCOPE_IN_E, weighted=True)
        res = sp.run(lambda be, comm: distributed_sssp_native(be, seed, xs[comm.rank]))
        assert np.array_equal(np.concatenate([x[0] for x in res]), od), seed
        assert all(x[1][0] == int((od != ABSENT).sum()) for x in res)
        assert len({x[2] for x in res}) == 1 and res[0][2] > 0   # every rank ran the same phases
        # (the phase count itself may differ run to run: atomicMin races decide whether an
        # improvement lands in this phase or the next — the converged distances do not)
    pr = Ranks(world, n, src, dst, L.SCOPE_IN_E, layout=True, apply_cap=True, hard_limit=limit)
    opr, _ = fr.OracleGraph.from_edges(n, src, dst, hard_limit=limit).pagerank(0.85, n, 15)
    fin = np.isfinite(opr)
    got = {}
    for mode in (PR_EXCHANGE_ALLGATHER, PR_EXCHANGE_GHOST):
        res = pr.run(lambda be, comm: distributed_pagerank_native(be, 0.85, n, 15, xs[comm.rank], mode=mode))
        got[mode] = (np.concatenate([x[0] for x in res]), sum(x[1] for x in res))
        assert np.array_equal(np.isfinite(got[mode][0]), fin)
        assert np.abs(got[mode][0][fin] - opr[fin]).sum() <= 1e-6
    assert np.array_equal(got[0][0], got[1][0])
    if world > 1:
        assert 0 < got[PR_EXCHANGE_GHOST][1] < got[PR_EXCHANGE_ALLGATHER][1]
    py = pr.run(lambda be, comm: distributed_pagerank(be, 0.85, n, 15, comm=comm))
    assert np.array_equal(np.concatenate(py), got[0][0])


@pytest.mark.parametrize("world", [1, 2, 3])
def test_partitioned_pagerank_out_of_range_reruns_plain(world, monkeypatch):
    """The blocked layout's fixed-point passes flag a message outside their exact range (spmv.hip
    FxGuard); every rank then re-runs the program on the plain layout (all-reduced flag), in the
    native loop (both exchanges) and the Python driver.  vertexCount = 0 makes every rank +inf
    (Java 1/0), 2^60 puts every contribution below the 2^-53 floor; N = n stays blocked."""
    from titan_amd.distributed import (NativeExchange, PR_EXCHANGE_ALLGATHER, PR_EXCHANGE_GHOST,
                                       distributed_pagerank_native)
    monkeypatch.setenv("TGO_PR_HOT", "512")
    monkeypatch.setenv("TGO_PR_SEG", "256")
    scale = 11
    n = 1 << scale
    if world == 3:
        n = 3 * 704
    src, dst, _ = rmat_edges(scale, 16, seed=61)
    og = fr.OracleGraph.from_edges(n, src, dst)
    ranks = Ranks(world, n, src, dst, L.SCOPE_IN_E, layout=True)
    xs = NativeExchange.local_group(world)
    for N in (0, 1 << 60, n):
        opr, _ = og.pagerank(0.85, N, 7)
        fin = np.isfinite(opr)
        for mode in (PR_EXCHANGE_ALLGATHER, PR_EXCHANGE_GHOST):
            res = ranks.run(lambda be, comm: distributed_pagerank_native(be, 0.85, N, 7, xs[comm.rank], mode=mode))
            pr = np.concatenate([x[0] for x in res])
            assert np.array_equal(np.isposinf(pr), np.isposinf(opr)) and np.array_equal(np.isnan(pr), np.isnan(opr))
            assert np.allclose(pr[fin], opr[fin], rtol=1e-9, atol=0) and np.abs(pr[fin] - opr[fin]).sum() <= 1e-6
            assert {be.e.stats()["exact_reruns"] for be in ranks.backends} == ({0} if N == n else {1})
        py = np.concatenate(ranks.run(lambda be, comm: distributed_pagerank(be, 0.85, N, 7, comm=comm)))
        assert np.array_equal(np.isposinf(py), np.isposinf(opr))
        assert np.allclose(py[fin], opr[fin], rtol=1e-9, atol=0)
        assert {be.e.stats()["exact_reruns"] for be in ranks.backends} == ({0} if N == n else {1})


def test_sssp_negative_weight_fails_every_rank():
    """a negative weight held by ONE rank failed only that rank's tgo_part_sssp_begin
    while its peers waited in the first collective.  The drivers now agree on the global minimum
    weight first (tgo_part_weight_min, all-reduce MIN): every rank raises, native and Python."""
    from titan_amd.distributed import NativeExchange, distributed_sssp_native
    scale = 10
    n = 1 << scale
    src, dst, w = rmat_edges(scale, 16, seed=63, weights=True)
    w = w.copy()
    i = int(np.nonzero((src >= n // 2) & (dst >= n // 2))[0][0])   # an edge only rank 1 holds
    w[i] = -2
    ranks = Ranks(2, n, src, dst, L.SCOPE_IN_E, weight=w)
    assert ranks.backends[0].weight_min() >= 0 and ranks.backends[1].weight_min() == -2
    xs = NativeExchange.local_group(2)

    def body(run):
        def f(be, comm):
            try:
                run(be, comm)
                return "ran"
            except TitanException as e:
                return e.code
        return f
    assert ranks.run(body(lambda be, comm: distributed_sssp_native(be, int(src[0]), xs[comm.rank]))) == [L.TGO_E_INVALID] * 2
    assert ranks.run(body(lambda be, comm: distributed_sssp(be, int(src[0]), 0, comm=comm))) == [L.TGO_E_INVALID] * 2


def test_native_drivers_rccl_world1():
    """The three native loops over the RCCL exchange (one rank)."""
    from titan_amd.distributed import (NativeExchange, distributed_bfs_native, distributed_pagerank_native,
                                       distributed_sssp_native)
    scale = 11
    n = 1 << scale
    src, dst, w = rmat_edges(scale, 16, seed=59, weights=True)
    ids = (np.arange(n, dtype=np.int64) + 1) << 3
    st = torch.cuda.Stream()
    with torch.cuda.stream(st):
        x = NativeExchange.rccl(0, comm=InProcessGroup(1).comm(0))
        be = HipPartBackend(Engine(stream=st.cuda_stream).load_partition(n, 0, n, src, dst, L.SCOPE_BOTH_E,
                                                                         apply_cap=False), n, 0, n)
        og = fr.OracleGraph.from_edges(n, src, dst, w)
        seed = int(src[0])
        d, r, _ = distributed_bfs_native(be, seed, n, x)
        od, _ = og.shortest_distance(int(ids[seed]), n, 2)
        assert np.array_equal(d, od) and r[0] == int((od != ABSENT).sum())
        wb = HipPartBackend(Engine(stream=st.cuda_stream).load_partition(n, 0, n, src, dst, L.SCOPE_IN_E, weight=w,
                                                                         apply_cap=False), n, 0, n)
        d, r, _ = distributed_sssp_native(wb, seed, x)
        od, _ = og.shortest_distance(int(ids[seed]), n, L.SCOPE_IN_E, weighted=True)
        assert np.array_equal(d, od)
        p, _ = distributed_pagerank_native(wb, 0.85, n, 10, x)
        opr, _ = og.pagerank(0.85, n, 10)
        fin = np.isfinite(opr)
        assert np.abs(p[fin] - opr[fin]).sum() <= 1e-6
        del x


# ----------------------------------------------------------------------------- partition from rows
class RowRanks:
    """tgo_load_partition_rows: each thread rank loads ITS contiguous row range of a scan
    (balanced_row_ranges) over an in-process exchange group; backends over the slot ids."""

    def __init__(self, world, rows, sd, scope, limit, weight_key=0, layout=True, labels=(), batch_rows=None):
        from titan_amd import Schema
        from titan_amd.distributed import NativeExchange, balanced_row_ranges
        self.world = world
        self.ranges = balanced_row_ranges(rows.entry_begin, world)
        self.xs = NativeExchange.local_group(world)
        self.streams = [torch.cuda.Stream() for _ in range(world)]

        def load(rank, comm):
            torch.cuda.set_stream(self.streams[rank])
            eng = Engine(stream=self.streams[rank].cuda_stream, hard_query_limit=limit)
            live, S, total = eng.load_partition_rows(self.xs[rank], rows.slice(*self.ranges[rank]), Schema.from_dict(sd),
                                                     scope, weight_key=weight_key, layout=layout, labels=labels,
                                                     batch_rows=batch_rows)
            return eng, live, S, total
        res = InProcessGroup(world).run(load)
        self.S = res[0][2]
        assert all(r[2] == self.S for r in res)
        self.n_global = world * self.S
        self.live = [r[1] for r in res]
        assert all(r[3] == sum(self.live) for r in res)
        self.engines = [r[0] for r in res]
        self.backends = []
        for r, e in enumerate(self.engines):
            with torch.cuda.stream(self.streams[r]):
                self.backends.append(HipPartBackend(e, self.n_global, r * self.S, (r + 1) * self.S))
        self.ids = [e.vertex_ids()[:lv] for e, lv in zip(self.engines, self.live)]
        self.slot = {int(v): r * self.S + i for r, ids in enumerate(self.ids) for i, v in enumerate(ids)}

    def run(self, fn):
        def body(rank, comm):
            torch.cuda.set_stream(self.streams[rank])
            return fn(self.backends[rank], comm, self.xs[rank])
        return InProcessGroup(self.world).run(body)

    def gather(self, per_rank, ids_to):
        """Concatenate the ranks' live results and order them as ids_to."""
        got = {}
        for ids, vals, lv in zip(self.ids, per_rank, self.live):
            got.update(zip((int(v) for v in ids), vals[:lv]))
        return np.array([got[int(v)] for v in ids_to])


@pytest.mark.parametrize("world", [1, 2, 3, 4, 8])
def test_partition_rows_match_one_gpu_rows(world, monkeypatch):
    """tgo_load_partition_rows on two-label rows whose hubs are cut in column
    order at a small hard limit: every native partitioned program over the row-range partition
    equals the one-GPU tgo_load_rows load of the same rows — BFS (bothE), multi-source BFS and
    weighted delta SSSP (capped inE: the push rows come from every rank's cut pull lists) bit-exact,
    equal summed truncated_results, both loads equal to the oracle."""
    from titan_amd import Schema
    from titan_amd.distributed import distributed_bfs_native, distributed_msbfs_native, distributed_sssp_native
    from test_gpu_parity import two_label_rows
    rows, vids, sd, osch, knows, likes, wkey = two_label_rows(n=900)
    limit, n = 12, len(vids)
    for scope in (L.SCOPE_BOTH_E, L.SCOPE_IN_E):
        one = Engine(hard_query_limit=limit).load_rows(rows, Schema.from_dict(sd), scope, weight_key=wkey)
        o = fr.OracleGraph.from_rows(rows, osch, scope, hard_limit=limit, weight_key=wkey)
        ids1 = one.vertex_ids()
        rr = RowRanks(world, rows, sd, scope, limit, weight_key=wkey, batch_rows=64 if world % 2 else None)
        assert sum(rr.live) == len(ids1) and sorted(np.concatenate(rr.ids)) == sorted(ids1)
        assert sum(be.e.stats()["truncated_results"] for be in rr.backends) == one.stats()["truncated_results"] \
            == o.stats.truncated_results
        if scope == L.SCOPE_IN_E:
            assert one.stats()["truncated_results"] > 0
        seeds = [int(vids[i]) for i in (0, 1, 5, 77)]
        for s in seeds:
            if scope == L.SCOPE_BOTH_E:
                want = one.bfs(s, n, scope)
                assert np.array_equal(want, o.shortest_distance(s, n, scope)[0])
                res = rr.run(lambda be, comm, x: distributed_bfs_native(be, rr.slot[s], rr.n_global, x))
            else:
                want = one.sssp(s, n, scope, mode=L.SSSP_DELTA)
                assert np.array_equal(want, o.shortest_distance(s, n, scope, weighted=True)[0])
                res = rr.run(lambda be, comm, x: distributed_sssp_native(be, rr.slot[s], x))
            assert np.array_equal(rr.gather([r[0] for r in res], ids1), want), (scope, s)
        if scope == L.SCOPE_BOTH_E:
            res = rr.run(lambda be, comm, x: (distributed_msbfs_native(be, [rr.slot[s] for s in seeds], rr.n_global, x),
                                              [be.ms_levels(i) for i in range(len(seeds))]))
            for i, s in enumerate(seeds):
                assert np.array_equal(rr.gather([r[1][i] for r in res], ids1), one.bfs(s, n, scope)), i


@pytest.mark.parametrize("world", [1, 2, 4, 8])
def test_partition_rows_pagerank_zero_edge_count(world, monkeypatch):
    """PageRank over the row-range partition of the zero-edgeCount fixture (hubs whose cut rows
    keep no OUT entry while their targets read them): the blocked layout's fixed-point passes
    flag the +inf, every rank re-runs on the plain layout, and the ranks equal the one-GPU
    tgo_load_rows result and the oracle (same +inf positions, finite part within 1e-6 L1), for
    both exchanges."""
    from titan_amd import Schema
    from titan_amd.distributed import PR_EXCHANGE_ALLGATHER, PR_EXCHANGE_GHOST, distributed_pagerank_native
    from test_gpu_parity import assert_pagerank_like_oracle, zero_edge_count_rows
    monkeypatch.setenv("TGO_PR_HOT", "128")
    monkeypatch.setenv("TGO_PR_SEG", "128")
    rows, vids, sd, osch = zero_edge_count_rows()
    limit, n = 24, len(vids)
    one = Engine(hard_query_limit=limit).load_rows(rows, Schema.from_dict(sd), L.SCOPE_IN_E)
    ids1 = one.vertex_ids()
    opr = fr.OracleGraph.from_rows(rows, osch, L.SCOPE_IN_E, hard_limit=limit).pagerank(0.85, n, 8)[0]
    want = one.pagerank(0.85, n, 8)
    assert_pagerank_like_oracle(want, opr)
    rr = RowRanks(world, rows, sd, L.SCOPE_IN_E, limit)
    for mode in (PR_EXCHANGE_ALLGATHER, PR_EXCHANGE_GHOST):
        res = rr.run(lambda be, comm, x: distributed_pagerank_native(be, 0.85, n, 8, x, mode=mode))
        got = rr.gather([r[0] for r in res], ids1)
        assert_pagerank_like_oracle(got, opr)
        fin = np.isfinite(want)
        assert np.abs(got[fin] - want[fin]).sum() <= 1e-9
        assert {be.e.stats()["exact_reruns"] for be in rr.backends} == {1}


def test_partition_rows_refuses_vertex_cuts_on_every_rank():
    """Vertex cuts fold into their canonical vertex on one GPU only: the partitioned rows load
    fails with TGO_E_UNSUPPORTED on every rank (agreed before any further collective)."""
    from titan_amd import Schema
    from conftest import load_fixture
    rows, vids, sd, npz = load_fixture("partition_groups")
    with pytest.raises(TitanException) as ei:
        RowRanks(2, rows, sd, L.SCOPE_IN_E, 100000)
    assert ei.value.code in (L.TGO_E_UNSUPPORTED, L.TGO_E_INVALID)

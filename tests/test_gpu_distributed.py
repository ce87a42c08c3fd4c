"""GPU: the partitioned (multi-GPU) local steps of the HIP engine, driven by the same
exchange driver as the real multi-GPU run.  The 1-GPU box has one device, so the ranks
are simulated in ONE process: every "rank" is an Engine holding its partition, and a
tiny in-process communicator performs the all-to-all / all-gather / all-reduce with
torch ops on the device.  Results must equal the oracle bit-for-bit (BFS) / 1e-6 L1 (PR).
"""
import numpy as np
import pytest
import torch

import fulgora as fr
from titan_amd import Engine, rmat_edges
from titan_amd import _lib as L
from titan_amd.distributed import HipPartBackend, exchange_stream, local_layout, partition_range

pytestmark = pytest.mark.gpu
ABSENT = L.DIST_ABSENT


def run_bfs(backends, seed, max_depth, alpha=15.0, beta=18.0):
    """The distributed_bfs protocol with the collectives done in-process."""
    world = len(backends)
    n = backends[0].n_global
    nwl = backends[0].n_local // 64
    dev = backends[0].device
    fb = [b.tensor(n // 64, torch.int64) for b in backends]
    nb = [b.tensor(nwl, torch.int64) for b in backends]
    disc = [b.tensor(n // 64, torch.int64) for b in backends]
    recv = [b.tensor(n // 64, torch.int64) for b in backends]

    def allgather():
        g = torch.cat(nb)
        for t in fb:
            t.copy_(g)

    total = sum(b.total_entries for b in backends)
    c = sum(b.bfs_begin(seed, nb[i]) for i, b in enumerate(backends))
    allgather()
    nf, mf = c
    mu = total - mf
    bottom_up = False
    for level in range(max_depth):
        if nf == 0:
            break
        if not bottom_up and mf > mu / alpha:
            bottom_up = True
        elif bottom_up and nf < n / beta:
            bottom_up = False
        cs = []
        if bottom_up:
            for i, b in enumerate(backends):
                cs.append(b.bfs_bu(level, fb[i], nb[i]))
        else:
            for i, b in enumerate(backends):
                disc[i].zero_()
                b.bfs_td(level, disc[i])
            torch.cuda.synchronize()
            for r in range(world):          # all_to_all_single: slice r of every sender -> rank r
                recv[r].copy_(torch.cat([disc[s][r * nwl:(r + 1) * nwl] for s in range(world)]))
            for i, b in enumerate(backends):
                cs.append(b.bfs_claim(level, recv[i], world, nb[i]))
        allgather()
        nf, mf = sum(cs)
        mu -= mf
    outs = [b.bfs_end(True) for b in backends]
    return np.concatenate([o[0] for o in outs]), sum(o[1] for o in outs)


def run_msbfs(backends, seeds, max_depth, ms_alpha=12.0, sparse=False):
    """The distributed_msbfs protocol with the collectives done in-process (sparse: the
    packed-pair exchange of the sparse levels, tgo_part_ms_pack / ms_settle_pairs)."""
    world = len(backends)
    n = backends[0].n_global
    nl = backends[0].n_local
    fr_ = [b.tensor(nl, torch.int64) for b in backends]
    frn = [b.tensor(nl, torch.int64) for b in backends]
    fg = [b.tensor(n, torch.int64) for b in backends]
    cand = [b.tensor(n, torch.int64) for b in backends]
    recv = [b.tensor(2 * n + 2 * world if sparse else n, torch.int64) for b in backends]
    send = [b.tensor(2 * n + 2 * world, torch.int64) for b in backends] if sparse else None
    total = sum(b.total_entries for b in backends)
    nf, mf = sum(b.ms_begin(seeds, fr_[i]) for i, b in enumerate(backends))
    for level in range(max_depth):
        if nf == 0:
            break
        cs = []
        if mf * ms_alpha > total:
            torch.cuda.synchronize()
            g = torch.cat(fr_)
            for t in fg:
                t.copy_(g)
            torch.cuda.synchronize()
            for i, b in enumerate(backends):
                cs.append(b.ms_pull(level, fg[i], frn[i]))
        elif sparse == "fixed":         # tgo_part_ms_pack_fixed / ms_settle_fixed, equal splits
            cap = int(min(mf, nl))
            slot = 2 * (cap + 1)
            for i, b in enumerate(backends):
                b.ms_push(level, fr_[i], cand[i])
                b.ms_pack_fixed(cand[i], send[i], world, cap)
                assert int(torch.count_nonzero(cand[i])) == 0
            torch.cuda.synchronize()
            for r in range(world):      # all_to_all with equal splits: sender s's slot for rank r
                recv[r][:world * slot].copy_(torch.cat([send[s][r * slot:(r + 1) * slot] for s in range(world)]))
            torch.cuda.synchronize()
            for i, b in enumerate(backends):
                cs.append(b.ms_settle_fixed(level, recv[i], world, cap, frn[i]))
        elif sparse:
            counts = []
            for i, b in enumerate(backends):
                b.ms_push(level, fr_[i], cand[i])
                counts.append(b.ms_pack(cand[i], send[i], world))
                assert int(torch.count_nonzero(cand[i])) == 0        # pack clears what it packs
            torch.cuda.synchronize()
            offs = [np.concatenate([[0], np.cumsum(c)]) for c in counts]
            for r in range(world):      # all_to_all with split sizes: sender s's run for rank r
                parts = [send[s][2 * offs[s][r]:2 * offs[s][r + 1]] for s in range(world)]
                got = torch.cat(parts)
                recv[r][:got.numel()].copy_(got)
            torch.cuda.synchronize()
            for i, b in enumerate(backends):
                cs.append(b.ms_settle_pairs(level, recv[i], [counts[s][i] for s in range(world)], frn[i]))
        else:
            for i, b in enumerate(backends):
                cand[i].zero_()
                b.ms_push(level, fr_[i], cand[i])
            torch.cuda.synchronize()
            for r in range(world):
                recv[r].copy_(torch.cat([cand[s][r * nl:(r + 1) * nl] for s in range(world)]))
            torch.cuda.synchronize()
            for i, b in enumerate(backends):
                cs.append(b.ms_settle(level, recv[i], world, frn[i]))
        fr_, frn = frn, fr_
        nf, mf = sum(cs)
    ends = [b.ms_end(len(seeds)) for b in backends]
    reached = sum(e[0] for e in ends)
    levels = [np.concatenate([b.ms_levels(s) for b in backends]) for s in range(len(seeds))]
    return levels, reached


INT64_MAX = (1 << 63) - 1


def run_sssp(backends, seed, delta):
    """The distributed_sssp protocol with the collectives done in-process."""
    world = len(backends)
    n = backends[0].n_global
    send = [b.tensor(2 * n, torch.int64) for b in backends]
    recv = [b.tensor(2 * n, torch.int64) for b in backends]
    st = [b.sssp_begin(seed, delta) for b in backends]
    if delta <= 0:
        delta = max(int(s[1]) for s in st)
    q = [int(s[0]) for s in st]
    thr = delta
    while True:
        if sum(q) == 0:
            mn = min(int(b.sssp_pending_min()[0]) for b in backends)
            if mn == INT64_MAX:
                break
            if mn >= thr:
                thr = (mn // delta + 1) * delta
            q = [int(b.sssp_extract(thr)[0]) for b in backends]
            continue
        sc = [b.sssp_relax(thr, send[i], world) for i, b in enumerate(backends)]
        torch.cuda.synchronize()
        npairs = []
        for r in range(world):            # all_to_all_single: rank s's block r -> rank r
            parts = [send[s][2 * int(sc[s][:r].sum()): 2 * int(sc[s][:r + 1].sum())] for s in range(world)]
            cat = torch.cat(parts)
            recv[r][:cat.numel()].copy_(cat)
            npairs.append(cat.numel() // 2)
        torch.cuda.synchronize()
        q = [int(b.sssp_apply(thr, recv[r], npairs[r])[0]) for r, b in enumerate(backends)]
    outs = [b.sssp_end(True) for b in backends]
    return np.concatenate([o[0] for o in outs]), sum(o[1] for o in outs)


def make_backends(world, n, src, dst, scope, weight=None, layout=False):
    """One Engine per simulated rank; layout=True loads every rank with the all-gathered
    degree-grouped layout (tgo_part_layout), as bench.py does."""
    lay = None
    if layout:
        lay = np.concatenate([local_layout(src, dst, n, *partition_range(n, world, r)) for r in range(world)])
        assert np.array_equal(np.sort(lay), np.arange(n))
    backends = []
    for r in range(world):
        lo, hi = partition_range(n, world, r)
        eng = Engine(stream=exchange_stream()).load_partition(
            n, lo, hi, src, dst, scope, weight=weight, apply_cap=False, layout=lay)
        backends.append(HipPartBackend(eng, n, lo, hi))
    return backends


@pytest.mark.parametrize("layout", [False, True])
@pytest.mark.parametrize("world,scope", [(2, L.SCOPE_IN_E), (4, L.SCOPE_OUT_E), (4, L.SCOPE_BOTH_E)])
def test_partitioned_delta_stepping(world, scope, layout):
    scale = 12
    n = 1 << scale
    src, dst, w = rmat_edges(scale, 16, seed=35, weights=True)
    backends = make_backends(world, n, src, dst, scope, weight=w, layout=layout)
    og = fr.OracleGraph.from_edges(n, src, dst, w)
    ids = (np.arange(n, dtype=np.int64) + 1) << 3
    for seed in (int(src[0]), int(dst[9])):
        od, _ = og.shortest_distance(int(ids[seed]), n, scope, weighted=True)
        for delta in (0, 1, 1 << 40):
            d, reached = run_sssp(backends, seed, delta)
            assert np.array_equal(d, od), (seed, delta)
            assert reached[0] == int((od != ABSENT).sum())


@pytest.mark.parametrize("layout", [False, True])
@pytest.mark.parametrize("world", [2, 4])
def test_partitioned_multi_source_bfs(world, layout):
    scale = 12
    n = 1 << scale
    src, dst, _ = rmat_edges(scale, 16, seed=33)
    backends = make_backends(world, n, src, dst, L.SCOPE_BOTH_E, layout=layout)
    og = fr.OracleGraph.from_edges(n, src, dst)
    ids = (np.arange(n, dtype=np.int64) + 1) << 3
    rng = np.random.default_rng(5)
    seeds = [int(s) for s in rng.choice(n, 40, replace=False)] + [int(src[0])]
    expect = [og.shortest_distance(int(ids[s]), n, 2)[0] for s in seeds]
    for ms_alpha, sparse in ((12.0, False), (12.0, True), (12.0, "fixed"), (1e9, False), (1e9, True), (1e9, "fixed"),
                             (1e-9, False)):
        levels, reached = run_msbfs(backends, seeds, n, ms_alpha, sparse)
        for i, od in enumerate(expect):
            assert np.array_equal(levels[i], od), (ms_alpha, i)
            assert reached[i] == int((od != ABSENT).sum())


@pytest.mark.parametrize("layout", [False, True])
@pytest.mark.parametrize("world", [2, 4])
def test_partitioned_bfs_and_pagerank(world, layout):
    scale = 12
    n = 1 << scale
    src, dst, _ = rmat_edges(scale, 16, seed=31)
    backends = make_backends(world, n, src, dst, L.SCOPE_BOTH_E, layout=layout)
    og = fr.OracleGraph.from_edges(n, src, dst)
    ids = (np.arange(n, dtype=np.int64) + 1) << 3
    for seed in (int(src[0]), int(dst[9]), int(src[100])):
        for alpha in (15.0, 1e9):
            d, reached = run_bfs(backends, seed, n, alpha=alpha)
            od, _ = og.shortest_distance(int(ids[seed]), n, 2)
            assert np.array_equal(d, od)
            assert reached[0] == int((od != ABSENT).sum())
    # PageRank: in-process all-gather of the contributions
    iters = 10
    cl = [b.tensor(b.n_local, torch.float64) for b in backends]
    cg = [b.tensor(n, torch.float64) for b in backends]
    for b, c in zip(backends, cl):
        b.pr_begin(0.85, n, iters, c)
    for _ in range(2, iters + 1):
        torch.cuda.synchronize()
        g = torch.cat(cl)
        for t in cg:
            t.copy_(g)
        torch.cuda.synchronize()
        for b, c, gg in zip(backends, cl, cg):
            b.pr_step(gg, c)
    pr = np.concatenate([b.pr_end(True) for b in backends])
    opr, _ = og.pagerank(0.85, n, iters)
    fin = np.isfinite(opr)
    assert np.array_equal(np.isfinite(pr), fin)
    assert np.abs(pr[fin] - opr[fin]).sum() <= 1e-6


def run_pagerank_blocked(backends, n, iters):
    """distributed_pagerank's blocked protocol in-process: agree on the active span, build
    the hot-first gathered layout, cold slices gathered before step_cold, hot slices before
    step_hot."""
    world = len(backends)
    span = max(b.active_rows() for b in backends)
    hots = {b.pr_layout(world, span) for b in backends}
    assert len(hots) == 1
    hot = hots.pop()
    cl = [b.tensor(b.n_local, torch.float64) for b in backends]
    cg = [b.tensor(world * span, torch.float64) for b in backends]
    for b, c in zip(backends, cl):
        b.pr_begin(0.85, n, iters, c)
    for _ in range(2, iters + 1):
        torch.cuda.synchronize()
        cold = torch.cat([c[hot:span] for c in cl])
        for t in cg:
            t[world * hot:].copy_(cold)
            t[:world * hot].fill_(float("nan"))          # the hot gather is still in flight
        torch.cuda.synchronize()
        for b, gg in zip(backends, cg):
            b.pr_step_cold(gg)
        torch.cuda.synchronize()
        hotv = torch.cat([c[:hot] for c in cl])
        for t in cg:
            t[:world * hot].copy_(hotv)
        torch.cuda.synchronize()
        for b, c, gg in zip(backends, cl, cg):
            b.pr_step_hot(gg, c)
    return hot, span, np.concatenate([b.pr_end(True) for b in backends])


@pytest.mark.parametrize("layout", [False, True])
@pytest.mark.parametrize("world", [1, 2, 4])
def test_partitioned_pagerank_cache_blocked(world, layout, monkeypatch):
    """tgo_part_pr_blocked: the owned in-lists re-expressed in the hot-first gathered index
    space and cache-blocked (small hot set / segments so every rank has hot rows, cold
    pieces in several segments and entry-less rows past the span)."""
    monkeypatch.setenv("TGO_PR_HOT", "512")
    monkeypatch.setenv("TGO_PR_SEG", "256")
    scale = 12
    n = 1 << scale
    src, dst, _ = rmat_edges(scale, 16, seed=37)
    backends = make_backends(world, n, src, dst, L.SCOPE_IN_E, layout=layout)
    og = fr.OracleGraph.from_edges(n, src, dst)
    for iters in (2, 10):
        hot, span, pr = run_pagerank_blocked(backends, n, iters)
        assert hot == max(64, 512 // world // 64 * 64)
        if layout:
            assert span < n // world                    # entry-less rows are not exchanged
        opr, _ = og.pagerank(0.85, n, iters)
        fin = np.isfinite(opr)
        assert np.array_equal(np.isfinite(pr), fin)
        assert np.abs(pr[fin] - opr[fin]).sum() <= 1e-6
    with pytest.raises(Exception):                      # rank property only after the last step
        backends[0].pr_begin(0.85, n, 5, backends[0].tensor(backends[0].n_local, torch.float64))
        backends[0].pr_end(True)


def test_drivers_on_a_real_world1_group(monkeypatch):
    """The real drivers (titan_amd.distributed) on a one-rank RCCL group: device-resident
    level counts (tgo_part_device_counts) for BFS / multi-source BFS, and the cache-blocked
    PageRank exchange with the hot all-gather overlapping the cold phase."""
    import socket
    import torch.distributed as dist
    from titan_amd.distributed import (distributed_bfs, distributed_msbfs, distributed_pagerank, pagerank_layout)
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

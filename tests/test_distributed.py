"""CPU, world_size 2 and 4 over gloo: the multi-GPU exchange protocol of
titan_amd/distributed.py (partitioning, bitmap all-to-all / all-gather, count
all-reduce, direction switching, PageRank contribution all-gather) against the oracle.

The per-rank local steps are a numpy test double with the exact contract of the HIP
backend (include/titan_gpu_olap_part.h); the GPU backend itself is exercised by
tests/test_gpu_distributed.py on the device.
"""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

ABSENT = -(1 << 63)
INF = (1 << 63) - 1


class NumpyPartBackend:
    """Reference implementation of the per-rank local steps (test double)."""

    def __init__(self, n_global, lo, hi, src, dst, w=None, scope=2):
        self.n_global, self.lo, self.hi = n_global, lo, hi
        self.n_local = hi - lo
        self.device = torch.device("cpu")
        self.scope = scope
        w = np.ones(len(src), np.int64) if w is None else w
        own_o = (src >= lo) & (src < hi)
        own_i = (dst >= lo) & (dst < hi)
        self.out = [[] for _ in range(self.n_local)]
        self.inn = [[] for _ in range(self.n_local)]
        self.out_w = [[] for _ in range(self.n_local)]
        self.inn_w = [[] for _ in range(self.n_local)]
        for s, d, x in zip(src[own_o], dst[own_o], w[own_o]):
            self.out[s - lo].append(int(d))
            self.out_w[s - lo].append(int(x))
        for s, d, x in zip(src[own_i], dst[own_i], w[own_i]):
            self.inn[d - lo].append(int(s))
            self.inn_w[d - lo].append(int(x))
        self.total_entries = sum(map(len, self.out)) + sum(map(len, self.inn))

    def _push(self, u):
        """(target, weight) of u's push entries: the reversed scope (outE -> OUT, inE -> IN)."""
        lists = {0: [(self.out, self.out_w)], 1: [(self.inn, self.inn_w)]}.get(self.scope,
                                                                             [(self.out, self.out_w), (self.inn, self.inn_w)])
        return [(t, x) for adj, ww in lists for t, x in zip(adj[u], ww[u])]

    # ---- delta-stepping SSSP local steps (contract: include/titan_gpu_olap_part.h)
    def weight_min(self):
        ws = [x for lst in self.out_w + self.inn_w for x in lst]
        return min(ws) if ws else 0

    def sssp_begin(self, seed, delta):
        self.sd = np.full(self.n_local, INF, np.int64)
        self.pend, self.rbest, self.sq, self.snext = set(), {}, [], []
        if self.lo <= seed < self.hi:
            self.sd[seed - self.lo] = 0
            self.sq = [seed - self.lo]
        return np.array([len(self.sq), delta if delta > 0 else 256])

    def sssp_relax(self, thr, send, nranks):
        msg = {u: int(self.sd[u]) for u in self.sq}
        for u in self.sq:
            self.pend.discard(u)
        self.snext, marked = [], set()
        for u in self.sq:
            if self.sd[u] < msg[u]:
                continue
            for t, x in self._push(u):
                cand = msg[u] + x
                if self.lo <= t < self.hi:
                    self._improve(t - self.lo, cand, thr)
                elif cand < self.rbest.get(t, INF):
                    self.rbest[t] = cand
                    marked.add(t)
        buf = send.numpy()
        counts = np.zeros(nranks, np.int64)
        pos = 0
        for r in range(nranks):
            for t in sorted(x for x in marked if x // self.n_local == r):
                buf[2 * pos], buf[2 * pos + 1] = t - r * self.n_local, self.rbest[t]
                pos += 1
                counts[r] += 1
        return counts

    def _improve(self, v, d, thr):
        if d < self.sd[v]:
            self.sd[v] = d
            if v not in self.pend:
                self.pend.add(v)
                if d < thr:
                    self.snext.append(v)

    def sssp_apply(self, thr, recv, npairs):
        r = recv.numpy()
        for i in range(npairs):
            self._improve(int(r[2 * i]), int(r[2 * i + 1]), thr)
        self.sq = self.snext
        return np.array([len(self.sq), 0])

    def sssp_pending_min(self):
        if not self.pend:
            return np.array([INF, 0])
        return np.array([min(int(self.sd[v]) for v in self.pend), len(self.pend)])

    def sssp_extract(self, thr):
        self.sq = sorted(v for v in self.pend if self.sd[v] < thr)
        self.pend -= set(self.sq)
        return np.array([len(self.sq), 0])

    def sssp_end(self, fetch=True, stats=True):
        d = np.where(self.sd == INF, ABSENT, self.sd)
        return d, np.array([int((self.sd != INF).sum()), 0])

    def tensor(self, n, dtype):
        return torch.zeros(n, dtype=dtype)

    @staticmethod
    def _u(t):
        return t.numpy().view(np.uint64)

    def _deg(self, v):
        return len(self.out[v]) + len(self.inn[v])

    def bfs_begin(self, seed, nb_local):
        self.level = np.full(self.n_local, -1, np.int64)
        self.vis = np.zeros(self.n_local, bool)
        nb = self._u(nb_local)
        nb[:] = 0
        self.queue = []
        if self.lo <= seed < self.hi:
            v = seed - self.lo
            self.level[v] = 0
            self.vis[v] = True
            nb[v >> 6] |= np.uint64(1 << (v & 63))
            self.queue = [v]
            return np.array([1, self._deg(v)])
        return np.array([0, 0])

    def bfs_td(self, level, disc):
        d = self._u(disc)
        for u in self.queue:
            for w in self.out[u] + self.inn[u]:
                if self.lo <= w < self.hi and self.vis[w - self.lo]:
                    continue
                d[w >> 6] |= np.uint64(1 << (w & 63))

    def _finish(self, level, fresh, nb_local):
        nb = self._u(nb_local)
        nb[:] = 0
        self.queue = []
        ent = 0
        for v in fresh:
            self.level[v] = level + 1
            self.vis[v] = True
            nb[v >> 6] |= np.uint64(1 << (v & 63))
            self.queue.append(v)
            ent += self._deg(v)
        return np.array([len(fresh), ent])

    def bfs_claim(self, level, recv, nslices, nb_local):
        r = self._u(recv).reshape(nslices, -1)
        bits = np.bitwise_or.reduce(r, axis=0)
        fresh = [v for v in range(self.n_local) if (int(bits[v >> 6]) >> (v & 63)) & 1 and not self.vis[v]]
        return self._finish(level, fresh, nb_local)

    def bfs_bu(self, level, fb_global, nb_local):
        fb = self._u(fb_global)
        fresh = []
        for v in range(self.n_local):
            if self.vis[v]:
                continue
            if any((int(fb[w >> 6]) >> (w & 63)) & 1 for w in self.out[v] + self.inn[v]):
                fresh.append(v)
        return self._finish(level, fresh, nb_local)

    def bfs_end(self, fetch=True, stats=True):
        d = np.where(self.level >= 0, self.level, ABSENT)
        reached = np.array([int((self.level >= 0).sum()), sum(self._deg(v) for v in range(self.n_local) if self.level[v] >= 0)])
        return d, reached

    # ---- multi-source BFS local steps
    def _ms_fresh(self, level, cand, fr_next):
        fn = self._u(fr_next)
        fn[:] = 0
        self.msq = []
        cnt = ent = 0
        for v in range(self.n_local):
            fresh = int(cand[v]) & ~int(self.msvis[v]) & self.full
            if fresh:
                self.msvis[v] = np.uint64(int(self.msvis[v]) | fresh)
                fn[v] = np.uint64(fresh)
                for r in range(self.nseeds):
                    if (fresh >> r) & 1:
                        self.mslvl[v, r] = level + 1
                self.msq.append(v)
                cnt += 1
                ent += self._deg(v)
        return np.array([cnt, ent])

    def ms_begin(self, seeds, fr_local):
        self.nseeds = len(seeds)
        self.full = (1 << self.nseeds) - 1
        self.msvis = np.zeros(self.n_local, np.uint64)
        self.mslvl = np.full((self.n_local, self.nseeds), -1, np.int64)
        fr = self._u(fr_local)
        fr[:] = 0
        self.msq = []
        for r, s in enumerate(seeds):
            if self.lo <= s < self.hi:
                v = s - self.lo
                self.msvis[v] = np.uint64(int(self.msvis[v]) | (1 << r))
                fr[v] = np.uint64(int(fr[v]) | (1 << r))
                self.mslvl[v, r] = 0
                if v not in self.msq:
                    self.msq.append(v)
        return np.array([len(self.msq), sum(self._deg(v) for v in self.msq)])

    def ms_pull(self, level, fr_global, fr_next):
        fg = self._u(fr_global)
        acc = np.zeros(self.n_local, np.uint64)
        for v in range(self.n_local):
            a = 0
            for w in self.out[v] + self.inn[v]:
                a |= int(fg[w])
            acc[v] = np.uint64(a)
        return self._ms_fresh(level, acc, fr_next)

    def ms_push(self, level, fr_local, cand):
        fr = self._u(fr_local)
        c = self._u(cand)
        for u in self.msq:
            for w in self.out[u] + self.inn[u]:
                c[w] = np.uint64(int(c[w]) | int(fr[u]))

    def ms_settle(self, level, recv, nslices, fr_next):
        r = self._u(recv).reshape(nslices, -1)
        return self._ms_fresh(level, np.bitwise_or.reduce(r, axis=0), fr_next)

    def ms_pack_dev(self, cand, send, nranks, send_elems):
        """tgo_part_ms_pack_dev: the split sizes (int64 elements) land in a tensor."""
        send_elems.copy_(torch.from_numpy(2 * np.asarray(self.ms_pack(cand, send, nranks), np.int64)))

    def ms_pack(self, cand, send, nranks):
        c = self._u(cand)
        s = send.numpy()
        counts = np.zeros(nranks, np.int64)
        p = 0
        for r in range(nranks):
            sl = c[r * self.n_local:(r + 1) * self.n_local]
            nz = np.nonzero(sl)[0][::-1]            # any order: the receiver ORs the masks
            s[2 * p:2 * (p + len(nz)):2] = nz
            s[2 * p + 1:2 * (p + len(nz)):2] = sl[nz].view(np.int64)
            sl[nz] = 0
            counts[r] = len(nz)
            p += len(nz)
        return counts

    def ms_pack_fixed(self, cand, send, nranks, cap):
        """tgo_part_ms_pack_fixed: owner r's slot = header (count, 0) + up to cap pairs."""
        self.n_fixed = getattr(self, "n_fixed", 0) + 1
        counts = self.ms_pack(cand, self._fixed_tmp(send), nranks)
        tmp = self._fixed_tmp(send).numpy()
        s = send.numpy()
        p = 0
        for r in range(nranks):
            assert counts[r] <= cap                  # the driver's bound: pairs <= frontier entries
            base = 2 * r * (cap + 1)
            s[base], s[base + 1] = counts[r], 0
            s[base + 2:base + 2 + 2 * counts[r]] = tmp[2 * p:2 * (p + counts[r])]
            p += counts[r]

    def _fixed_tmp(self, like):
        if getattr(self, "_ftmp", None) is None or self._ftmp.numel() < like.numel():
            self._ftmp = torch.zeros(like.numel(), dtype=torch.int64)
        return self._ftmp

    def ms_settle_fixed(self, level, recv, nslices, cap, fr_next):
        r = recv.numpy()
        acc = np.zeros(self.n_local, np.uint64)
        for s in range(nslices):
            base = 2 * s * (cap + 1)
            k = int(r[base])
            np.bitwise_or.at(acc, r[base + 2:base + 2 + 2 * k:2], r[base + 3:base + 3 + 2 * k:2].view(np.uint64))
        return self._ms_fresh(level, acc, fr_next)

    def ms_settle_pairs(self, level, recv, recv_counts, fr_next):
        r = recv.numpy()
        k = int(np.sum(recv_counts))
        acc = np.zeros(self.n_local, np.uint64)
        np.bitwise_or.at(acc, r[0:2 * k:2], r[1:2 * k:2].view(np.uint64))
        return self._ms_fresh(level, acc, fr_next)

    def ms_end(self, nseeds, stats=True):
        if not stats:
            return None, None
        reached = np.array([int((self.mslvl[:, r] >= 0).sum()) for r in range(nseeds)])
        entries = np.array([sum(self._deg(v) for v in range(self.n_local) if self.mslvl[v, r] >= 0)
                            for r in range(nseeds)])
        return reached, entries

    pr_hot = 0          # blocked gathered layout: hot rows per rank (0 = plain layout)

    def active_rows(self):
        act = [v for v in range(self.n_local) if self.out[v] or self.inn[v]]
        return act[-1] + 1 if act else 0

    def pr_layout(self, world, span):
        """tgo_part_pr_blocked's contract: the hot-first gathered layout of world * span."""
        self.world, self.span = world, span
        self.hot = min(self.pr_hot, span)
        return self.hot

    def _split(self, v):
        from titan_amd.distributed import gathered_index
        idx = gathered_index(np.array(self.inn[v], np.int64), self.n_local, self.world, self.hot, self.span)
        return idx[idx < self.world * self.hot], idx[idx >= self.world * self.hot]

    pr_bad = 0          # tgo_part_pr_exact_check: a non-finite message reached the blocked passes
    plain = False       # tgo_part_pr_plain

    def pr_step_cold(self, gathered):
        g = gathered.numpy()        # only the cold region is complete here (hot gather in flight)
        cold = [g[self._split(v)[1]] for v in range(self.n_local)]
        self.pr_bad |= int(any(not np.isfinite(c).all() for c in cold))
        self.csum = np.array([c.sum() for c in cold])

    def pr_step_hot(self, gathered, contrib_local):
        g = gathered.numpy()
        hot = [g[self._split(v)[0]] for v in range(self.n_local)]
        self.pr_bad |= int(any(not np.isfinite(h).all() for h in hot))
        s = np.array([h.sum() for h in hot]) + self.csum
        self.pr = self.alpha * s + self.base
        with np.errstate(divide="ignore"):
            contrib_local.numpy()[:] = self.pr / self.ec

    def pr_begin(self, alpha, N, iters, contrib_local):
        N = np.float64(N)                   # Java doubles: 1 / 0 = +inf
        self.alpha, self.base = alpha, np.divide(1 - alpha, N)
        self.ec = np.array([float(len(o)) for o in self.out])
        self.pr = np.full(self.n_local, 1.0 / N)
        with np.errstate(divide="ignore"):
            contrib_local.numpy()[:] = np.divide(1.0, N) / self.ec

    def pr_step(self, contrib_global, contrib_local):
        cg = contrib_global.numpy()
        s = np.array([cg[self.inn[v]].sum() if self.inn[v] else 0.0 for v in range(self.n_local)])
        self.pr = self.alpha * s + self.base
        with np.errstate(divide="ignore"):
            contrib_local.numpy()[:] = self.pr / self.ec

    def pr_end(self, fetch=True):
        return self.pr

    def pr_exact_check(self):
        b, self.pr_bad = self.pr_bad, 0
        return b

    def pr_plain(self, on):
        self.plain = bool(on)


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, scale, roots, out_q, alpha):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from titan_amd import rmat_edges
    from titan_amd.distributed import distributed_bfs, distributed_pagerank, partition_range
    n = 1 << scale
    src, dst, _ = rmat_edges(scale, 8, seed=21)
    lo, hi = partition_range(n, world, rank)
    be = NumpyPartBackend(n, lo, hi, src, dst)
    res = {"bfs": [], "reached": []}
    for r in roots:
        d, reached, levels = distributed_bfs(be, int(r), n, alpha=alpha)
        full = [torch.zeros(be.n_local, dtype=torch.int64) for _ in range(world)]
        dist.all_gather(full, torch.from_numpy(d.astype(np.int64)))
        res["bfs"].append(torch.cat(full).numpy())
        res["reached"].append(reached)
    from titan_amd.distributed import distributed_msbfs
    # mixed, always push (fixed-capacity pairs, sized pairs, dense slices), always pull
    for ms_alpha, sparse, fixed in ((12.0, True, None), (1e9, True, None), (1e9, True, 0), (1e9, False, None),
                                    (1e-9, True, None)):
        r, e, _ = distributed_msbfs(be, roots, n, ms_alpha=ms_alpha, sparse_exchange=sparse,
                                    fixed_exchange_bytes=fixed)
        lv = []
        for i in range(len(roots)):
            loc = np.where(be.mslvl[:, i] >= 0, be.mslvl[:, i], ABSENT)
            full = [torch.zeros(be.n_local, dtype=torch.int64) for _ in range(world)]
            dist.all_gather(full, torch.from_numpy(loc.astype(np.int64)))
            lv.append(torch.cat(full).numpy())
        res.setdefault("ms", []).append((lv, r))
    res["n_fixed"] = getattr(be, "n_fixed", 0)
    for hot in (0, 16):             # plain rank-major all-gather; blocked hot-first layout
        be.pr_hot = hot
        pr = distributed_pagerank(be, 0.85, n, 10)
        full = [torch.zeros(be.n_local, dtype=torch.float64) for _ in range(world)]
        dist.all_gather(full, torch.from_numpy(pr))
        res.setdefault("pr", []).append(torch.cat(full).numpy())
    # vertexCount 0: every message +inf, outside the blocked passes' exact range — the ranks
    # agree (all-reduce MAX of the flag) and re-run on the plain layout
    be.pr_hot = 16
    pr = distributed_pagerank(be, 0.85, 0, 5)
    full = [torch.zeros(be.n_local, dtype=torch.float64) for _ in range(world)]
    dist.all_gather(full, torch.from_numpy(pr))
    res["pr_inf"] = (torch.cat(full).numpy(), be.plain)
    if rank == 0:
        out_q.put(res)
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("world,alpha", [(2, 15.0), (2, 1e9), (4, 15.0), (8, 15.0)])
def test_distributed_bfs_and_pagerank_match_oracle(world, alpha):
    import fulgora as fr
    from titan_amd import rmat_edges
    scale = 9
    n = 1 << scale
    src, dst, _ = rmat_edges(scale, 8, seed=21)
    roots = [int(src[0]), int(dst[5]), int(src[77])]
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, scale, roots, q, alpha)) for r in range(world)]
    for p in procs:
        p.start()
    res = q.get(timeout=240)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    og = fr.OracleGraph.from_edges(n, src, dst)
    ids = (np.arange(n, dtype=np.int64) + 1) << 3
    for r, d, reached in zip(roots, res["bfs"], res["reached"]):
        od, _ = og.shortest_distance(int(ids[r]), n, 2)
        assert np.array_equal(d, od)
        assert reached[0] == int((od != ABSENT).sum())
    assert res["n_fixed"] > 0                    # the fixed-capacity exchange ran
    for lv, reached in res["ms"]:
        for i, r in enumerate(roots):
            od, _ = og.shortest_distance(int(ids[r]), n, 2)
            assert np.array_equal(lv[i], od)
            assert reached[i] == int((od != ABSENT).sum())
    opr, _ = og.pagerank(0.85, n, 10)
    fin = np.isfinite(opr)
    for pr in res["pr"]:
        assert np.array_equal(np.isfinite(pr), fin)
        assert np.abs(pr[fin] - opr[fin]).sum() <= 1e-6
    pinf, plain_left_on = res["pr_inf"]
    assert np.array_equal(np.isposinf(pinf), np.isposinf(og.pagerank(0.85, 0, 5)[0])) and np.isposinf(pinf).all()
    assert not plain_left_on


def _sssp_worker(rank, world, port, scale, seeds, scope, deltas, out_q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from titan_amd import rmat_edges
    from titan_amd.distributed import distributed_sssp, partition_range
    n = 1 << scale
    src, dst, w = rmat_edges(scale, 8, seed=23, weights=True)
    lo, hi = partition_range(n, world, rank)
    be = NumpyPartBackend(n, lo, hi, src, dst, w=w, scope=scope)
    res = []
    for s in seeds:
        for delta in deltas:
            d, reached, phases = distributed_sssp(be, int(s), delta)
            full = [torch.zeros(be.n_local, dtype=torch.int64) for _ in range(world)]
            dist.all_gather(full, torch.from_numpy(d.astype(np.int64)))
            res.append((int(s), delta, torch.cat(full).numpy(), int(reached[0])))
    if rank == 0:
        out_q.put(res)
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("world,scope", [(2, 1), (4, 0), (2, 2)])
def test_distributed_delta_stepping_matches_oracle(world, scope):
    """The partitioned delta-stepping protocol (relax -> per-owner pair all-to-all -> apply,
    bucket threshold by all-reduce MIN) gives the converged distances of the reference
    program, for bucket widths from 1 to one bucket."""
    import fulgora as fr
    from titan_amd import rmat_edges
    scale = 8
    n = 1 << scale
    src, dst, w = rmat_edges(scale, 8, seed=23, weights=True)
    seeds = [int(src[0]), int(dst[3])]
    deltas = [1, 50, 1 << 40]
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_sssp_worker, args=(r, world, port, scale, seeds, scope, deltas, q))
             for r in range(world)]
    for p in procs:
        p.start()
    res = q.get(timeout=240)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    og = fr.OracleGraph.from_edges(n, src, dst, w)
    ids = (np.arange(n, dtype=np.int64) + 1) << 3
    for s, delta, d, reached in res:
        od, _ = og.shortest_distance(int(ids[s]), n, scope, weighted=True)
        assert np.array_equal(d, od), (s, delta)
        assert reached == int((od != ABSENT).sum())


def test_partition_range_is_word_aligned():
    from titan_amd.distributed import partition_range
    assert partition_range(1 << 10, 4, 3) == (768, 1024)
    with pytest.raises(ValueError):
        partition_range(1000, 4, 0)


def _layout_worker(rank, world, port, scale, out_q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from titan_amd import rmat_edges
    from titan_amd.distributed import all_gather_layout, entry_imbalance, partition_range, pick_roots_partitioned
    n = 1 << scale
    src, dst, _ = rmat_edges(scale, 8, seed=23)
    lo, hi = partition_range(n, world, rank)
    lay = all_gather_layout(src, dst, n, lo, hi, torch.device("cpu"), threads=2)
    mine = ((src >= lo) & (src < hi)) | ((dst >= lo) & (dst < hi))      # the rank's partition edges
    roots = pick_roots_partitioned(n, src[mine], dst[mine], lo, hi, 16, 7, torch.device("cpu"))
    owned = int(((src >= lo) & (src < hi)).sum() + ((dst >= lo) & (dst < hi)).sum())
    out_q.put((rank, (lay, roots, entry_imbalance(owned, torch.device("cpu")))))
    dist.barrier()
    dist.destroy_process_group()


def test_all_gathered_layout_is_a_rangewise_degree_order():
    """tgo_part_layout (host code of the C-ABI) + the all-gather every rank loads with: a
    permutation keeping each owned range, hottest half-octave degree group first, stable."""
    from titan_amd import rmat_edges
    from titan_amd.distributed import partition_range
    world, scale = 2, 10
    n = 1 << scale
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_layout_worker, args=(r, world, port, scale, q)) for r in range(world)]
    for p in procs:
        p.start()
    got = dict(q.get(timeout=240) for _ in range(world))
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    (lay0, roots0, imb0), (lay1, roots1, imb1) = got[0], got[1]
    assert np.array_equal(lay0, lay1)
    lay = lay0.astype(np.int64)
    src, dst, _ = rmat_edges(scale, 8, seed=23)
    from titan_amd import pick_roots
    assert roots0 == roots1 == [int(x) for x in pick_roots(n, src, dst, 16, seed=7)]   # the one-GPU bench's roots
    ent = [int(((src >= lo) & (src < hi)).sum() + ((dst >= lo) & (dst < hi)).sum())
           for lo, hi in (partition_range(n, world, r) for r in range(world))]
    assert imb0 == imb1 and imb0[0] == ent and abs(imb0[1] - max(ent) / np.mean(ent)) < 1e-12
    deg = np.bincount(src, minlength=n) + np.bincount(dst, minlength=n)
    bucket = np.where(deg == 0, 0, 1 + np.floor(2.0 * np.log2(np.maximum(deg, 1))).astype(np.int64))
    for r in range(world):
        lo, hi = partition_range(n, world, r)
        part = lay[lo:hi]
        assert np.array_equal(np.sort(part), np.arange(lo, hi))
        inv = np.empty(hi - lo, np.int64)
        inv[part - lo] = np.arange(lo, hi)
        b = bucket[inv]
        assert np.all(np.diff(b) <= 0)                       # hottest group first
        for g in np.unique(b):                               # row order kept inside a group
            assert np.all(np.diff(inv[b == g]) > 0)


def _subgroup_worker(rank, world, port, scale, roots, out_q):
    """Ranks {0, 3} and {1, 2} run the drivers concurrently on two subgroups: every
    collective (counts included) must stay inside its group or the run hangs / mixes sums."""
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from titan_amd import rmat_edges
    from titan_amd.distributed import (distributed_bfs, distributed_msbfs, distributed_pagerank, distributed_sssp,
                                       partition_range)
    groups = {0: dist.new_group([0, 3]), 1: dist.new_group([1, 2])}
    gid = 0 if rank in (0, 3) else 1
    grp = groups[gid]
    grank = dist.get_rank(grp)
    n = 1 << scale
    src, dst, w = rmat_edges(scale, 8, seed=31 + gid, weights=True)
    lo, hi = partition_range(n, 2, grank)
    res = {}
    be = NumpyPartBackend(n, lo, hi, src, dst)
    d, reached, _ = distributed_bfs(be, roots[gid], n, group=grp)
    r, e, _ = distributed_msbfs(be, [roots[gid], roots[1 - gid]], n, group=grp)
    pr = distributed_pagerank(be, 0.85, n, 6, group=grp)
    bw = NumpyPartBackend(n, lo, hi, src, dst, w=w, scope=1)
    sd, sreached, _ = distributed_sssp(bw, roots[gid], 40, group=grp)
    res = {"gid": gid, "lo": lo, "bfs": d, "reached": reached, "ms_reached": r, "pr": pr, "sssp": sd}
    out_q.put(res)
    dist.barrier()
    dist.destroy_process_group()


def test_distributed_drivers_on_subgroups():
    import fulgora as fr
    from titan_amd import rmat_edges
    world, scale = 4, 8
    n = 1 << scale
    roots = [3, 77]
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_subgroup_worker, args=(r, world, port, scale, roots, q)) for r in range(world)]
    for p in procs:
        p.start()
    got = [q.get(timeout=240) for _ in range(world)]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    ids = (np.arange(n, dtype=np.int64) + 1) << 3
    for gid in (0, 1):
        parts = sorted((g for g in got if g["gid"] == gid), key=lambda g: g["lo"])
        assert len(parts) == 2
        src, dst, w = rmat_edges(scale, 8, seed=31 + gid, weights=True)
        og = fr.OracleGraph.from_edges(n, src, dst, w)
        od, _ = og.shortest_distance(int(ids[roots[gid]]), n, 2)
        assert np.array_equal(np.concatenate([p["bfs"] for p in parts]), od)
        assert parts[0]["reached"][0] == int((od != ABSENT).sum())
        assert parts[0]["ms_reached"][0] == int((od != ABSENT).sum())
        opr, _ = og.pagerank(0.85, n, 6)
        assert np.abs(np.concatenate([p["pr"] for p in parts]) - opr).sum() <= 1e-6
        osd, _ = og.shortest_distance(int(ids[roots[gid]]), n, 1, weighted=True)
        assert np.array_equal(np.concatenate([p["sssp"] for p in parts]), osd)


def test_in_process_group_runs_the_real_drivers():
    """InProcessGroup (one thread per rank, the drivers' collectives as thread rendezvous):
    the same drivers over the numpy local steps give the oracle's results at world 2 and 4 —
    the communicator the one-GPU GPU tests drive the HIP local steps with."""
    import fulgora as fr
    from titan_amd import rmat_edges
    from titan_amd.distributed import (InProcessGroup, distributed_bfs, distributed_msbfs, distributed_pagerank,
                                       distributed_sssp, partition_range)
    scale = 8
    n = 1 << scale
    src, dst, w = rmat_edges(scale, 8, seed=29, weights=True)
    og = fr.OracleGraph.from_edges(n, src, dst, w)
    ids = (np.arange(n, dtype=np.int64) + 1) << 3
    roots = [int(src[0]), int(dst[11])]
    for world in (2, 4):
        bes = [NumpyPartBackend(n, *partition_range(n, world, r), src, dst) for r in range(world)]
        wbes = [NumpyPartBackend(n, *partition_range(n, world, r), src, dst, w=w, scope=1) for r in range(world)]

        def body(rank, comm):
            be = bes[rank]
            d, reached, _ = distributed_bfs(be, roots[0], n, comm=comm)
            r, _, _ = distributed_msbfs(be, roots, n, comm=comm)
            lv = [np.where(be.mslvl[:, i] >= 0, be.mslvl[:, i], ABSENT) for i in range(len(roots))]
            pr = distributed_pagerank(be, 0.85, n, 8, comm=comm)
            sd, sreached, _ = distributed_sssp(wbes[rank], roots[1], 0, comm=comm)
            return d, reached, r, lv, pr, sd, sreached

        res = InProcessGroup(world).run(body)
        od, _ = og.shortest_distance(int(ids[roots[0]]), n, 2)
        assert np.array_equal(np.concatenate([x[0] for x in res]), od)
        assert all(x[1][0] == int((od != ABSENT).sum()) for x in res)
        for i, root in enumerate(roots):
            o, _ = og.shortest_distance(int(ids[root]), n, 2)
            assert np.array_equal(np.concatenate([x[3][i] for x in res]), o)
            assert res[0][2][i] == int((o != ABSENT).sum())
        opr, _ = og.pagerank(0.85, n, 8)
        assert np.abs(np.concatenate([x[4] for x in res]) - opr).sum() <= 1e-6
        osd, _ = og.shortest_distance(int(ids[roots[1]]), n, 1, weighted=True)
        assert np.array_equal(np.concatenate([x[5] for x in res]), osd)


def test_slot_partition_balances_entries_and_round_trips():
    """SlotPartition.balanced: 64-aligned ranges of near-equal entries + vertices, equal
    exchange slots, caller <-> slot ids round trip; a skewed weight vector is cut at the
    boundary closest to the even share."""
    from titan_amd import rmat_edges
    from titan_amd.distributed import SlotPartition, word_weights
    p = SlotPartition.balanced(np.array([10, 1, 1, 1, 50, 1, 1, 1, 1, 1]), 3)
    assert list(p.bounds) == [0, 256, 320, 640] and p.slot == 320 and p.n_slots == 960
    scale = 14
    n = 1 << scale
    src, dst, _ = rmat_edges(scale, 16, seed=5)
    ww = word_weights(src, dst, 0, n)
    assert int(ww.sum()) == 2 * len(src) + n
    for world in (2, 4, 8):
        bal, eq = SlotPartition.balanced(ww, world), SlotPartition.equal(n, world)
        wb, we = bal.weights(ww), eq.weights(ww)
        assert sum(wb) == sum(we) == int(ww.sum())
        assert max(wb) / np.mean(wb) <= max(we) / np.mean(we)
        assert max(wb) / np.mean(wb) < 1.1           # word granularity: hub words are coarse at scale 14
        assert bal.slot % 64 == 0 and bal.slot >= n // world
        v = np.arange(n, dtype=np.int32)
        s = bal.to_slots(v)
        assert s.dtype == np.int32 and len(np.unique(s)) == n and s.max() < bal.n_slots
        assert np.array_equal(bal.from_slots(s), v)
        for r in range(world):
            lo, hi = bal.range(r)
            assert np.array_equal(s[lo:hi], np.arange(r * bal.slot, r * bal.slot + hi - lo))
    with pytest.raises(ValueError):
        SlotPartition([0, 100, 256], 256)


def test_balanced_partition_runs_the_real_drivers():
    """The edge-balanced partition end to end over InProcessGroup: weights all-gathered from
    equal ranges, the same bounds on every rank, the roots of the one-GPU bench, and the real
    drivers over slot ids (numpy local steps) — results mapped back equal the oracle's."""
    import fulgora as fr
    from titan_amd import pick_roots, rmat_edges
    from titan_amd.distributed import (InProcessGroup, balanced_partition, distributed_bfs, distributed_msbfs,
                                       distributed_pagerank, distributed_sssp, partition_range,
                                       pick_roots_partitioned)
    scale = 9
    n = 1 << scale
    src, dst, w = rmat_edges(scale, 8, seed=41, weights=True)
    og = fr.OracleGraph.from_edges(n, src, dst, w)
    ids = (np.arange(n, dtype=np.int64) + 1) << 3
    for world in (2, 4):
        def body(rank, comm):
            elo, ehi = partition_range(n, world, rank)
            mine = ((src >= elo) & (src < ehi)) | ((dst >= elo) & (dst < ehi))
            part, ww = balanced_partition(src[mine], dst[mine], n, elo, ehi, torch.device("cpu"), comm=comm)
            lo, hi = part.range(rank)
            mine = ((src >= lo) & (src < hi)) | ((dst >= lo) & (dst < hi))
            roots = pick_roots_partitioned(n, src[mine], dst[mine], lo, hi, 3, 7, torch.device("cpu"), comm=comm,
                                           part=part)
            s, d, wt = part.to_slots(src[mine]), part.to_slots(dst[mine]), w[mine]
            ns, (slo, shi) = part.n_slots, part.slot_range(rank)
            be = NumpyPartBackend(ns, slo, shi, s, d)
            rs = [int(x) for x in part.to_slots(np.asarray(roots))]
            bd, _, _ = distributed_bfs(be, rs[0], ns, comm=comm)
            distributed_msbfs(be, rs, ns, comm=comm)
            lv = [part.slot_results(rank, np.where(be.mslvl[:, i] >= 0, be.mslvl[:, i], ABSENT))
                  for i in range(len(rs))]
            pr = distributed_pagerank(be, 0.85, n, 8, comm=comm)
            wbe = NumpyPartBackend(ns, slo, shi, s, d, w=wt, scope=1)
            sd, _, _ = distributed_sssp(wbe, rs[1], 0, comm=comm)
            return (list(part.bounds), roots, part.slot_results(rank, bd), lv, part.slot_results(rank, pr),
                    part.slot_results(rank, sd))

        res = InProcessGroup(world).run(body)
        assert all(x[0] == res[0][0] for x in res) and all(x[1] == res[0][1] for x in res)
        assert res[0][1] == [int(x) for x in pick_roots(n, src, dst, 3, seed=7)]
        roots = res[0][1]
        od, _ = og.shortest_distance(int(ids[roots[0]]), n, 2)
        assert np.array_equal(np.concatenate([x[2] for x in res]), od)
        for i, root in enumerate(roots):
            o, _ = og.shortest_distance(int(ids[root]), n, 2)
            assert np.array_equal(np.concatenate([x[3][i] for x in res]), o)
        opr, _ = og.pagerank(0.85, n, 8)
        got = np.concatenate([x[4] for x in res])
        fin = np.isfinite(opr)
        assert np.array_equal(np.isfinite(got), fin) and np.abs(got[fin] - opr[fin]).sum() <= 1e-6
        osd, _ = og.shortest_distance(int(ids[roots[1]]), n, 1, weighted=True)
        assert np.array_equal(np.concatenate([x[5] for x in res]), osd)


def test_in_process_group_propagates_a_rank_failure():
    from titan_amd.distributed import InProcessGroup

    def body(rank, comm):
        t = torch.ones(4)
        if rank == 1:
            raise ValueError("rank 1 fails")
        comm.all_reduce(t)            # rank 0 would wait forever without the abort
        return t

    with pytest.raises(ValueError, match="rank 1 fails"):
        InProcessGroup(2, timeout=30).run(body)


def _negative_weight_worker(rank, world, port, out_q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from titan_amd import rmat_edges
    from titan_amd.distributed import distributed_sssp, partition_range
    from titan_amd.engine import TitanException
    n = 3 * 128                                     # 64-aligned thirds past the RMAT range
    src, dst, w = rmat_edges(8, 8, seed=23, weights=True)
    src, dst = src + 128, dst + 128                 # every rank holds edges
    w = w.astype(np.int64)
    lo, hi = partition_range(n, world, rank)
    last = partition_range(n, world, world - 1)
    i = int(np.nonzero((src >= last[0]) & (dst >= last[0]))[0][0])   # an edge only the last rank holds
    w[i] = -3
    be = NumpyPartBackend(n, lo, hi, src, dst, w=w, scope=1)
    try:
        distributed_sssp(be, int(src[0]), 0)
        out_q.put((rank, "ran"))
    except TitanException as e:
        out_q.put((rank, e.code))
    dist.barrier()
    dist.destroy_process_group()


def test_negative_weight_fails_every_rank():
    """a negative weight on ONE rank made that rank fail before the first collective
    while its peers waited in it.  The ranks now agree on the minimum weight first (all-reduce
    MIN, tgo_part_weight_min) and all of them raise."""
    from titan_amd import _lib as L
    world = 3
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_negative_weight_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = dict(q.get(timeout=120) for _ in range(world))
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    assert res == {r: L.TGO_E_INVALID for r in range(world)}

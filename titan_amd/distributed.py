"""Multi-GPU driver: 1-D vertex-partitioned BFS and PageRank, one process per GPU.

Rank r owns global vertices [r*n/N, (r+1)*n/N) and their Titan rows (include/
titan_gpu_olap_part.h).  Every superstep is one local kernel on the rank's GPU plus one
exchange through torch.distributed — backend "nccl", i.e. RCCL over xGMI on MI355X:

  BFS top-down level   : local frontier marks neighbours in a global "discovered" bitmap
                         -> all_to_all_single (slice r to rank r, n/8/N bytes each)
                         -> owners OR the slices and claim unvisited vertices
  BFS bottom-up level  : all_gather_into_tensor of owned next-frontier bitmap slices
                         (n/8 bytes in total) -> unvisited owned vertices probe it
  PageRank iteration   : all_gather_into_tensor of owned fp64 contributions (8n bytes), or
                         cache-blocked: cold slices, then hot slices overlapping the cold
                         gather kernels (tgo_part_pr_blocked; entry-less rows not sent)
  every level          : all_reduce(SUM) of (frontier size, frontier entries), reduced in
                         place on the device and read once (tgo_part_device_counts)

RCCL has no bitwise-OR reduction, hence slice exchanges (all-to-all / all-gather) instead
of an all-reduce of bitmaps.  The direction switch is Beamer's, on global counts.

The driver is written against a small "local step" backend so the exchange protocol is
the same code on the GPU (HipPartBackend over the C-ABI, device tensors, RCCL) and in the
CPU tests (a numpy backend with CPU tensors over gloo, tests/test_distributed.py).
"""
from __future__ import annotations

import ctypes as C

import os

import numpy as np
import torch
import torch.distributed as dist

from . import _lib as L


class TorchComm:
    """The collectives the drivers issue, over a torch.distributed group: backend "nccl"
    (RCCL over xGMI) on MI355X, "gloo" in the CPU tests.  All on torch's current stream."""

    _OPS = {"sum": dist.ReduceOp.SUM, "min": dist.ReduceOp.MIN, "max": dist.ReduceOp.MAX}

    def __init__(self, group=None):
        self.group = group

    @property
    def world(self) -> int:
        return dist.get_world_size(self.group)

    @property
    def rank(self) -> int:
        return dist.get_rank(self.group)

    def all_gather_into_tensor(self, out, inp, async_op=False):
        return dist.all_gather_into_tensor(out, inp, group=self.group, async_op=async_op)

    def all_to_all_single(self, out, inp, output_split_sizes=None, input_split_sizes=None):
        dist.all_to_all_single(out, inp, output_split_sizes=output_split_sizes, input_split_sizes=input_split_sizes,
                               group=self.group)

    def all_reduce(self, t, op="sum"):
        dist.all_reduce(t, op=self._OPS[op], group=self.group)


class _Done:
    def wait(self):
        return None


class InProcessGroup:
    """`world` ranks in ONE process, one Python thread each (InProcessGroup.run): every rank
    runs the real driver over its own backend (its own ctx and HIP stream), and the
    collectives are rendezvous of the threads that copy / reduce with torch ops.  What the
    one-GPU box can run of the partitioned path: the drivers' exchange protocol against the
    HIP local steps (tests/test_gpu_distributed.py)."""

    def __init__(self, world: int, timeout: float = 300.0):
        import threading
        self.world = world
        self._bar = threading.Barrier(world, timeout=timeout)
        self._slots = [None] * world

    def comm(self, rank: int) -> "InProcessComm":
        return InProcessComm(self, rank)

    def run(self, fn):
        """fn(rank, comm) on every rank's thread; returns the results in rank order and
        re-raises the first failure (the rendezvous is aborted so no rank waits forever)."""
        import threading
        res, errs = [None] * self.world, [None] * self.world

        def body(r):
            try:
                res[r] = fn(r, self.comm(r))
            except BaseException as e:          # noqa: BLE001 — re-raised in the caller
                errs[r] = e
                self._bar.abort()

        th = [threading.Thread(target=body, args=(r,), daemon=True) for r in range(self.world)]
        for t in th:
            t.start()
        for t in th:
            t.join()
        first = next((e for e in errs if e is not None and not isinstance(e, threading.BrokenBarrierError)), None)
        if first is None:
            first = next((e for e in errs if e is not None), None)
        if first is not None:
            raise first
        return res


class InProcessComm:
    """One rank's view of an InProcessGroup (the TorchComm interface)."""

    def __init__(self, grp: InProcessGroup, rank: int):
        self.g, self.rank, self.world = grp, rank, grp.world

    @staticmethod
    def _sync(t):
        if t.is_cuda:
            torch.cuda.current_stream(t.device).synchronize()

    def _rendezvous(self, t, item, compute):
        """Publish `item` (after this rank's stream has produced t), compute this rank's
        result from every rank's item, and wait until every rank has finished reading."""
        self._sync(t)
        self.g._slots[self.rank] = item
        self.g._bar.wait()
        compute(list(self.g._slots))
        self._sync(t)
        self.g._bar.wait()

    def all_gather_into_tensor(self, out, inp, async_op=False):
        def compute(items):
            out.copy_(torch.cat([x.to(out.device) for x in items]))
        self._rendezvous(out, inp, compute)
        return _Done() if async_op else None

    def all_to_all_single(self, out, inp, output_split_sizes=None, input_split_sizes=None):
        w = self.world
        ins = list(input_split_sizes) if input_split_sizes is not None else [inp.numel() // w] * w

        def compute(items):
            parts = []
            for x, splits in items:
                off = int(sum(splits[:self.rank]))
                parts.append(x[off:off + int(splits[self.rank])].to(out.device))
            got = torch.cat(parts)
            if output_split_sizes is not None and got.numel() != int(sum(output_split_sizes)):
                raise RuntimeError("all_to_all_single: output split sizes do not match the senders'")
            if got.numel() > out.numel():
                raise RuntimeError("all_to_all_single: output too small")
            out[:got.numel()].copy_(got)
        self._rendezvous(out, (inp, ins), compute)

    def all_reduce(self, t, op="sum"):
        def compute(items):
            st = torch.stack([x.to(t.device) for x in items])
            r = st.sum(0) if op == "sum" else (st.min(0).values if op == "min" else st.max(0).values)
            t.copy_(r)
        self._rendezvous(t, t.clone(), compute)


def _comm(comm, group):
    return comm if comm is not None else TorchComm(group)


def partition_range(n_global: int, world: int, rank: int):
    """Contiguous owned range; every slice is a whole number of 64-bit bitmap words."""
    if n_global % (64 * world):
        raise ValueError("n_global must be a multiple of 64 * world_size")
    per = n_global // world
    return rank * per, (rank + 1) * per


class SlotPartition:
    """Edge-balanced 1-D partition (contiguous ranges balanced by entries +
    vertices).  Rank r owns the caller's vertices [bounds[r], bounds[r+1]) — 64-aligned, of
    unequal sizes — and every exchange runs in a SLOT space of `world` equal slots of `slot`
    ids (the largest range, rounded up to a word): caller id v of rank r is slot id
    r * slot + (v - bounds[r]).  The C-ABI's partitioned path (titan_gpu_olap_part.h) keeps
    its equal-slice exchanges (all-gathers need equal slices; owner = id // n_local) over
    n_slots = world * slot ids; a slot past the end of its rank's range is an entry-less
    vertex that no program reaches and no result reports (slot_results drops it)."""

    def __init__(self, bounds, n: int):
        b = np.asarray(bounds, np.int64)
        if b[0] != 0 or b[-1] != n or np.any(np.diff(b) <= 0) or np.any(b % 64):
            raise ValueError("bounds must be increasing, 64-aligned and cover [0, n)")
        self.bounds, self.n, self.world = b, int(n), len(b) - 1
        self.slot = int(np.diff(b).max())
        self.n_slots = self.world * self.slot

    @classmethod
    def equal(cls, n: int, world: int):
        return cls([partition_range(n, world, r)[0] for r in range(world)] + [n], n)

    @classmethod
    def balanced(cls, word_weight, world: int):
        """Ranges of near-equal total weight over 64-vertex words (word_weight[i] = the list
        entries of vertices [64 i, 64 i + 64) plus their count): boundary r is the word
        boundary whose running weight is closest to r/world of the total; every range keeps
        >= 1 word."""
        w = np.asarray(word_weight, np.int64)
        nw = len(w)
        if nw < world:
            raise ValueError("fewer 64-vertex words than ranks")
        c = np.concatenate([[0], np.cumsum(w)])          # c[k] = weight of words [0, k)
        tot = int(c[-1])
        cut = [0]
        for r in range(1, world):
            t = tot * r / world
            k = int(np.searchsorted(c, t, side="left"))  # first boundary with c[k] >= t
            if k > 0 and t - c[k - 1] < c[k] - t:
                k -= 1
            k = max(k, cut[-1] + 1)
            k = min(k, nw - (world - r))
            cut.append(k)
        cut.append(nw)
        return cls(np.asarray(cut, np.int64) * 64, nw * 64)

    def range(self, rank: int):
        return int(self.bounds[rank]), int(self.bounds[rank + 1])

    def slot_range(self, rank: int):
        return rank * self.slot, (rank + 1) * self.slot

    def to_slots(self, v):
        """Caller ids -> slot ids (vectorised; int32 arrays stay int32 when the slots fit)."""
        v = np.asarray(v)
        r = np.searchsorted(self.bounds, v, side="right") - 1
        s = r.astype(np.int64) * self.slot + (v.astype(np.int64) - self.bounds[r])
        return s.astype(np.int32) if v.dtype == np.int32 and self.n_slots < 2**31 else s

    def from_slots(self, s):
        s = np.asarray(s, np.int64)
        r, o = s // self.slot, s % self.slot
        if np.any(o >= self.bounds[r + 1] - self.bounds[r]):
            raise ValueError("slot id past its rank's range")
        return self.bounds[r] + o

    def slot_results(self, rank: int, local):
        """A rank's slot-local results (n_local = slot values) cut to its owned caller range."""
        lo, hi = self.range(rank)
        return np.asarray(local)[:hi - lo]

    def weights(self, word_weight):
        """Per-rank total weight (the imbalance this partition leaves)."""
        c = np.concatenate([[0], np.cumsum(np.asarray(word_weight, np.int64))])
        return [int(c[self.bounds[r + 1] // 64] - c[self.bounds[r] // 64]) for r in range(self.world)]


def word_weights(src, dst, lo: int, hi: int):
    """Entries + vertices of the owned rows per 64-vertex word of [lo, hi): each edge gives
    an OUT entry to its source row and an IN entry to its target row."""
    w = np.zeros((hi - lo) // 64, np.int64)
    for x in (np.asarray(src), np.asarray(dst)):
        x = x[(x >= lo) & (x < hi)].astype(np.int64)
        w += np.bincount((x - lo) >> 6, minlength=len(w))
    return w + 64


def balanced_partition(src, dst, n: int, lo: int, hi: int, device, group=None, comm=None):
    """The edge-balanced SlotPartition every rank agrees on: each rank weighs the words of
    its equal range [lo, hi) from its partition edges (word_weights), the weights are
    all-gathered (n / 64 int64) and SlotPartition.balanced cuts them — same bounds on every
    rank.  The caller then takes the edges of its new range and maps them to slot ids."""
    cm = _comm(comm, group)
    loc = torch.from_numpy(word_weights(src, dst, lo, hi)).to(device)
    out = torch.empty(n // 64, dtype=torch.int64, device=device)
    cm.all_gather_into_tensor(out, loc)
    w = out.cpu().numpy()
    return SlotPartition.balanced(w, cm.world), w


def local_layout(src, dst, n_global: int, lo: int, hi: int, threads: int = 16):
    """tgo_part_layout: internal global ids of the owned vertices [lo, hi) (degree-grouped,
    hottest first, kept inside the owned range).  Host code only (no device needed)."""
    lib = L.load()
    src = np.ascontiguousarray(src, np.int32)
    dst = np.ascontiguousarray(dst, np.int32)
    e = L.Edges(n_global, len(src), L.ptr(src, C.c_int32), L.ptr(dst, C.c_int32), None, None)
    out = np.empty(hi - lo, np.int32)
    rc = lib.tgo_part_layout(C.byref(e), n_global, lo, hi, threads, L.ptr(out, C.c_int32))
    if rc:
        raise RuntimeError(f"tgo_part_layout rc={rc}")
    return out


def all_gather_layout(src, dst, n_global: int, lo: int, hi: int, device, group=None, threads: int = 16, comm=None):
    """Every rank's local_layout slice, all-gathered into the global layout (host int32,
    n_global) that every rank passes to Engine.load_partition(layout=...)."""
    loc = torch.from_numpy(local_layout(src, dst, n_global, lo, hi, threads)).to(device)
    out = torch.empty(n_global, dtype=torch.int32, device=device)
    _comm(comm, group).all_gather_into_tensor(out, loc)
    return out.cpu().numpy()


_MASK64 = (1 << 64) - 1


def _splitmix64(x: int) -> int:
    x = (x + 0x9E3779B97F4A7C15) & _MASK64
    x = ((x ^ (x >> 30)) * 0xBF58476D1CE4E5B9) & _MASK64
    x = ((x ^ (x >> 27)) * 0x94D049BB133111EB) & _MASK64
    return x ^ (x >> 31)


def pick_roots_partitioned(n_global: int, src, dst, lo: int, hi: int, nroots: int, seed: int, device, group=None,
                           comm=None, part: "SlotPartition" = None):
    """The roots tgo_pick_roots draws on the whole edge list (synth.cpp), from a rank's
    partition edges: owned "has an entry" flags are all-gathered (n bytes), then every rank
    walks the same splitmix64 candidate sequence — the partitioned bench runs the same
    sources as the one-GPU bench.  Caller ids throughout; with a SlotPartition the flags
    travel in its equal slots (lo, hi = the rank's caller range)."""
    width = part.slot if part is not None else hi - lo
    has = np.zeros(width, np.uint8)
    for x in (src, dst):
        x = np.asarray(x)
        has[x[(x >= lo) & (x < hi)] - lo] = 1
    loc = torch.from_numpy(has).to(device)
    out = torch.empty(width * _comm(comm, group).world, dtype=torch.uint8, device=device)
    _comm(comm, group).all_gather_into_tensor(out, loc)
    has = out.cpu().numpy()
    if part is not None:
        has = np.concatenate([has[r * part.slot:r * part.slot + (part.bounds[r + 1] - part.bounds[r])]
                              for r in range(part.world)])
    if int(has.sum()) < nroots:
        raise ValueError("fewer vertices with entries than roots")
    roots, used, i = [], set(), 0
    base = (seed * 0x9E3779B97F4A7C15) & _MASK64
    while len(roots) < nroots:
        v = _splitmix64((base + i) & _MASK64) % n_global
        i += 1
        if has[v] and v not in used:
            used.add(v)
            roots.append(v)
    return roots


def entry_imbalance(entries_local: int, device, group=None, comm=None):
    """Per-rank owned entries, all-gathered: (list, max / mean) — the load imbalance of the
    1-D partition."""
    cm = _comm(comm, group)
    t = torch.tensor([int(entries_local)], dtype=torch.int64, device=device)
    out = torch.empty(cm.world, dtype=torch.int64, device=device)
    cm.all_gather_into_tensor(out, t)
    e = [int(x) for x in out.cpu()]
    mean = sum(e) / len(e)
    return e, (max(e) / mean if mean else 1.0)


def exchange_stream() -> int:
    """The HIP stream handle the partitioned engine must share with torch's collectives.
    torch's default stream has handle 0, which the C-ABI reads as "ctx-owned stream" (not
    ordered with torch's work), so switch this thread to a dedicated side stream first."""
    cur = torch.cuda.current_stream()
    if cur.cuda_stream == 0:
        cur = torch.cuda.Stream()
        torch.cuda.set_stream(cur)
    return cur.cuda_stream


class HipPartBackend:
    """Local steps on this rank's GPU through the C-ABI (titan_gpu_olap_part.h).  The
    engine runs on torch's current (non-default) stream, so its kernels and the RCCL
    collectives of the driver are ordered on one stream (see exchange_stream)."""

    # steps whose level counts can stay on the device (tgo_part_device_counts)
    DEVICE_COUNT_STEPS = frozenset({"tgo_part_bfs_claim", "tgo_part_bfs_bu", "tgo_part_ms_pull", "tgo_part_ms_settle",
                                    "tgo_part_ms_settle_pairs", "tgo_part_ms_settle_fixed"})

    def __init__(self, engine, n_global, lo, hi, device_counts=False):
        if engine.stream == 0 or engine.stream != torch.cuda.current_stream().cuda_stream:
            raise ValueError("HipPartBackend: the Engine must run on torch's current non-default stream "
                             "(Engine(stream=exchange_stream()))")
        self.e = engine
        self.n_global, self.lo, self.hi = n_global, lo, hi
        self.n_local = hi - lo
        self.device = torch.device("cuda", torch.cuda.current_device())
        self.total_entries = int(engine.stats()["out_entries"] + engine.stats()["in_entries"])
        # device_counts: level counts are returned as this device tensor (all-reduced in
        # place by the driver, read once per level) instead of a host array per call
        self.dc = None
        if device_counts:
            # [0..1] all-reduced counts, [2] this rank's queue length: one host read per level
            self.dc = torch.zeros(3, dtype=torch.int64, device=self.device)
            engine.part_call("tgo_part_device_counts", self._vp(self.dc))
            self.dc._tgo_backend = self

    def tensor(self, n, dtype):
        return torch.zeros(n, dtype=dtype, device=self.device)

    @staticmethod
    def _vp(t):
        return C.c_void_p(t.data_ptr())

    def _counts(self, fn, *args):
        if self.dc is not None and fn in self.DEVICE_COUNT_STEPS:
            self.e.part_call(fn, *args, None)
            return self.dc
        c = np.zeros(2, np.int64)
        self.e.part_call(fn, *args, L.ptr(c, C.c_int64))
        return c

    def bfs_begin(self, seed, nb_local):
        return self._counts("tgo_part_bfs_begin", C.c_int64(seed), self._vp(nb_local))

    def bfs_td(self, level, disc):
        self.e.part_call("tgo_part_bfs_td", level, self._vp(disc))

    def bfs_claim(self, level, recv, nslices, nb_local):
        return self._counts("tgo_part_bfs_claim", level, self._vp(recv), nslices, self._vp(nb_local))

    def bfs_bu(self, level, fb_global, nb_local):
        return self._counts("tgo_part_bfs_bu", level, self._vp(fb_global), self._vp(nb_local))

    def bfs_end(self, fetch=True, stats=True):
        out = np.zeros(self.n_local, np.int64) if fetch else None
        reached = np.zeros(2, np.int64) if stats else None
        self.e.part_call("tgo_part_bfs_end", L.ptr(out, C.c_int64), L.ptr(reached, C.c_int64))
        return out, reached

    # multi-source BFS local steps
    def ms_begin(self, seeds, fr_local):
        sd = np.ascontiguousarray(seeds, np.int64)
        return self._counts("tgo_part_ms_begin", L.ptr(sd, C.c_int64), len(sd), self._vp(fr_local))

    def ms_pull(self, level, fr_global, fr_next):
        return self._counts("tgo_part_ms_pull", level, self._vp(fr_global), self._vp(fr_next))

    def ms_push(self, level, fr_local, cand):
        self.e.part_call("tgo_part_ms_push", level, self._vp(fr_local), self._vp(cand))

    def ms_settle(self, level, recv, nslices, fr_next):
        return self._counts("tgo_part_ms_settle", level, self._vp(recv), nslices, self._vp(fr_next))

    def ms_pack_dev(self, cand, send, nranks, send_elems):
        self.e.part_call("tgo_part_ms_pack_dev", self._vp(cand), nranks, self._vp(send), self._vp(send_elems))

    def ms_pack(self, cand, send, nranks):
        sc = np.zeros(nranks, np.int64)
        self.e.part_call("tgo_part_ms_pack", self._vp(cand), nranks, self._vp(send), L.ptr(sc, C.c_int64))
        return sc

    def ms_pack_fixed(self, cand, send, nranks, cap):
        self.e.part_call("tgo_part_ms_pack_fixed", self._vp(cand), nranks, C.c_int64(cap), self._vp(send))

    def ms_settle_fixed(self, level, recv, nslices, cap, fr_next):
        return self._counts("tgo_part_ms_settle_fixed", level, self._vp(recv), nslices, C.c_int64(cap), self._vp(fr_next))

    def ms_settle_pairs(self, level, recv, recv_counts, fr_next):
        rc = np.ascontiguousarray(recv_counts, np.int64)
        return self._counts("tgo_part_ms_settle_pairs", level, self._vp(recv), L.ptr(rc, C.c_int64), len(rc),
                            self._vp(fr_next))

    def ms_end(self, nseeds, stats=True):
        if not stats:
            self.e.part_call("tgo_part_ms_end", None, None)
            return None, None
        r = np.zeros(nseeds, np.int64)
        e = np.zeros(nseeds, np.int64)
        self.e.part_call("tgo_part_ms_end", L.ptr(r, C.c_int64), L.ptr(e, C.c_int64))
        return r, e

    def ms_levels(self, source):
        out = np.zeros(self.n_local, np.int64)
        self.e.part_call("tgo_part_ms_levels", source, L.ptr(out, C.c_int64))
        return out

    # delta-stepping SSSP local steps
    def weight_min(self):
        """The smallest weight of this rank's load, 0 without weights (tgo_part_weight_min)."""
        w = C.c_int64()
        self.e.part_call("tgo_part_weight_min", C.byref(w))
        return w.value

    def sssp_begin(self, seed, delta):
        c = np.zeros(2, np.int64)
        self.e.part_call("tgo_part_sssp_begin", C.c_int64(seed), C.c_int64(delta), L.ptr(c, C.c_int64))
        return c

    def sssp_relax(self, thr, send, nranks):
        sc = np.zeros(nranks, np.int64)
        self.e.part_call("tgo_part_sssp_relax", C.c_int64(thr), nranks, self._vp(send), L.ptr(sc, C.c_int64))
        return sc

    def sssp_apply(self, thr, recv, npairs):
        return self._counts("tgo_part_sssp_apply", C.c_int64(thr), self._vp(recv), C.c_int64(npairs))

    def sssp_pending_min(self):
        c = np.zeros(2, np.int64)
        self.e.part_call("tgo_part_sssp_pending_min", L.ptr(c, C.c_int64))
        return c

    def sssp_extract(self, thr):
        return self._counts("tgo_part_sssp_extract", C.c_int64(thr))

    def sssp_end(self, fetch=True, stats=True):
        out = np.zeros(self.n_local, np.int64) if fetch else None
        reached = np.zeros(2, np.int64) if stats else None
        self.e.part_call("tgo_part_sssp_end", L.ptr(out, C.c_int64), L.ptr(reached, C.c_int64))
        return out, reached

    def active_rows(self):
        a = C.c_int64()
        self.e.part_call("tgo_part_active_rows", C.byref(a))
        return a.value

    def pr_layout(self, world, active_span):
        """Hot rows per rank of the blocked gathered layout (tgo_part_pr_blocked); 0 = plain."""
        h = C.c_int64()
        self.e.part_call("tgo_part_pr_blocked", int(world), C.c_int64(active_span), C.byref(h))
        return h.value

    def pr_begin(self, alpha, vertex_count, iters, contrib_local):
        a = L.PrArgs(alpha, int(vertex_count), int(iters), 0)
        self.e.part_call("tgo_part_pr_begin", C.byref(a), self._vp(contrib_local))

    def pr_step(self, contrib_global, contrib_local):
        self.e.part_call("tgo_part_pr_step", self._vp(contrib_global), self._vp(contrib_local))

    def pr_step_cold(self, gathered):
        self.e.part_call("tgo_part_pr_step_cold", self._vp(gathered))

    def pr_step_hot(self, gathered, contrib_local):
        self.e.part_call("tgo_part_pr_step_hot", self._vp(gathered), self._vp(contrib_local))

    def pr_end(self, fetch=True):
        out = np.zeros(self.n_local, np.float64) if fetch else None
        self.e.part_call("tgo_part_pr_end", L.ptr(out, C.c_double))
        return out

    def pr_exact_check(self):
        """1 when a fixed-point pass of the blocked layout saw a message outside its exact range
        since the last check (tgo_part_pr_exact_check; the flag is cleared)."""
        b = C.c_int32()
        self.e.part_call("tgo_part_pr_exact_check", C.byref(b))
        return b.value

    def pr_plain(self, on):
        """Run the next programs on the plain layout (tgo_part_pr_plain)."""
        self.e.part_call("tgo_part_pr_plain", 1 if on else 0)


def _scratch(backend, name, n, dtype):
    """Exchange buffers live as long as the backend (allocated zero-filled once, reused by
    every run: the drivers only rely on zeros where the local steps restore them)."""
    bufs = backend.__dict__.setdefault("_scratch", {})
    t = bufs.get(name)
    if t is None or t.numel() < n or t.dtype != dtype:
        t = backend.tensor(n, dtype)
        bufs[name] = t
    return t[:n]


def _allreduce_counts(c, device, comm):
    """Global sums of per-rank counters (frontier size / entries, reached, ...) over `comm`.
    A device tensor (HipPartBackend device_counts) is reduced in place and read once per level
    together with the rank's own queue length, which goes back to the engine."""
    be = getattr(c, "_tgo_backend", None)
    if be is not None:
        comm.all_reduce(c[:2])
        v = c.cpu().numpy()
        be.e.part_call("tgo_part_set_local_qlen", C.c_int64(int(v[2])))
        return v[:2]
    t = c if isinstance(c, torch.Tensor) else torch.tensor(c, dtype=torch.int64, device=device)
    comm.all_reduce(t)
    return t.cpu().numpy()


# Direction switch of the single-source BFS (Beamer): bottom-up once the frontier's entries pass
# 1/BFS_ALPHA of the unexplored ones, top-down again below n/BFS_BETA frontier vertices — the
# one-GPU engine's defaults (api.cpp run_bfs, round 5: 30 / 5000 against Beamer's 15 / 18,
# profiles/r05ab_bfs_switch_ab.log).
BFS_ALPHA = 30.0
BFS_BETA = 5000.0


def distributed_bfs(backend, seed: int, max_depth: int, alpha: float = BFS_ALPHA, beta: float = BFS_BETA,
                    fetch: bool = True, stats: bool = True, group=None, comm=None):
    """ShortestDistance with unit weights over bothE on a vertex-partitioned graph.
    Returns (local distances or None, global reached [vertices, entries] or None, levels)."""
    cm = _comm(comm, group)
    world = cm.world
    nwl = backend.n_local // 64
    nwg = backend.n_global // 64
    dev = backend.device
    fb_global = _scratch(backend, "bfs_fb", nwg, torch.int64)
    nb_local = _scratch(backend, "bfs_nb", nwl, torch.int64)
    disc = _scratch(backend, "bfs_disc", nwg, torch.int64)
    recv = _scratch(backend, "bfs_recv", nwg, torch.int64)
    total = _allreduce_counts([backend.total_entries, 0], dev, cm)[0]
    c = backend.bfs_begin(seed, nb_local)
    cm.all_gather_into_tensor(fb_global, nb_local)
    nf, mf = _allreduce_counts(c, dev, cm)
    mu = total - mf
    bottom_up = False
    levels = 0
    n = backend.n_global
    for level in range(max_depth):
        if nf == 0:
            break
        if not bottom_up and mf > mu / alpha:
            bottom_up = True
        elif bottom_up and nf < n / beta:
            bottom_up = False
        if bottom_up:
            c = backend.bfs_bu(level, fb_global, nb_local)
        else:
            disc.zero_()
            backend.bfs_td(level, disc)
            cm.all_to_all_single(recv, disc)
            c = backend.bfs_claim(level, recv, world, nb_local)
        cm.all_gather_into_tensor(fb_global, nb_local)
        nf, mf = _allreduce_counts(c, dev, cm)
        mu -= mf
        levels += 1
    out, reached = backend.bfs_end(fetch, stats)
    if stats:
        reached = _allreduce_counts(reached, dev, cm)
    return out, reached, levels


def _exchange_pairs(send, counts, recv, dev, comm):
    """all_to_all of the per-rank pair counts, then of the (id, value) int64 pairs with
    split sizes; returns the received count per sender."""
    sct = torch.from_numpy(2 * np.asarray(counts, np.int64)).to(dev)
    rct = torch.empty_like(sct)
    comm.all_to_all_single(rct, sct)
    ins = [int(x) for x in sct.cpu()]
    outs = [int(x) for x in rct.cpu()]
    comm.all_to_all_single(recv[:sum(outs)], send[:sum(ins)], output_split_sizes=outs, input_split_sizes=ins)
    return np.asarray(outs, np.int64) // 2


def _exchange_pairs_dev(send, sct, recv, comm):
    """As _exchange_pairs with the split sizes already on the device (sct, int64 elements per
    destination): one all_to_all of the sizes, ONE host read of both size vectors."""
    rct = torch.empty_like(sct)
    comm.all_to_all_single(rct, sct)
    both = torch.cat([sct, rct]).cpu().numpy()
    w = len(sct)
    ins = [int(x) for x in both[:w]]
    outs = [int(x) for x in both[w:]]
    comm.all_to_all_single(recv[:sum(outs)], send[:sum(ins)], output_split_sizes=outs, input_split_sizes=ins)
    return np.asarray(outs, np.int64) // 2


# sparse multi-source levels whose per-rank send fits this many bytes use the fixed-capacity
# exchange (equal splits bounded by the frontier entries, no all-to-all of split sizes)
FIXED_EXCHANGE_BYTES = int(os.environ.get("TGO_MS_FIXED_BYTES", 64 << 20))


def distributed_msbfs(backend, seeds, max_depth: int, ms_alpha: float = 12.0, stats: bool = True, group=None,
                      sparse_exchange: bool = True, fixed_exchange_bytes: int = None, comm=None):
    """Up to 64 ShortestDistance programs with unit weights over bothE, run together with
    bit-parallel frontier masks on a vertex-partitioned graph.
      dense level : all_gather of owned frontier masks (8 bytes per vertex) -> local pull
      sparse level: local push into global candidate masks -> pack the nonzero ones into
                    (owner-local id, mask) pairs -> all_to_all with split sizes -> settle
                    (sparse_exchange=False: all_to_all of the whole n_global-word slices)
    Returns (per-seed global reached vertices, per-seed reached entries, levels)."""
    cm = _comm(comm, group)
    world = cm.world
    nseeds = len(seeds)
    dev = backend.device
    if fixed_exchange_bytes is None:
        fixed_exchange_bytes = FIXED_EXCHANGE_BYTES
    # the owned masks are the rank's slice of a global buffer (two, alternating by level), so
    # a dense level's all-gather is in place: no copy of the rank's own slice
    lo, nl = backend.lo, backend.n_local
    glob = [_scratch(backend, "ms_fr_global", backend.n_global, torch.int64),
            _scratch(backend, "ms_frn_global", backend.n_global, torch.int64)]
    fr, frn = glob[0][lo:lo + nl], glob[1][lo:lo + nl]
    # no clearing: every level rewrites the active rows of the next mask, and the entry-less
    # tail stays zero (tgo_part_ms_begin leaves entry-less seeds out of the masks)
    cand = _scratch(backend, "ms_cand", backend.n_global, torch.int64)     # all-zero between sparse levels
    send = recv = None
    total = _allreduce_counts([backend.total_entries, 0], dev, cm)[0]
    nf, mf = _allreduce_counts(backend.ms_begin(seeds, fr), dev, cm)
    levels = 0
    for level in range(max_depth):
        if nf == 0:
            break
        if mf * ms_alpha > total:
            cm.all_gather_into_tensor(glob[0], fr)
            c = backend.ms_pull(level, glob[0], frn)
        elif sparse_exchange:
            send = _scratch(backend, "pairs_send", 2 * backend.n_global + 2 * world, torch.int64)
            recv = _scratch(backend, "pairs_recv", 2 * backend.n_global + 2 * world, torch.int64)
            backend.ms_push(level, fr, cand)           # cand is all-zero here: the pack clears it
            # small frontier: equal splits bounded by the frontier entries, no size exchange
            cap = int(min(mf, backend.n_local))
            if hasattr(backend, "ms_pack_fixed") and cap > 0 and world * (cap + 1) * 16 <= fixed_exchange_bytes:
                ne = 2 * world * (cap + 1)
                backend.ms_pack_fixed(cand, send, world, cap)
                cm.all_to_all_single(recv[:ne], send[:ne])
                c = backend.ms_settle_fixed(level, recv, world, cap, frn)
            elif hasattr(backend, "ms_pack_dev"):
                sct = _scratch(backend, "pairs_sct", world, torch.int64)
                backend.ms_pack_dev(cand, send, world, sct)
                rcounts = _exchange_pairs_dev(send, sct, recv, cm)
                c = backend.ms_settle_pairs(level, recv, rcounts, frn)
            else:
                rcounts = _exchange_pairs(send, backend.ms_pack(cand, send, world), recv, dev, cm)
                c = backend.ms_settle_pairs(level, recv, rcounts, frn)
        else:
            recv = _scratch(backend, "slices_recv", backend.n_global, torch.int64)
            cand.zero_()
            backend.ms_push(level, fr, cand)
            cm.all_to_all_single(recv, cand)
            cand.zero_()
            c = backend.ms_settle(level, recv, world, frn)
        fr, frn = frn, fr
        glob.reverse()
        nf, mf = _allreduce_counts(c, dev, cm)
        levels += 1
    r, e = backend.ms_end(nseeds, stats)
    if stats:
        t = torch.tensor(np.concatenate([r, e]), dtype=torch.int64, device=dev)
        cm.all_reduce(t)
        t = t.cpu().numpy()
        r, e = t[:nseeds], t[nseeds:]
    return r, e, levels


class NativeExchange:
    """An exchange object of the native partitioned driver (titan_gpu_olap_part.h
    tgo_exchange_*): RCCL over xGMI (rccl(), one process per GPU) or an in-process group of
    thread ranks on one device (local_group(), tests).  Destroyed with the wrapper."""

    def __init__(self, handle):
        self.h = C.c_void_p(handle)
        # bound now: at interpreter exit the module globals (L) may be gone before __del__ runs
        self._destroy = L.load().tgo_exchange_destroy

    @classmethod
    def rccl(cls, device: int, group=None, comm=None):
        """Rank 0 makes the RCCL unique id, every rank receives it over `comm` (an all-gather
        of 128 bytes per rank, rank 0's slice taken) and joins the communicator."""
        lib = L.load()
        cm = _comm(comm, group)
        # 128 id bytes + a status byte per rank: rank 0's failure to make the id travels with
        # the all-gather, so every rank raises instead of the peers waiting for an id forever
        uid = np.zeros(136, np.uint8)
        if cm.rank == 0 and lib.tgo_exchange_rccl_id(L.ptr(uid, C.c_uint8)):
            uid[128] = 1
        dev = torch.device("cuda", device) if torch.cuda.is_available() else torch.device("cpu")
        out = torch.empty(136 * cm.world, dtype=torch.uint8, device=dev)
        cm.all_gather_into_tensor(out, torch.from_numpy(uid).to(dev))
        got = out[:136].cpu().numpy()
        if got[128]:
            raise RuntimeError("tgo_exchange_rccl_id failed on rank 0")
        uid = np.ascontiguousarray(got[:128])
        h = C.c_void_p()
        rc = lib.tgo_exchange_rccl_create(cm.world, cm.rank, L.ptr(uid, C.c_uint8), device, C.byref(h))
        if rc:
            raise RuntimeError(f"tgo_exchange_rccl_create rc={rc}")
        return cls(h.value)

    @classmethod
    def local_group(cls, world: int):
        lib = L.load()
        hs = (C.c_void_p * world)()
        if lib.tgo_exchange_local_group(world, hs):
            raise RuntimeError("tgo_exchange_local_group failed")
        return [cls(h) for h in hs]

    def __del__(self):
        destroy = getattr(self, "_destroy", None)
        if destroy is not None and getattr(self, "h", None) is not None and self.h.value:
            destroy(self.h)
            self.h = None


def distributed_msbfs_native(backend, seeds, max_depth: int, exchange: NativeExchange, ms_alpha: float = 12.0,
                             fixed_exchange_bytes: int = None, stats: bool = True):
    """distributed_msbfs as ONE native call (tgo_part_msbfs_run): the same protocol, the level
    loop and its collectives in C++ on the engine's stream.  Returns (per-seed global reached
    vertices, per-seed reached entries, levels); without stats the counts are None."""
    if fixed_exchange_bytes is None:
        fixed_exchange_bytes = FIXED_EXCHANGE_BYTES
    sd = np.ascontiguousarray(seeds, np.int64)
    r = np.zeros(len(sd), np.int64) if stats else None
    e = np.zeros(len(sd), np.int64) if stats else None
    lv = C.c_int32()
    lib = backend.e.lib
    rc = lib.tgo_part_msbfs_run(backend.e.ctx, exchange.h, L.ptr(sd, C.c_int64), len(sd), int(max_depth),
                                float(ms_alpha), int(fixed_exchange_bytes), L.ptr(r, C.c_int64), L.ptr(e, C.c_int64),
                                C.byref(lv))
    if rc:
        from .engine import TitanException
        raise TitanException(rc, (lib.tgo_last_error(backend.e.ctx) or b"").decode())
    return r, e, lv.value


def _native_check(backend, rc):
    if rc:
        from .engine import TitanException
        raise TitanException(rc, (backend.e.lib.tgo_last_error(backend.e.ctx) or b"").decode())


def distributed_bfs_native(backend, seed: int, max_depth: int, exchange: NativeExchange, alpha: float = BFS_ALPHA,
                           beta: float = BFS_BETA, fetch: bool = True, stats: bool = True):
    """distributed_bfs as ONE native call (tgo_part_bfs_run).  Returns (local distances or
    None, global [reached vertices, entries] or None, levels)."""
    out = np.zeros(backend.n_local, np.int64) if fetch else None
    reached = np.zeros(2, np.int64) if stats else None
    lv = C.c_int32()
    _native_check(backend, backend.e.lib.tgo_part_bfs_run(backend.e.ctx, exchange.h, int(seed), int(max_depth),
                                                          float(alpha), float(beta), L.ptr(out, C.c_int64),
                                                          L.ptr(reached, C.c_int64), C.byref(lv)))
    return out, reached, lv.value


def distributed_sssp_native(backend, seed: int, exchange: NativeExchange, delta: int = 0, fetch: bool = True,
                            stats: bool = True):
    """distributed_sssp as ONE native call (tgo_part_sssp_run).  Returns (local distances or
    None, global [reached vertices, entries] or None, phases)."""
    out = np.zeros(backend.n_local, np.int64) if fetch else None
    reached = np.zeros(2, np.int64) if stats else None
    ph = C.c_int32()
    _native_check(backend, backend.e.lib.tgo_part_sssp_run(backend.e.ctx, exchange.h, int(seed), int(delta),
                                                           L.ptr(out, C.c_int64), L.ptr(reached, C.c_int64),
                                                           C.byref(ph)))
    return out, reached, ph.value


PR_EXCHANGE_ALLGATHER, PR_EXCHANGE_GHOST = 0, 1


def distributed_pagerank_native(backend, alpha: float, vertex_count: int, iterations: int, exchange: NativeExchange,
                                mode: int = PR_EXCHANGE_GHOST, fetch: bool = True):
    """distributed_pagerank as ONE native call (tgo_part_pagerank_run): the layout agreed
    inside, then every update refreshes the gathered vector by an all-gather (mode 0) or the
    ghost exchange (mode 1, only the contributions this rank reads).  Returns (local ranks or
    None, bytes this rank received)."""
    if iterations == 0:
        return (np.full(backend.n_local, np.nan) if fetch else None), 0
    out = np.zeros(backend.n_local, np.float64) if fetch else None
    moved = C.c_int64()
    a = L.PrArgs(float(alpha), int(vertex_count), int(iterations), 0)
    _native_check(backend, backend.e.lib.tgo_part_pagerank_run(backend.e.ctx, exchange.h, C.byref(a), int(mode),
                                                               L.ptr(out, C.c_double), C.byref(moved)))
    return out, moved.value


INT64_MAX = (1 << 63) - 1


def distributed_sssp(backend, seed: int, delta: int = 0, fetch: bool = True, stats: bool = True, group=None,
                     comm=None):
    """Delta-stepping ShortestDistance (converged distances) on a vertex-partitioned graph.
      phase  : local relax of the owned near queue; improvements of remote vertices are
               packed per owner -> all_to_all of the pair counts, all_to_all_single of the
               (owner-local id, distance) pairs -> owners min them in and queue the ones
               below the bucket threshold
      bucket : when every near queue is empty, all_reduce(MIN) of the pending distances
               moves the threshold to the end of the next non-empty bucket
    Returns (local distances or None, global [reached vertices, entries] or None, phases)."""
    cm = _comm(comm, group)
    world = cm.world
    dev = backend.device
    n = backend.n_global
    # negative weights fail every rank together, before a peer could wait in an exchange
    wmin = torch.tensor([int(backend.weight_min())], dtype=torch.int64, device=dev)
    cm.all_reduce(wmin, op="min")
    if int(wmin.item()) < 0:
        from .engine import TitanException
        raise TitanException(L.TGO_E_INVALID, "delta-stepping needs non-negative weights (a rank holds a negative weight)")
    send = _scratch(backend, "pairs_send", 2 * n, torch.int64)
    recv = _scratch(backend, "pairs_recv", 2 * n, torch.int64)
    qlen, dflt = (int(x) for x in backend.sssp_begin(seed, delta))
    if delta <= 0:      # ranks' default widths differ with their local mean weight: agree on one
        t = torch.tensor([dflt], dtype=torch.int64, device=dev)
        cm.all_reduce(t, op="max")
        delta = int(t.item())
    thr, phases = delta, 0
    while True:
        if int(_allreduce_counts([qlen, 0], dev, cm)[0]) == 0:
            mn = torch.tensor([int(backend.sssp_pending_min()[0])], dtype=torch.int64, device=dev)
            cm.all_reduce(mn, op="min")
            mn = int(mn.item())
            if mn == INT64_MAX:
                break
            if mn >= thr:
                thr = (mn // delta + 1) * delta
            qlen = int(backend.sssp_extract(thr)[0])
            continue
        sc = backend.sssp_relax(thr, send, world)
        sct = torch.from_numpy(2 * sc).to(dev)
        rct = torch.empty_like(sct)
        cm.all_to_all_single(rct, sct)
        ins = [int(x) for x in 2 * sc]
        outs = [int(x) for x in rct.cpu()]
        cm.all_to_all_single(recv[:sum(outs)], send[:sum(ins)], output_split_sizes=outs, input_split_sizes=ins)
        qlen = int(backend.sssp_apply(thr, recv, sum(outs) // 2)[0])
        phases += 1
    out, reached = backend.sssp_end(fetch, stats)
    if stats:
        reached = _allreduce_counts(reached, dev, cm)
    return out, reached, phases


def balanced_row_ranges(entry_begin, world: int):
    """Contiguous row ranges [(a, b)] of a scan's rows for `world` ranks, balanced by entries +
    rows (a row holds its vertex's OUT and IN entries, so this is the edge-balanced 1-D vertex
    partition of tgo_load_partition_rows; java PartitionedRun.rowRanges restates it): range r
    ends at the first row whose prefix weight reaches (r + 1) / world of the total."""
    eb = np.asarray(entry_begin, np.int64)
    nrows = len(eb) - 1
    prefix = eb + np.arange(nrows + 1, dtype=np.int64)       # entries + rows before row i
    total = int(prefix[-1])
    cuts = [0]
    for r in range(1, world):
        target = (total * r + world - 1) // world
        cuts.append(max(cuts[-1], min(nrows, int(np.searchsorted(prefix, target, side="left")))))
    cuts.append(nrows)
    return [(cuts[r], cuts[r + 1]) for r in range(world)]


def gathered_index(u, n_local: int, world: int, hot: int, span: int):
    """Position of global source u in the blocked gathered contribution vector
    (tgo_part_pr_blocked): rank-major hot slices [0, hot) first, then the cold slices
    [hot, span) — the layout the two all-gathers of distributed_pagerank produce."""
    u = np.asarray(u, np.int64)
    r, o = u // n_local, u % n_local
    return np.where(o < hot, r * hot + o, world * hot + r * (span - hot) + (o - hot))


def pagerank_layout(backend, group=None, comm=None):
    """(hot rows per rank H, active span A) agreed by every rank: A = max active rows
    (all-reduce MAX), H from the backend (0 = plain rank-major layout, A = n_local)."""
    cm = _comm(comm, group)
    world = cm.world
    t = torch.tensor([backend.active_rows()], dtype=torch.int64, device=backend.device)
    cm.all_reduce(t, op="max")
    span = int(t.item())
    hot = backend.pr_layout(world, span)
    return (hot, span) if hot > 0 else (0, backend.n_local)


def distributed_pagerank(backend, alpha: float, vertex_count: int, iterations: int, fetch: bool = True,
                         group=None, layout=None, overlap: bool = True, comm=None):
    """PageRankVertexProgram on a vertex-partitioned graph; returns local ranks.
      plain   : all_gather of the owned contributions (8 n_local B per rank) -> local update
      blocked : (pagerank_layout) cold slices [H, A) all-gathered first; the hot slices
                [0, H) all-gather asynchronously while the cold segments are gathered
                (pr_step_cold); then the hot pass finishes the update (pr_step_hot).  Rows
                past A hold no entries anywhere and are not exchanged."""
    if iterations == 0:
        return np.full(backend.n_local, np.nan) if fetch else None
    cm = _comm(comm, group)
    world = cm.world
    hot, span = layout if layout is not None else pagerank_layout(backend, comm=cm)
    contrib_local = _scratch(backend, "pr_local", backend.n_local, torch.float64)
    contrib_global = _scratch(backend, "pr_global", world * span, torch.float64)
    backend.pr_begin(alpha, vertex_count, iterations, contrib_local)
    for _ in range(2, iterations + 1):
        if hot == 0:
            cm.all_gather_into_tensor(contrib_global, contrib_local)
            backend.pr_step(contrib_global, contrib_local)
            continue
        cm.all_gather_into_tensor(contrib_global[world * hot:], contrib_local[hot:span])
        if not overlap:
            cm.all_gather_into_tensor(contrib_global[:world * hot], contrib_local[:hot])
            backend.pr_step(contrib_global, contrib_local)
            continue
        work = cm.all_gather_into_tensor(contrib_global[:world * hot], contrib_local[:hot], async_op=True)
        backend.pr_step_cold(contrib_global)
        work.wait()
        backend.pr_step_hot(contrib_global, contrib_local)
    if hot > 0:
        # the blocked layout's fixed-point passes are exact only inside a range: a message
        # outside it on ANY rank (+inf from a vertex whose row cut left it no OUT entry, NaN, ...)
        # and every rank runs the program again on the plain layout's fp64 gather
        bad = torch.tensor([backend.pr_exact_check()], dtype=torch.int64, device=backend.device)
        cm.all_reduce(bad, op="max")
        if int(bad.item()):
            backend.pr_plain(True)
            try:
                return distributed_pagerank(backend, alpha, vertex_count, iterations, fetch, layout=(0, backend.n_local),
                                            overlap=overlap, comm=cm)
            finally:
                backend.pr_plain(False)
    return backend.pr_end(fetch)

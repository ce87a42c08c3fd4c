#!/usr/bin/env python3
"""Bench: BFS GTEPS + PageRank s/iter on RMAT (BASELINE.json metric).

One step = one pass of the hot path over the synthetic graph resident in HBM:
  a 64-root BFS sweep (ShortestDistanceVertexProgram with unit weights over bothE, full
  hop depth = Graph500-style undirected BFS) + one PageRankVertexProgram run with
  iterations(20) (19 rank updates, alpha 0.85, N = 2^scale, parity cap on).
value = BFS GTEPS over the timed steps = sum of input edges with a reached endpoint
(m_R / 2 for bothE) / BFS wall time.  PageRank is reported as pagerank_s_per_iter.

N = 1: RMAT scale 24 on one MI355X (configs[2]).
N > 1: weak scaling, RMAT scale 24 + log2(N) (N = 8 -> scale 27, configs[3]), 1-D vertex
       partitioned, one process per GPU, RCCL exchanges (titan_amd/distributed.py).
Launch: python bench.py [--steps K --warmup W]; N > 1 via torch.distributed.run.
"""
from __future__ import annotations

import argparse
import json
import math
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

JSON_OUT = sys.stdout    # the one result line; the partitioned path moves fd 1 (see main)
HBM_PEAK_GBS = 8000.0   # MI355X_MICROARCH.md: HBM3E 8 TB/s peak (spec)
METRIC = "BFS GTEPS + PageRank s/iter, RMAT scale-24 (1 GPU) and scale-27 (1/2/4/8 GPU)"


def log(*a):
    if int(os.environ.get("RANK", "0")) == 0:
        print("[bench]", *a, file=sys.stderr, flush=True)


def host_cores():
    """CPUs this process may run on: the affinity mask, capped by a cgroup CPU quota
    (cpu.max) when one is set — on the GPU box os.cpu_count() shows the whole machine."""
    n = len(os.sched_getaffinity(0)) if hasattr(os, "sched_getaffinity") else (os.cpu_count() or 1)
    try:
        with open("/sys/fs/cgroup/cpu.max") as f:
            quota, period = f.read().split()[:2]
        if quota != "max":
            n = min(n, max(1, int(int(quota) // int(period))))
    except (OSError, ValueError):
        pass
    return max(1, n)


def parse():
    p = argparse.ArgumentParser()
    p.add_argument("--gpus", type=int, default=1)
    p.add_argument("--steps", type=int, default=3)
    p.add_argument("--warmup", type=int, default=1)
    p.add_argument("--scale", type=int, default=24, help="per-GPU scale; N GPUs run scale + log2(N)")
    p.add_argument("--edge-factor", type=int, default=16)
    p.add_argument("--roots", type=int, default=64)
    p.add_argument("--pr-iters", type=int, default=20)
    p.add_argument("--cpu-baseline", type=int, default=1, help="0 disables the oracle timing")
    p.add_argument("--cpu-threads", type=int, default=0, help="oracle threads (0 = every CPU this process may use)")
    p.add_argument("--rows-scale", type=int, default=20,
                   help="configs[1]: single-source BFS over byte-exact edgestore rows of this RMAT scale (0 = off)")
    p.add_argument("--sssp-roots", type=int, default=4, help="delta-stepping SSSP leg (configs[4]); 0 disables")
    p.add_argument("--delta", type=int, default=0, help="delta-stepping bucket width (0 = engine default)")
    p.add_argument("--layout", type=int, default=1,
                   help="partitioned path: degree-grouped device layout (tgo_part_layout); 0 = global ids as given")
    p.add_argument("--partitioned", action="store_true",
                   help="use the vertex-partitioned multi-GPU path even at N=1 (for testing it on one GPU)")
    p.add_argument("--native", type=int, default=1,
                   help="partitioned path: every program as one native call over RCCL (tgo_part_msbfs_run / "
                        "_bfs_run / _pagerank_run / _sssp_run); 0 = the Python level drivers")
    p.add_argument("--pr-exchange", choices=["ghost", "allgather"], default="ghost",
                   help="partitioned PageRank: ghost exchange (only the contributions a rank reads) or all-gather")
    p.add_argument("--balanced", type=int, default=1,
                   help="partitioned path: edge-balanced ranges (entries + vertices, SlotPartition); 0 = equal ranges")
    return p.parse_args()


PMC_FILE = os.path.join(ROOT, "profiles", "pmc_traffic.json")


def pmc_traffic(group):
    """HBM bytes per unit (one rank update / one 64-source sweep) from the committed PMC
    passes of this workload (scripts/gpu_pmc.sh -> scripts/pmc_traffic.py); None if absent.
    PMC counters cannot be read from inside a timed run, so they come from separate
    rocprofv3 --pmc runs of the same bench command."""
    try:
        with open(PMC_FILE) as f:
            ent = json.load(f).get(group)
    except (OSError, ValueError):
        return None, None
    if not ent:
        return None, None
    return ent["traffic_bytes"], ent


def roofline(kernel, achieved_gbs, unit_desc, group=None, alg_bytes=None):
    traffic, ent = pmc_traffic(group) if group else (None, None)
    r = {"kernel": kernel, "bound": "hbm", "achieved": round(achieved_gbs, 2), "peak": HBM_PEAK_GBS,
         "unit": "GB/s", "frac": round(achieved_gbs / HBM_PEAK_GBS, 4),
         "traffic": round(traffic) if traffic else None, "bytes_per_unit": unit_desc}
    if alg_bytes:
        r["algorithmic_bytes"] = round(alg_bytes)
    if ent:
        r["traffic_detail"] = {"source": os.path.relpath(PMC_FILE, ROOT), "fetch_bytes_raw": round(ent["fetch_bytes_raw"]),
                               "write_bytes": round(ent["write_bytes"]), "l2_hit_rate": ent.get("l2_hit_rate"),
                               "ea_read_requests": ent.get("ea_read_requests"), "correction": ent["correction"]}
    return r


def result_line(args, world, scale, n, m, roots, elapsed, teps, hmean, pr_s_iter, e_in, roof_bfs, roof_pr,
                bfs_share, cpu, parallelism):
    return {
        "metric": METRIC,
        "value": round(teps / 1e9, 4),
        "unit": "GTEPS",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": round(elapsed / args.steps * 1e3, 3),
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "int32 (BFS levels); f64 (PageRank)",
        "data": "synthetic RMAT (Graph500 A/B/C=0.57/0.19/0.19, ef16, seeded), 64 seeded roots",
        "config": {"workload": f"rmat{scale}-msbfs{len(roots)}-bothE+pagerank{args.pr_iters}", "scale": scale,
                   "edge_factor": args.edge_factor, "vertices": n, "edges": int(m), "roots": len(roots),
                   "pr_iterations": args.pr_iters, "parallelism": parallelism},
        "bfs_mode": "multi-source (64 ShortestDistance programs per sweep, bit-parallel frontiers)",
        "single_source_gteps_hmean": round(hmean / 1e9, 4) if hmean else None,
        "pagerank_s_per_iter": round(pr_s_iter, 6),
        "pagerank_edges_per_s": round(e_in / pr_s_iter, 1),
        "bfs_share_of_step": round(bfs_share, 3),
        "roofline": roof_bfs if bfs_share >= 0.5 else roof_pr,
        "roofline_bfs": roof_bfs,
        "roofline_pagerank": roof_pr,
        "cpu_baseline": cpu,
    }


# ----------------------------------------------------------------------------- 1 GPU
def run_single(args):
    import torch
    from titan_amd import Engine, pick_roots, rmat_edges
    from titan_amd import _lib as L
    scale = args.scale
    n = 1 << scale
    cores = host_cores()
    t0 = time.perf_counter()
    src, dst, _ = rmat_edges(scale, args.edge_factor, seed=0x54495441)
    m = len(src)
    roots = pick_roots(n, src, dst, args.roots, seed=7)
    log(f"rmat scale {scale}: n={n} m={m} generated in {time.perf_counter() - t0:.1f}s ({cores} host cores)")
    load = {}
    t0 = time.perf_counter()
    bfs_eng = Engine(device=0, host_threads=cores).load_edges(n, src, dst, L.SCOPE_BOTH_E, apply_cap=False)
    load["bfs_bothE_wall_ms"] = round((time.perf_counter() - t0) * 1e3, 1)
    load["bfs_bothE_engine_ms"] = round(bfs_eng.stats()["load_ms"], 1)
    log(f"bfs graph (bothE, uncapped) loaded in {time.perf_counter() - t0:.1f}s")
    t0 = time.perf_counter()
    pr_eng = Engine(device=0, host_threads=cores).load_edges(n, src, dst, L.SCOPE_IN_E, apply_cap=True)
    pst = pr_eng.stats()
    load["pagerank_inE_wall_ms"] = round((time.perf_counter() - t0) * 1e3, 1)
    load["pagerank_inE_engine_ms"] = round(pst["load_ms"], 1)
    log(f"pagerank graph (inE, capped: {pst['truncated_results']} truncated rows) loaded in "
        f"{time.perf_counter() - t0:.1f}s")
    # per-root reached counts (untimed): m_R, n_R for GTEPS and algorithmic bytes
    bfs_eng.bfs_multi(roots, n, L.SCOPE_BOTH_E, seed_is_dense=True, stats=True, fetch=False)
    nR, mR = bfs_eng.multi_stats(len(roots))
    # self-check (untimed): two of the sweep's sources against their single-source runs
    import ctypes as C
    ms = np.empty(n, np.int64)
    checked = 0
    for i in (0, len(roots) - 1):
        bfs_eng.lib.tgo_copy_multi_distances(bfs_eng.ctx, i, L.ptr(ms, C.c_int64))
        checked += int(np.array_equal(ms, bfs_eng.bfs(int(roots[i]), n, L.SCOPE_BOTH_E, seed_is_dense=True)))
    # single-source side measurement (untimed, Graph500 style: every one of the 64 roots)
    ss_t, depth0 = [], 1
    for i, r in enumerate(roots):
        bfs_eng.bfs(int(r), n, L.SCOPE_BOTH_E, seed_is_dense=True, fetch=False)
        t = time.perf_counter()
        bfs_eng.bfs(int(r), n, L.SCOPE_BOTH_E, seed_is_dense=True, fetch=False)
        ss_t.append(time.perf_counter() - t)
        if i == 0:
            depth0 = bfs_eng.stats()["levels"]
    ss_hmean = len(ss_t) / float(np.sum(np.array(ss_t) / (mR[:len(ss_t)] / 2.0)))

    def step():
        t = time.perf_counter()
        bfs_eng.bfs_multi(roots, n, L.SCOPE_BOTH_E, seed_is_dense=True, fetch=False)
        bt = time.perf_counter() - t
        bk = bfs_eng.stats()["last_kernel_ms"] / 1e3
        t = time.perf_counter()
        pr_eng.pagerank(0.85, n, args.pr_iters, fetch=False)
        return bt, bk, time.perf_counter() - t, pr_eng.stats()["last_kernel_ms"] / 1e3

    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize()
    T0 = time.perf_counter()
    res = [step() for _ in range(args.steps)]
    torch.cuda.synchronize()
    elapsed = time.perf_counter() - T0
    bts = np.array([r[0] for r in res])
    bks = np.array([r[1] for r in res])
    pts = np.array([r[2] for r in res])
    pks = np.array([r[3] for r in res])
    edges_in = mR / 2.0                      # Graph500 undirected count for bothE
    teps = float(edges_in.sum()) * args.steps / float(bts.sum())
    # roofline of the multi-source sweep: every reached vertex's entries and offsets read
    # once (4*E_R + 16*n_R) + the 64 levels of every vertex written once as P bit planes
    # (P = bits of the deepest level: 8*P bytes per vertex)
    nR_u = int(nR.max())
    e_all = int(mR.max())
    planes = max(1, int(bfs_eng.stats()["levels"]).bit_length())
    ms_bytes = 4.0 * e_all + 16.0 * nR_u + 8.0 * planes * n
    roof_bfs = roofline("msbfs sweep (64 sources, all level launches)", ms_bytes / bks.mean() / 1e9,
                        f"4*E + 16*n_R + 8*P*n per 64-source sweep (P = {planes} level bit planes)", "msbfs_sweep",
                        ms_bytes)
    hmean = ss_hmean
    depth = np.array([depth0])
    upd = max(args.pr_iters - 1, 1)
    e_in = int(pst["in_entries"])
    pr_bytes = 4.0 * e_in + 8.0 * (n + 1) + 24.0 * n
    roof_pr = roofline("pagerank_update (cache-blocked, fixed-point tile sums: cold_fx + cold_fold + gather_hot_fx + long rows)",
                       pr_bytes / (pks.mean() / upd) / 1e9,
                       "4*m + 8*(n+1) + 24*n per update", "pagerank_update", pr_bytes)
    bfs_share = float(bts.sum()) / (float(bts.sum()) + float(pts.sum()))
    del pr_eng, bfs_eng
    sssp = sssp_leg(args, n, src, dst, roots, cores) if args.sssp_roots > 0 else None
    rows_leg = config2_rows_leg(args, cores) if args.rows_scale > 0 else None
    cpu = None
    if args.cpu_baseline:
        # levels counts the final empty level; the eccentricity is one less
        cpu = cpu_baseline(args, n, src, dst, roots, mR, max(int(depth[0]) - 1, 1),
                           args.cpu_threads or cores, pr_s_iter_gpu=float(pks.mean()) / upd)
    line = result_line(args, 1, scale, n, m, roots, elapsed, teps, hmean, float(pts.mean()) / upd, e_in,
                       roof_bfs, roof_pr, bfs_share, cpu, "single")
    line["load"] = load
    line["validation"] = {"msbfs_vs_single_source": f"{checked}/2 sources bit-exact (untimed self-check); "
                                                    "full-size oracle parity: tests/test_gpu_fullsize.py"}
    line["sssp"] = sssp
    line["config2_rows"] = rows_leg
    print(json.dumps(line), flush=True)


def config2_rows_leg(args, cores):
    """configs[1]: RMAT scale 20 as byte-exact edgestore rows (what the scan hands to
    VertexJobConverter), fed to tgo_load_rows in readBatchSize work blocks, then
    single-source BFS (bothE, Graph500 style) from 64 seeded roots.  Reports the decode +
    CSR assembly + upload time separately from the traversal."""
    from titan_amd import Engine, Schema, pick_roots, rmat_edges, synth_rows
    from titan_amd import _lib as L
    scale = args.rows_scale
    n = 1 << scale
    src, dst, _ = rmat_edges(scale, args.edge_factor, seed=0x54495441)
    roots = pick_roots(n, src, dst, args.roots, seed=7)
    label = (1 << 6) | 21                      # IDManager.getSchemaId(UserEdgeLabel, 1)
    t0 = time.perf_counter()
    rows = synth_rows(n, src, dst, None, label_id=label, threads=cores)
    encode_s = time.perf_counter() - t0
    vid = ((roots >> 5) + 1) << 5
    vid = (vid + (roots & 31)) << 3             # IDManager.constructId(i/32 + 1, i%32), pb = 5
    schema = Schema([{"type_id": label, "multiplicity": 0}], [])
    # the host decoder once, for comparison (same rows, same work blocks; untimed for GTEPS)
    os.environ["TGO_HOST_DECODE"] = "1"
    t0 = time.perf_counter()
    Engine(device=0, host_threads=cores).load_rows(rows, schema, L.SCOPE_BOTH_E, batch_rows=10 * 1024)
    host_load_s = time.perf_counter() - t0
    os.environ.pop("TGO_HOST_DECODE")
    t0 = time.perf_counter()
    eng = Engine(device=0, host_threads=cores).load_rows(rows, schema, L.SCOPE_BOTH_E, batch_rows=10 * 1024)
    load_s = time.perf_counter() - t0
    st = eng.stats()
    nbytes, nent = int(rows.byte_begin[-1]), int(rows.entry_begin[-1])
    del rows
    t_all, mR = [], []
    for r in vid:
        eng.bfs(int(r), n, L.SCOPE_BOTH_E, stats=True, fetch=False)
        mR.append(eng.stats()["reached_entries"])
        t = time.perf_counter()
        eng.bfs(int(r), n, L.SCOPE_BOTH_E, fetch=False)
        t_all.append(time.perf_counter() - t)
    mR = np.array(mR, np.float64) / 2.0
    t_all = np.array(t_all)
    return {"workload": f"rmat{scale}-edgestore-rows-bothE-single-source-bfs", "roots": len(vid),
            "rows": int(st["num_vertices"]), "entries": nent, "row_bytes": nbytes,
            "rows_encode_s": round(encode_s, 3),
            "load_rows_ms": round(load_s * 1e3, 1), "engine_load_ms": round(st["load_ms"], 1),
            "decode": "device (decode.hip), work blocks of 10240 rows",
            "load_rows_ms_host_decode": round(host_load_s * 1e3, 1),
            "decode_entries_per_s": round(nent / load_s, 1),
            "gteps_hmean": round(len(t_all) / float(np.sum(t_all / mR)) / 1e9, 4),
            "ms_per_root": round(float(t_all.mean()) * 1e3, 3)}


def sssp_leg(args, n, src, dst, roots, cores=16):
    """configs[4] on one GPU: delta-stepping SSSP (ShortestDistanceVertexProgram, inE scope,
    int32 weights w = 1 + splitmix64 mod 255, parity cap on) from a few of the BFS roots on
    the same RMAT graph; GTEPS = pull entries of reached vertices / device time."""
    from titan_amd import Engine, rmat_edges
    from titan_amd import _lib as L
    _, _, w = rmat_edges(args.scale, args.edge_factor, seed=0x54495441, weights=True)
    eng = Engine(device=0, host_threads=cores).load_edges(n, src, dst, L.SCOPE_IN_E, weight=w, apply_cap=True)
    del w
    res = []
    for r in roots:
        if len(res) == args.sssp_roots:
            break
        eng.sssp(int(r), n, L.SCOPE_IN_E, mode=L.SSSP_DELTA, seed_is_dense=True, stats=True, fetch=False,
                 delta=args.delta)
        st = eng.stats()
        if st["reached"] * 4 < n:        # directed scope: skip roots whose reach is not the giant component
            continue
        t = time.perf_counter()
        eng.sssp(int(r), n, L.SCOPE_IN_E, mode=L.SSSP_DELTA, seed_is_dense=True, fetch=False, delta=args.delta)
        wall = time.perf_counter() - t
        res.append((st["reached_entries"], st["relaxed_entries"], eng.stats()["last_kernel_ms"] / 1e3, wall,
                    st["levels"]))
    mR = np.array([x[0] for x in res], np.float64)
    dev = np.array([x[2] for x in res])
    wall = np.array([x[3] for x in res])
    return {"workload": f"rmat{args.scale}-weighted-inE-delta-sssp", "roots": len(res),
            "gteps_hmean": round(len(res) / float(np.sum(wall / mR)) / 1e9, 4),
            "ms_per_root": round(float(wall.mean()) * 1e3, 3), "device_ms_per_root": round(float(dev.mean()) * 1e3, 3),
            "reached_entries": int(mR.mean()), "relaxed_entries": int(np.mean([x[1] for x in res])),
            "phases": int(np.mean([x[4] for x in res]))}


# ----------------------------------------------------------------------------- N GPUs
def run_partitioned(args, world, rank, local_rank):
    import ctypes as C
    import torch
    import torch.distributed as dist
    from titan_amd import Engine
    from titan_amd import _lib as L
    from titan_amd.distributed import (PR_EXCHANGE_ALLGATHER, PR_EXCHANGE_GHOST, HipPartBackend, NativeExchange,
                                       SlotPartition, all_gather_layout, balanced_partition, distributed_bfs,
                                       distributed_bfs_native, distributed_msbfs, distributed_msbfs_native,
                                       distributed_pagerank, distributed_pagerank_native, entry_imbalance,
                                       exchange_stream, pagerank_layout, partition_range, pick_roots_partitioned,
                                       word_weights)
    torch.cuda.set_device(local_rank)
    dist.init_process_group("nccl", device_id=torch.device("cuda", local_rank))
    dev = torch.device("cuda", local_rank)
    scale = args.scale + int(round(math.log2(world)))
    n = 1 << scale
    m = args.edge_factor << scale
    lib = L.load()

    def edges_of(lo, hi):
        """The RMAT stream's edges with an endpoint in [lo, hi), generated and selected on this
        rank's GPU (tgo_rmat_partition_device; the host stream of tgo_rmat_partition)."""
        t0 = time.perf_counter()
        cap = int(2.3 * m * (hi - lo) / n) + (1 << 22)
        src = np.empty(cap, np.int32)
        dst = np.empty(cap, np.int32)
        wgt = np.empty(cap, np.int32) if args.sssp_roots > 0 else None
        cnt = C.c_int64()
        rc = lib.tgo_rmat_partition_device(scale, args.edge_factor, 0x54495441, lo, hi, L.ptr(src, C.c_int32),
                                           L.ptr(dst, C.c_int32), L.ptr(wgt, C.c_int32), cap, C.byref(cnt), local_rank)
        if rc:
            raise RuntimeError(f"tgo_rmat_partition rc={rc} count={cnt.value} cap={cap}")
        log(f"rmat scale {scale} partition [{lo},{hi}) of {world}: {cnt.value} edges in "
            f"{time.perf_counter() - t0:.1f}s")
        return src[:cnt.value], dst[:cnt.value], (wgt[:cnt.value] if wgt is not None else None)

    # Edge-balanced ranges: the words of the equal ranges are weighed (entries +
    # vertices) and all-gathered, every rank cuts the same balanced bounds, then takes the
    # edges of its own range.  The exchanges run over equal slots (SlotPartition): the edges
    # are handed to the engine in slot ids, results and roots map back to caller ids.
    elo, ehi = partition_range(n, world, rank)
    src, dst, wgt = edges_of(elo, ehi)
    if args.balanced:
        part, ww = balanced_partition(src, dst, n, elo, ehi, dev)
    else:
        part = SlotPartition.equal(n, world)
        loc = torch.from_numpy(word_weights(src, dst, elo, ehi)).to(dev)
        wg = torch.empty(n // 64, dtype=torch.int64, device=dev)
        dist.all_gather_into_tensor(wg, loc)
        ww = wg.cpu().numpy()
    lo, hi = part.range(rank)
    if (lo, hi) != (elo, ehi):
        del src, dst, wgt
        src, dst, wgt = edges_of(lo, hi)
    # the one-GPU bench's roots (tgo_pick_roots over the whole edge list), from partition edges
    roots = pick_roots_partitioned(n, src, dst, lo, hi, args.roots, 7, dev, part=part)
    ns, (slo, shi) = part.n_slots, part.slot_range(rank)
    src, dst = part.to_slots(src), part.to_slots(dst)
    roots_s = [int(x) for x in part.to_slots(np.asarray(roots, np.int64))]
    stream = exchange_stream()     # kernels and RCCL collectives ordered on one (non-default) stream
    t0 = time.perf_counter()
    lay = all_gather_layout(src, dst, ns, slo, shi, dev) if args.layout else None
    bfs_be = HipPartBackend(Engine(device=local_rank, host_threads=16, stream=stream)
                            .load_partition(ns, slo, shi, src, dst, L.SCOPE_BOTH_E, apply_cap=False, layout=lay),
                            ns, slo, shi, device_counts=True)
    pr_eng = Engine(device=local_rank, host_threads=16, stream=stream).load_partition(ns, slo, shi, src, dst,
                                                                                    L.SCOPE_IN_E, apply_cap=True,
                                                                                    layout=lay)
    pr_be = HipPartBackend(pr_eng, ns, slo, shi)
    pr_layout = pagerank_layout(pr_be)       # cache-blocked hot-first exchange (tgo_part_pr_blocked)
    log(f"partition graphs loaded in {time.perf_counter() - t0:.1f}s")
    # per-rank owned entries of the bothE graph: the partition's load imbalance (max / mean)
    ent = bfs_be.e.stats()
    rank_entries, imbalance = entry_imbalance(int(ent["out_entries"] + ent["in_entries"]), dev)
    # the sweep: one native call whose level loop issues RCCL collectives on the engine stream
    # (tgo_part_msbfs_run), or the Python level driver
    xchg = NativeExchange.rccl(local_rank) if args.native else None

    def sweep(stats):
        if xchg is not None:
            return distributed_msbfs_native(bfs_be, roots_s, ns, xchg, stats=stats)
        return distributed_msbfs(bfs_be, roots_s, ns, stats=stats)
    # per-root reached entries (untimed) for GTEPS
    _, mR, depth_ms = sweep(True)
    # single-source side measurement (untimed, every root, Graph500 style harmonic mean)
    ss_t = []

    def single(r):
        if xchg is not None:
            return distributed_bfs_native(bfs_be, r, ns, xchg, fetch=False, stats=False)
        return distributed_bfs(bfs_be, r, ns, fetch=False, stats=False)
    single(roots_s[0])
    for r in roots_s:
        torch.cuda.synchronize()
        t = time.perf_counter()
        single(r)
        torch.cuda.synchronize()
        ss_t.append(time.perf_counter() - t)
    pr_mode = PR_EXCHANGE_GHOST if args.pr_exchange == "ghost" else PR_EXCHANGE_ALLGATHER
    pr_moved = [0]

    def pagerank():
        if xchg is not None:
            _, pr_moved[0] = distributed_pagerank_native(pr_be, 0.85, n, args.pr_iters, xchg, mode=pr_mode, fetch=False)
        else:
            distributed_pagerank(pr_be, 0.85, n, args.pr_iters, fetch=False, layout=pr_layout)
    hmean = len(ss_t) / float(np.sum(np.array(ss_t) / (mR[:len(ss_t)] / 2.0)))

    def step():
        t = time.perf_counter()
        sweep(False)
        torch.cuda.synchronize()
        bt = time.perf_counter() - t
        t = time.perf_counter()
        pagerank()
        torch.cuda.synchronize()
        return bt, time.perf_counter() - t

    for _ in range(args.warmup):
        step()
    dist.barrier()
    torch.cuda.synchronize()
    T0 = time.perf_counter()
    res = [step() for _ in range(args.steps)]
    torch.cuda.synchronize()
    dist.barrier()
    elapsed = time.perf_counter() - T0
    bts = np.array([r[0] for r in res])
    pts = np.array([r[1] for r in res])
    t = torch.tensor([elapsed, float(bts.sum()), float(pts.mean())], dtype=torch.float64, device="cuda")
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    elapsed, bfs_wall, pr_wall = [float(x) for x in t.cpu()]
    e_loc = torch.tensor([float(pr_eng.stats()["in_entries"])], dtype=torch.float64, device="cuda")
    dist.all_reduce(e_loc)
    e_in = int(e_loc.item())
    planes = max(1, int(depth_ms).bit_length())      # level bit planes the sweeps wrote
    del pr_be, pr_eng
    sssp = None
    if wgt is not None:
        sssp = sssp_leg_partitioned(args, world, rank, local_rank, ns, slo, shi, src, dst, wgt, roots_s, stream, lay,
                                    n, xchg)
    if rank == 0:
        edges_in = mR / 2.0
        teps = float(edges_in.sum()) * args.steps / bfs_wall
        upd = max(args.pr_iters - 1, 1)
        # per-GPU algorithmic bytes over wall time (the exchange is inside the time)
        bfs_bytes = (4.0 * float(mR.max()) + 16.0 * n + 8.0 * planes * n) / world
        roof_bfs = roofline("msbfs sweep per GPU (local kernels + RCCL exchange)", bfs_bytes * args.steps / bfs_wall / 1e9,
                            f"(4*E + 16*n + 8*P*n)/N per 64-source sweep per GPU (P = {planes} level bit planes)")
        pr_bytes = (4.0 * e_in + 32.0 * n) / world
        roof_pr = roofline("pagerank_update per GPU (gather + all-gather)", pr_bytes / (pr_wall / upd) / 1e9,
                           "(4*m + 32*n)/N per update per GPU")
        bfs_share = bfs_wall / (bfs_wall + pr_wall * args.steps)
        line = result_line(args, world, scale, n, m, roots, elapsed, teps, hmean, pr_wall / upd, e_in,
                           roof_bfs, roof_pr, bfs_share, None, f"vertex-partition{world}")
        line["config"]["device_layout"] = "degree-grouped per rank" if args.layout else "global ids"
        line["config"]["msbfs_driver"] = ("native level loops, RCCL on the engine stream (tgo_part_msbfs_run / "
                                          "_bfs_run / _pagerank_run / _sssp_run)"
                                          if args.native else "Python level drivers (titan_amd/distributed.py)")
        line["pagerank_exchange"] = {"hot_rows_per_rank": pr_layout[0], "active_span": pr_layout[1],
                                     "mode": args.pr_exchange if args.native else "allgather (Python driver)",
                                     "allgather_bytes_per_rank_per_update": 8 * pr_layout[1] * (world - 1),
                                     "received_bytes_rank0_per_update": (pr_moved[0] // upd if args.native
                                                                         else 8 * pr_layout[1] * (world - 1))}
        wr = part.weights(ww)
        line["partition"] = {"ranges": ("edge-balanced 64-aligned ranges (entries + vertices) in equal exchange slots"
                                        if args.balanced else "equal 64-aligned vertex ranges of the seeded relabel"),
                             "bounds": [int(x) for x in part.bounds], "slot": part.slot,
                             "rank_entries": rank_entries, "entry_imbalance_max_over_mean": round(imbalance, 4),
                             "weight_imbalance_max_over_mean": round(max(wr) / (sum(wr) / len(wr)), 4)}
        line["sssp"] = sssp
        print(json.dumps(line), file=JSON_OUT, flush=True)
    torch.cuda.synchronize()
    del xchg                        # the native driver's RCCL communicator, before torch's group
    dist.barrier()
    dist.destroy_process_group()


def sssp_leg_partitioned(args, world, rank, local_rank, n, lo, hi, src, dst, wgt, roots, stream, lay, n_real, xchg=None):
    """configs[4] over N GPUs: delta-stepping SSSP on the vertex-partitioned weighted graph
    (inE scope, no preload cap), per-owner relaxation exchange over RCCL
    (titan_amd/distributed.distributed_sssp); roots whose reach is the giant component.
    n, lo, hi, src, dst, roots: slot ids (SlotPartition); n_real: the graph's vertices."""
    import torch
    import torch.distributed as dist
    from titan_amd import Engine
    from titan_amd import _lib as L
    from titan_amd.distributed import HipPartBackend, distributed_sssp, distributed_sssp_native

    def run(r, stats):
        if xchg is not None:
            return distributed_sssp_native(be, r, xchg, args.delta, fetch=False, stats=stats)
        return distributed_sssp(be, r, args.delta, fetch=False, stats=stats)
    eng = Engine(device=local_rank, host_threads=16, stream=stream).load_partition(n, lo, hi, src, dst, L.SCOPE_IN_E,
                                                                                 weight=wgt, apply_cap=False,
                                                                                 layout=lay)
    be = HipPartBackend(eng, n, lo, hi)
    res = []
    for r in roots:
        if len(res) == args.sssp_roots:
            break
        _, reached, _ = run(int(r), True)
        if reached[0] * 4 < n_real:
            continue
        torch.cuda.synchronize()
        dist.barrier()
        t = time.perf_counter()
        _, _, phases = run(int(r), False)
        torch.cuda.synchronize()
        wall = torch.tensor([time.perf_counter() - t], dtype=torch.float64, device="cuda")
        dist.all_reduce(wall, op=dist.ReduceOp.MAX)
        res.append((int(reached[1]), float(wall.item()), phases))
    if not res:
        return None
    mR = np.array([x[0] for x in res], np.float64)
    wall = np.array([x[1] for x in res])
    return {"workload": f"rmat{int(math.log2(n_real))}-weighted-inE-delta-sssp-partitioned", "roots": len(res),
            "gteps_hmean": round(len(res) / float(np.sum(wall / mR)) / 1e9, 4),
            "ms_per_root": round(float(wall.mean()) * 1e3, 3), "reached_entries": int(mR.mean()),
            "phases": int(np.mean([x[2] for x in res]))}


def cpu_baseline(args, n, src, dst, roots, mR, depth, threads, pr_s_iter_gpu=None):
    """The oracle (C restatement of Fulgora: every vertex executes every superstep and looks
    up each neighbour's message in a hash map by Titan id, as FulgoraVertexMemory does) on
    bounded samples of the same workload, on this host's cores:
      bfs      : root 0 of the sweep, bothE, maxDepth = its eccentricity (complete result)
      pagerank : iterations(3) on the capped inE graph -> seconds per superstep
      sssp     : 4 hop-bounded supersteps of the weighted inE program -> seconds per superstep
    Row decode / preload is timed apart (the reference pays it in EVERY superstep)."""
    out = {"value": None, "unit": "GTEPS", "cores": threads, "kind": "port"}
    try:
        sys.path.insert(0, os.path.join(ROOT, "oracle"))
        import fulgora as fr
        from titan_amd import rmat_edges
        t0 = time.perf_counter()
        g = fr.OracleGraph.from_edges(n, src, dst)
        load_s = time.perf_counter() - t0
        t0 = time.perf_counter()
        # maxDepth = the root's BFS depth: the reference runs iterations 0..maxDepth, and
        # this is the smallest maxDepth that yields the full BFS result.
        d, it = g.shortest_distance(int((int(roots[0]) + 1) << 3), int(depth), 2, weighted=False, threads=threads)
        t = time.perf_counter() - t0
        del g
        out["value"] = round(float(mR[0]) / 2.0 / t / 1e9, 6)
        out["sample"] = (f"BFS: 1 of {len(roots)} roots (root 0), same RMAT graph, bothE, maxDepth {depth} "
                         f"({it + 1} supersteps, {t:.1f}s); PageRank: iterations(3) (4 supersteps) on the capped inE "
                         f"graph; SSSP: maxDepth 3 (4 supersteps) weighted inE; edge-list preload timed apart")
        out["bfs"] = {"gteps": out["value"], "seconds": round(t, 3), "supersteps": it + 1,
                      "preload_s": round(load_s, 2)}
        _, _, w = rmat_edges(args.scale, args.edge_factor, seed=0x54495441, weights=True)
        t0 = time.perf_counter()
        g = fr.OracleGraph.from_edges(n, src, dst, w, hard_limit=100000)
        load_s = time.perf_counter() - t0
        del w
        t0 = time.perf_counter()
        g.pagerank(0.85, n, 3, threads=threads)
        t = time.perf_counter() - t0
        pr = {"s_per_superstep": round(t / 4, 4), "supersteps": 4, "preload_s": round(load_s, 2)}
        if pr_s_iter_gpu:
            pr["gpu_speedup_per_update"] = round(t / 4 / pr_s_iter_gpu, 1)
        out["pagerank_s_per_iter"] = pr
        t0 = time.perf_counter()
        g.shortest_distance(int((int(roots[0]) + 1) << 3), 3, 1, weighted=True, threads=threads)
        t = time.perf_counter() - t0
        out["sssp"] = {"s_per_superstep": round(t / 4, 4), "supersteps": 4}
        del g
    except Exception as e:  # noqa: BLE001
        out["sample"] = f"failed: {e}"
    return out


def main():
    args = parse()
    world = int(os.environ.get("WORLD_SIZE", "1"))
    if args.partitioned and "RANK" not in os.environ:     # one rank without a launcher
        import socket
        sk = socket.socket()
        sk.bind(("127.0.0.1", 0))
        port = sk.getsockname()[1]
        sk.close()
        os.environ.update(RANK="0", LOCAL_RANK="0", WORLD_SIZE="1", MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    if world > 1 or args.partitioned:
        # RCCL prints its version banner on fd 1: route native stdout to stderr and keep the
        # real stdout for the single JSON result line.
        global JSON_OUT
        sys.stdout.flush()
        JSON_OUT = os.fdopen(os.dup(1), "w")
        os.dup2(2, 1)
        run_partitioned(args, world, int(os.environ.get("RANK", "0")), int(os.environ.get("LOCAL_RANK", "0")))
    else:
        run_single(args)


if __name__ == "__main__":
    main()

#!/usr/bin/env python3
"""Bench: BFS GTEPS + PageRank s/iter on RMAT (BASELINE.json metric, configs[2]).

One step = one pass of the hot path over the synthetic graph resident in HBM:
  64-root BFS sweep (ShortestDistanceVertexProgram with unit weights over bothE, full
  hop depth = Graph500-style undirected BFS) + one PageRankVertexProgram run with
  iterations(20) (19 rank updates, alpha 0.85, N = 2^scale, parity cap on).
value = BFS GTEPS over the timed steps = sum of input edges with a reached endpoint
(m_R / 2 for bothE) / BFS wall time.  PageRank is reported as pagerank_s_per_iter.

Launch: python bench.py [--gpus 1 --steps K --warmup W]; N>1 via torch.distributed.run.
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

HBM_PEAK_GBS = 8000.0   # MI355X_MICROARCH.md: HBM3E 8 TB/s peak (spec)


def log(*a):
    if int(os.environ.get("RANK", "0")) == 0:
        print("[bench]", *a, file=sys.stderr, flush=True)


def parse():
    p = argparse.ArgumentParser()
    p.add_argument("--gpus", type=int, default=1)
    p.add_argument("--steps", type=int, default=3)
    p.add_argument("--warmup", type=int, default=1)
    p.add_argument("--scale", type=int, default=24)
    p.add_argument("--edge-factor", type=int, default=16)
    p.add_argument("--roots", type=int, default=64)
    p.add_argument("--pr-iters", type=int, default=20)
    p.add_argument("--cpu-baseline", type=int, default=1, help="0 disables the oracle timing")
    p.add_argument("--cpu-threads", type=int, default=16)
    return p.parse_args()


def main():
    args = parse()
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    import torch
    dist = None
    if world > 1:
        import torch.distributed as dist
        dist.init_process_group("gloo")
    from titan_amd import Engine, pick_roots, rmat_edges
    from titan_amd import _lib as L

    # Weak scaling: every rank keeps a scale-`args.scale` share (replicas until the
    # vertex-partitioned path lands; see DESIGN.md "Multi-GPU").
    scale = args.scale
    n = 1 << scale
    t0 = time.perf_counter()
    src, dst, _ = rmat_edges(scale, args.edge_factor, seed=0x54495441 + (rank if world > 1 else 0))
    m = len(src)
    roots = pick_roots(n, src, dst, args.roots, seed=7)
    log(f"rmat scale {scale}: n={n} m={m} generated in {time.perf_counter() - t0:.1f}s")

    t0 = time.perf_counter()
    bfs_eng = Engine(device=local_rank, host_threads=16).load_edges(n, src, dst, L.SCOPE_BOTH_E, apply_cap=False)
    log(f"bfs graph (bothE, uncapped) loaded in {time.perf_counter() - t0:.1f}s")
    t0 = time.perf_counter()
    pr_eng = Engine(device=local_rank, host_threads=16).load_edges(n, src, dst, L.SCOPE_IN_E, apply_cap=True)
    pst = pr_eng.stats()
    log(f"pagerank graph (inE, capped: {pst['truncated_results']} truncated rows) loaded in {time.perf_counter() - t0:.1f}s")

    # Per-root reached counts (untimed): m_R, n_R for GTEPS and algorithmic bytes.
    mR = np.zeros(len(roots), np.int64)
    nR = np.zeros(len(roots), np.int64)
    depth = np.zeros(len(roots), np.int64)
    for i, r in enumerate(roots):
        bfs_eng.bfs(int(r), n, L.SCOPE_BOTH_E, seed_is_dense=True, stats=True, fetch=False)
        st = bfs_eng.stats()
        mR[i], nR[i], depth[i] = st["reached_entries"], st["reached"], st["levels"]

    def step(timed):
        bt = np.zeros(len(roots))
        bk = np.zeros(len(roots))
        for i, r in enumerate(roots):
            t = time.perf_counter()
            bfs_eng.bfs(int(r), n, L.SCOPE_BOTH_E, seed_is_dense=True, fetch=False)
            bt[i] = time.perf_counter() - t
            bk[i] = bfs_eng.stats()["last_kernel_ms"] / 1e3
        t = time.perf_counter()
        pr_eng.pagerank(0.85, n, args.pr_iters, fetch=False)
        pt = time.perf_counter() - t
        pk = pr_eng.stats()["last_kernel_ms"] / 1e3
        return bt, bk, pt, pk

    for _ in range(args.warmup):
        step(False)
    if dist:
        dist.barrier()
    torch.cuda.synchronize() if torch.cuda.is_available() else None
    T0 = time.perf_counter()
    bts, bks, pts, pks = [], [], [], []
    for _ in range(args.steps):
        bt, bk, pt, pk = step(True)
        bts.append(bt); bks.append(bk); pts.append(pt); pks.append(pk)
    torch.cuda.synchronize() if torch.cuda.is_available() else None
    if dist:
        dist.barrier()
    elapsed = time.perf_counter() - T0
    bfs_wall = float(np.sum(bts))
    if dist:
        t = torch.tensor([elapsed, bfs_wall], dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed, bfs_wall = float(t[0]), float(t[1])

    edges_in = mR / 2.0                              # Graph500 undirected count for bothE
    teps_total = float(edges_in.sum()) * args.steps * world / bfs_wall
    per_root_t = np.mean(np.stack(bts), axis=0)
    hmean = len(roots) / float(np.sum(per_root_t / edges_in))
    # roofline: SURVEY.md §8(d) algorithmic bytes, per BFS root (all its level launches)
    bfs_bytes = 4.0 * mR + 8.0 * nR + 4.0 * n
    bfs_dev = np.mean(np.stack(bks), axis=0)
    bfs_achieved = float(bfs_bytes.sum() / bfs_dev.sum()) / 1e9
    upd = max(args.pr_iters - 1, 1)
    pr_s_iter = float(np.mean(pts)) / upd
    pr_dev_iter = float(np.mean(pks)) / upd
    # PageRank per update: in-CSR index 4m + offsets 8(n+1) + contributions read 8n +
    # rank write 8n + next contribution write 8n  
    res = {}
    if rank == 0:
        e_in = int(pst["in_entries"])
        pr_bytes = 4.0 * e_in + 8.0 * (n + 1) + 24.0 * n
        pr_achieved = pr_bytes / pr_dev_iter / 1e9
        bfs_share = float(np.sum(bts)) / (float(np.sum(bts)) + float(np.sum(pts)))
        roof_bfs = {"kernel": "bfs_root (all level launches of one root)", "bound": "hbm",
                    "achieved": round(bfs_achieved, 2), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                    "frac": round(bfs_achieved / HBM_PEAK_GBS, 4), "traffic": None,
                    "bytes_per_unit": "4*m_R + 8*n_R + 4*n per root"}
        roof_pr = {"kernel": "pagerank_update (gather_short + long-row chunks)", "bound": "hbm",
                   "achieved": round(pr_achieved, 2), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                   "frac": round(pr_achieved / HBM_PEAK_GBS, 4), "traffic": None,
                   "bytes_per_unit": "4*m + 8*(n+1) + 24*n per update"}
        dominant = roof_bfs if bfs_share >= 0.5 else roof_pr
        cpu = None
        if args.cpu_baseline:
            # levels counts the final empty level; the eccentricity is one less
            cpu = cpu_baseline(n, src, dst, roots, mR, max(int(depth[0]) - 1, 1), args.cpu_threads)
        res = {
            "metric": "BFS GTEPS + PageRank s/iter, RMAT scale-24 (1 GPU) and scale-27 (1/2/4/8 GPU)",
            "value": round(teps_total / 1e9, 4),
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
            "config": {"workload": f"rmat{scale}-bfs{len(roots)}-bothE+pagerank{args.pr_iters}",
                       "scale": scale, "edge_factor": args.edge_factor, "vertices": n, "edges": int(m),
                       "roots": len(roots), "pr_iterations": args.pr_iters,
                       "parallelism": "single" if world == 1 else f"replica{world}"},
            "gteps_hmean": round(hmean / 1e9, 4),
            "pagerank_s_per_iter": round(pr_s_iter, 6),
            "pagerank_edges_per_s": round(e_in / pr_s_iter, 1),
            "bfs_share_of_step": round(bfs_share, 3),
            "roofline": dominant,
            "roofline_bfs": roof_bfs,
            "roofline_pagerank": roof_pr,
            "cpu_baseline": cpu,
        }
        print(json.dumps(res), flush=True)
    if dist:
        dist.barrier()
        dist.destroy_process_group()


def cpu_baseline(n, src, dst, roots, mR, depth, threads):
    """Oracle (C restatement of Fulgora: every vertex every superstep, hash-map message
    lookup by Titan id) on ONE root of the same graph, timed on this host's cores."""
    try:
        sys.path.insert(0, os.path.join(ROOT, "oracle"))
        import fulgora as fr
        threads = max(1, min(threads, os.cpu_count() or 1))
        t0 = time.perf_counter()
        g = fr.OracleGraph.from_edges(n, src, dst)
        load_s = time.perf_counter() - t0
        t0 = time.perf_counter()
        # maxDepth = the root's BFS depth: the reference runs iterations 0..maxDepth, and
        # this is the smallest maxDepth that yields the full BFS result.
        d, it = g.shortest_distance(int((int(roots[0]) + 1) << 3), int(depth), 2, weighted=False, threads=threads)
        t = time.perf_counter() - t0
        reached_entries = float(mR[0])
        del g
        return {"value": round(reached_entries / 2.0 / t / 1e9, 6), "unit": "GTEPS", "cores": threads,
                "kind": "port", "sample": f"1 of {len(roots)} roots (root 0), same RMAT graph, bothE, full depth "
                                           f"({it} supersteps, {t:.1f}s; row decode/preload {load_s:.1f}s excluded)"}
    except Exception as e:  # noqa: BLE001
        return {"value": None, "unit": "GTEPS", "cores": threads, "kind": "port", "sample": f"failed: {e}"}


if __name__ == "__main__":
    main()

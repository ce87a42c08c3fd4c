#!/usr/bin/env python3
"""Per-source frontier sizes of the bench sweep (RMAT-24 bothE, 64 roots): for each level,
the frontier vertices and their entries per source (single-source BFS levels), to see how
unequal the 64 sources' frontiers are at the pull levels.
usage: python scripts/ms_sources.py [scale]"""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
from titan_amd import Engine, pick_roots, rmat_edges  # noqa: E402
from titan_amd import _lib as L  # noqa: E402

scale = int(sys.argv[1]) if len(sys.argv) > 1 else 24
n = 1 << scale
src, dst, _ = rmat_edges(scale, 16, seed=0x54495441)
deg = np.bincount(src, minlength=n) + np.bincount(dst, minlength=n)
roots = [int(r) for r in pick_roots(n, src, dst, 64, seed=7)]
eng = Engine(host_threads=16).load_edges(n, src, dst, L.SCOPE_BOTH_E, apply_cap=False)
del src, dst
per = []
for r in roots:
    d = eng.bfs(r, n, L.SCOPE_BOTH_E, seed_is_dense=True)
    lv = np.where(d >= 0, d, -1)
    per.append([(int((lv == k).sum()), int(deg[lv == k].sum())) for k in range(8)])
per = np.array(per)                     # [64, 8, 2]
tot = per[:, :, 1].sum(axis=0)
for k in range(8):
    e = np.sort(per[:, k, 1])
    print(f"level {k}: total entries {tot[k]:>11d}; per source min {e[0]} p10 {e[6]} p25 {e[16]} median {e[32]} "
          f"p75 {e[48]} max {e[-1]}; sources with < 1% of the level's mean: {(e < tot[k] / 64 / 100).sum()}",
          flush=True)

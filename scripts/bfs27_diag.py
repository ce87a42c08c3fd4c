#!/usr/bin/env python3
"""Diagnosis of multi-source vs single-source BFS disagreements on a large graph: for the
first seeds of the bench's 64, compare the multi-source sweep's levels, the direction-
optimizing single-source BFS and the hop-bounded Jacobi ShortestDistance (unit weights) —
three implementations; print mismatch counts and sample differences.
usage: python scripts/bfs27_diag.py [scale] [seeds]"""
import ctypes as C
import os
import sys

import numpy as np

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
from titan_amd import Engine, pick_roots, rmat_edges  # noqa: E402
from titan_amd import _lib as L  # noqa: E402

scale = int(sys.argv[1]) if len(sys.argv) > 1 else 27
k = int(sys.argv[2]) if len(sys.argv) > 2 else 8
n = 1 << scale
src, dst, _ = rmat_edges(scale, 16, seed=0x54495441)
roots = [int(r) for r in pick_roots(n, src, dst, 64, seed=7)]
deg = np.bincount(src, minlength=n) + np.bincount(dst, minlength=n)
eng = Engine(host_threads=16).load_edges(n, src, dst, L.SCOPE_BOTH_E, apply_cap=False)
del src, dst
eng.bfs_multi(roots, n, L.SCOPE_BOTH_E, seed_is_dense=True, fetch=False)
ms = np.empty(n, np.int64)
A = L.DIST_ABSENT
for i in range(k):
    eng.lib.tgo_copy_multi_distances(eng.ctx, i, L.ptr(ms, C.c_int64))
    bf = eng.bfs(roots[i], n, L.SCOPE_BOTH_E, seed_is_dense=True)
    lv_bfs = eng.stats()["levels"]
    hb = eng.sssp(roots[i], 16, L.SCOPE_BOTH_E, mode=L.SSSP_HOP_BOUNDED, seed_is_dense=True)
    d_ms_bf = np.flatnonzero(ms != bf)
    d_ms_hb = np.flatnonzero(ms != hb)
    d_bf_hb = np.flatnonzero(bf != hb)
    print(f"seed {i} root {roots[i]} deg {deg[roots[i]]}: bfs levels {lv_bfs}; mismatches ms/bfs {len(d_ms_bf)} "
          f"ms/hop {len(d_ms_hb)} bfs/hop {len(d_bf_hb)}; reached ms {(ms != A).sum()} bfs {(bf != A).sum()} "
          f"hop {(hb != A).sum()}", flush=True)
    for v in d_ms_bf[:6]:
        print(f"    v {v} (deg {deg[v]}): ms {ms[v]} bfs {bf[v]} hop {hb[v]}", flush=True)

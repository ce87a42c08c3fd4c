#!/usr/bin/env python3
"""Dev probe: BFS level trace + timing on RMAT for a few roots (TGO_TRACE=1 prints levels)."""
import os, sys, time
import numpy as np
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from titan_amd import Engine, pick_roots, rmat_edges
from titan_amd import _lib as L
scale = int(sys.argv[1]) if len(sys.argv) > 1 else 24
nroots = int(sys.argv[2]) if len(sys.argv) > 2 else 4
n = 1 << scale
src, dst, _ = rmat_edges(scale, 16, seed=0x54495441)
roots = pick_roots(n, src, dst, 64, seed=7)[:nroots]
eng = Engine(host_threads=16).load_edges(n, src, dst, L.SCOPE_BOTH_E, apply_cap=False)
for r in roots:
    eng.bfs(int(r), n, L.SCOPE_BOTH_E, seed_is_dense=True, stats=True, fetch=False)
    st = eng.stats()
    t = time.perf_counter()
    for _ in range(3):
        eng.bfs(int(r), n, L.SCOPE_BOTH_E, seed_is_dense=True, fetch=False)
    dt = (time.perf_counter() - t) / 3
    print(f"root {r}: levels {st['levels']} reached {st['reached']} m_R {st['reached_entries']} "
          f"dev {st['last_kernel_ms']:.2f} ms wall {dt*1e3:.2f} ms  GTEPS {st['reached_entries']/2/dt/1e9:.1f}", flush=True)

#!/usr/bin/env python3
"""Multi-source BFS sweep probe on the bench graph (RMAT scale 24, bothE, the bench's 64
roots): device ms per sweep (best of 3) and GTEPS; TGO_TRACE=1 prints the level plan.
Under `rocprofv3 --kernel-trace` the per-level kernels of the sweeps can be read in order.
usage: python scripts/ms_probe.py [scale] [sweeps]"""
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
from titan_amd import Engine, pick_roots, rmat_edges  # noqa: E402
from titan_amd import _lib as L  # noqa: E402

scale = int(sys.argv[1]) if len(sys.argv) > 1 else 24
sweeps = int(sys.argv[2]) if len(sys.argv) > 2 else 3
n = 1 << scale
src, dst, _ = rmat_edges(scale, 16, seed=0x54495441)
roots = [int(r) for r in pick_roots(n, src, dst, 64, seed=7)]
eng = Engine(host_threads=16).load_edges(n, src, dst, L.SCOPE_BOTH_E, apply_cap=False)
del src, dst
eng.bfs_multi(roots, n, L.SCOPE_BOTH_E, seed_is_dense=True, stats=True, fetch=False)
r, e = eng.multi_stats(len(roots))
edges = float(np.sum(e)) / 2.0
best = 1e9
for _ in range(sweeps):
    t = time.perf_counter()
    eng.bfs_multi(roots, n, L.SCOPE_BOTH_E, seed_is_dense=True, fetch=False)
    best = min(best, eng.stats()["last_kernel_ms"])
    wall = time.perf_counter() - t
print(f"msbfs scale {scale}: device {best:.3f} ms/sweep (wall {wall * 1e3:.3f}), levels {eng.stats()['levels']}, "
      f"GTEPS {edges / best / 1e6:.1f} reached {int(np.sum(r))} entries {int(np.sum(e))}  env={ {k: v for k, v in os.environ.items() if k.startswith('TGO_')} }",
      flush=True)

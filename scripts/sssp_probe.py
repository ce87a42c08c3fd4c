#!/usr/bin/env python3
"""Dev probe: delta-stepping SSSP on weighted RMAT over a sweep of bucket widths.
usage: sssp_probe.py [scale] [deltas comma-separated]"""
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from titan_amd import Engine, pick_roots, rmat_edges  # noqa: E402
from titan_amd import _lib as L  # noqa: E402

scale = int(sys.argv[1]) if len(sys.argv) > 1 else 24
deltas = [int(x) for x in (sys.argv[2] if len(sys.argv) > 2 else "0,16,32,64,128,256,512").split(",")]
n = 1 << scale
src, dst, w = rmat_edges(scale, 16, seed=0x54495441, weights=True)
roots = pick_roots(n, src, dst, 64, seed=7)
eng = Engine(host_threads=16).load_edges(n, src, dst, L.SCOPE_IN_E, weight=w, apply_cap=True)
good = []
for r in roots:
    eng.sssp(int(r), n, L.SCOPE_IN_E, mode=L.SSSP_DELTA, seed_is_dense=True, stats=True, fetch=False)
    if eng.stats()["reached"] * 4 >= n:
        good.append(int(r))
    if len(good) == 3:
        break
ref = eng.sssp(good[0], n, L.SCOPE_IN_E, mode=L.SSSP_DELTA, seed_is_dense=True, delta=1 << 40)
for d in deltas:
    t = []
    for r in good:
        eng.sssp(r, n, L.SCOPE_IN_E, mode=L.SSSP_DELTA, seed_is_dense=True, fetch=False, delta=d, stats=True)
        st = eng.stats()
        t0 = time.perf_counter()
        eng.sssp(r, n, L.SCOPE_IN_E, mode=L.SSSP_DELTA, seed_is_dense=True, fetch=False, delta=d)
        t.append((time.perf_counter() - t0, st["relaxed_entries"], st["reached_entries"], st["levels"]))
    chk = np.array_equal(ref, eng.sssp(good[0], n, L.SCOPE_IN_E, mode=L.SSSP_DELTA, seed_is_dense=True, delta=d))
    ms = np.mean([x[0] for x in t]) * 1e3
    print(f"delta {d:6d}: {ms:8.2f} ms/root  relaxed/reached {np.mean([x[1] / x[2] for x in t]):5.2f}  "
          f"phases {np.mean([x[3] for x in t]):6.1f}  GTEPS {np.mean([x[2] for x in t]) / ms / 1e6:6.2f}  exact={chk}",
          flush=True)

#!/usr/bin/env python3
"""Dev probe: RMAT-24 weighted inE delta SSSP (bench.py's configs[4] leg) on `nroots` roots that
reach a quarter of the graph, one run each after a warm-up run, printing the loop counters
(TGO_TRACE=1 adds the device loop's phase / bucket / extraction counts); SSSP_BINS=1,0 runs
the binned and the bitmap-scan loop (TGO_TUNE_DS_BINS), SSSP_PULL=0,0.01 the push and pull form
of finished buckets' heavy entries (TGO_TUNE_DS_PULL), and compares their distances.  Run it under
rocprofv3 --kernel-trace to split the time per kernel (scripts/ktrace.py).
usage: sssp_once.py [scale] [nroots]"""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from titan_amd import Engine, pick_roots, rmat_edges  # noqa: E402
from titan_amd import _lib as L  # noqa: E402

scale = int(sys.argv[1]) if len(sys.argv) > 1 else 24
nroots = int(sys.argv[2]) if len(sys.argv) > 2 else 1
n = 1 << scale
src, dst, w = rmat_edges(scale, 16, seed=0x54495441, weights=True, device=0)
roots = pick_roots(n, src, dst, 64, seed=7)
eng = Engine(host_threads=16).load_edges(n, src, dst, L.SCOPE_IN_E, weight=w, apply_cap=True)
del src, dst, w
good = []
for r in roots:
    eng.sssp(int(r), n, L.SCOPE_IN_E, mode=L.SSSP_DELTA, seed_is_dense=True, stats=True, fetch=False)
    if eng.stats()["reached"] * 4 >= n:
        good.append(int(r))
    if len(good) == nroots:
        break
# TGO_TUNE_DS_BINS values to run, each with the TGO_TUNE_DS_PULL fractions of SSSP_PULL
modes = [(int(x), float(p)) for x in os.environ.get("SSSP_BINS", "1").split(",")
         for p in os.environ.get("SSSP_PULL", "0").split(",")]
first = {}
for b, p in modes:
    eng.set_tuning(L.TUNE_DS_BINS, b).set_tuning(L.TUNE_DS_PULL, p)
    for r in good:
        eng.sssp(r, n, L.SCOPE_IN_E, mode=L.SSSP_DELTA, seed_is_dense=True, fetch=False)
        t0 = time.perf_counter()
        d = eng.sssp(r, n, L.SCOPE_IN_E, mode=L.SSSP_DELTA, seed_is_dense=True, stats=True)
        ms = (time.perf_counter() - t0) * 1e3
        st = eng.stats()
        same = first.setdefault(r, d) is d or (first[r] == d).all()
        print(f"bins={b} pull={p} root {r}: {ms:.2f} ms (incl. fetch), kernel {st['last_kernel_ms']:.2f} ms, phases {st['levels']}, "
              f"relaxed {st['relaxed_entries']}, reached_entries {st['reached_entries']}, "
              f"GTEPS(kernel) {st['reached_entries'] / st['last_kernel_ms'] / 1e6:.2f}, equal_first_mode={bool(same)}",
              flush=True)

#!/usr/bin/env python3
"""Load-phase trace at RMAT scale 27: the bothE and the capped inE
engine loads with TGO_TRACE=1 phase laps on stderr and the JSON trace of the load spans.
usage: TGO_TRACE=1 python scripts/load27_trace.py [scale] [out.json]"""
import os
import sys
import time

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
from titan_amd import Engine, rmat_edges, trace  # noqa: E402
from titan_amd import _lib as L  # noqa: E402

scale = int(sys.argv[1]) if len(sys.argv) > 1 else 27
out = sys.argv[2] if len(sys.argv) > 2 else None
if out:
    trace.enable(out)
n = 1 << scale
t0 = time.perf_counter()
src, dst, _ = rmat_edges(scale, 16, seed=0x54495441, device=0)
print(f"[load27] generated {len(src)} edges in {time.perf_counter() - t0:.1f} s", file=sys.stderr, flush=True)
for scope, cap, name in ((L.SCOPE_BOTH_E, False, "bothE"), (L.SCOPE_IN_E, True, "inE capped")):
    t0 = time.perf_counter()
    e = Engine(host_threads=16).load_edges(n, src, dst, scope, apply_cap=cap)
    print(f"[load27] {name} load {time.perf_counter() - t0:.2f} s ({e.stats()['device_bytes'] / 2**30:.1f} GiB)",
          file=sys.stderr, flush=True)
    del e
if out:
    trace.flush()

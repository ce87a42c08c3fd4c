#!/usr/bin/env python3
"""Dev probe: the 64-source sweep per level, one-GPU path (tgo_bfs_multi) against the
partitioned path at world 1 (tgo_part_msbfs_run over a one-rank local exchange), from the
program trace's device spans (msbfs.level / part.msbfs.level) plus the host wall time per sweep.
usage: ms_levels.py [scale] [sweeps]"""
import os
import sys
import tempfile
import time

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from titan_amd import Engine, pick_roots, rmat_edges, trace  # noqa: E402
from titan_amd import _lib as L  # noqa: E402
from titan_amd.distributed import HipPartBackend, NativeExchange, distributed_msbfs_native, local_layout  # noqa: E402

scale = int(sys.argv[1]) if len(sys.argv) > 1 else 24
sweeps = int(sys.argv[2]) if len(sys.argv) > 2 else 3
n = 1 << scale
src, dst, _ = rmat_edges(scale, 16, seed=0x54495441, device=0)
roots = [int(r) for r in pick_roots(n, src, dst, 64, seed=7)]
path = os.path.join(tempfile.mkdtemp(), "t.json")


def levels(name, fn):
    fn()                                            # warm-up
    trace.enable(path)
    trace.clear()
    wall = []
    for _ in range(sweeps):
        t = time.perf_counter()
        fn()
        wall.append((time.perf_counter() - t) * 1e3)
    trace.flush()
    trace.disable()
    ev = [e for e in trace.load_events(path) if e["name"] == name]
    per = {}
    for e in ev:
        per.setdefault(e["args"]["level"], []).append(e["dur"] / 1e3)
    out = {lv: float(np.median(v)) for lv, v in sorted(per.items())}
    return out, float(np.median(wall))


one = Engine(host_threads=16).load_edges(n, src, dst, L.SCOPE_BOTH_E, apply_cap=False)
a, wa = levels("msbfs.level", lambda: one.bfs_multi(roots, n, L.SCOPE_BOTH_E, seed_is_dense=True, fetch=False))
del one
# world 1 with the degree-grouped layout of its range (the bench's partitioned setup)
s = torch.cuda.Stream()
torch.cuda.set_stream(s)
lay = local_layout(src, dst, n, 0, n)
be = HipPartBackend(Engine(stream=s.cuda_stream, host_threads=16).load_partition(n, 0, n, src, dst, L.SCOPE_BOTH_E,
                                                                                 apply_cap=False, layout=lay),
                    n, 0, n, device_counts=True)
xs = NativeExchange.local_group(1)
b, wb = levels("part.msbfs.level", lambda: distributed_msbfs_native(be, roots, n, xs[0], stats=False))
print(f"one-GPU sweep {wa:.3f} ms wall, levels sum {sum(a.values()):.3f} ms")
print(f"partitioned world 1 sweep {wb:.3f} ms wall, levels sum {sum(b.values()):.3f} ms")
for lv in sorted(set(a) | set(b)):
    print(f"  level {lv}: one-GPU {a.get(lv, float('nan')):7.3f} ms   partitioned {b.get(lv, float('nan')):7.3f} ms")

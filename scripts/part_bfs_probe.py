#!/usr/bin/env python3
"""Partitioned single-source BFS at world 1 over RCCL (tgo_part_bfs_run, the native loop bench.py
runs at N > 1) next to the one-GPU tgo_bfs on the same RMAT bothE graph: kernel ms per root,
levels, and whether the levels agree.  Run under rocprofv3 --kernel-trace for the per-level
protocol.  usage: part_bfs_probe.py [scale] [roots]"""
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
from titan_amd import Engine, pick_roots, rmat_edges  # noqa: E402
from titan_amd import _lib as L  # noqa: E402
from titan_amd.distributed import (HipPartBackend, InProcessGroup, NativeExchange,  # noqa: E402
                                   distributed_bfs_native, local_layout)

scale = int(sys.argv[1]) if len(sys.argv) > 1 else 24
# PART_ALPHA / PART_BETA: the partitioned loop's direction switch (default: distributed.BFS_ALPHA / _BETA)
AB = {k: float(os.environ[e]) for k, e in (("alpha", "PART_ALPHA"), ("beta", "PART_BETA")) if e in os.environ}
nroots = int(sys.argv[2]) if len(sys.argv) > 2 else 4
n = 1 << scale
src, dst, _ = rmat_edges(scale, 16, seed=0x54495441, device=0)
roots = [int(r) for r in pick_roots(n, src, dst, 64, seed=7)]
one = Engine(host_threads=16).load_edges(n, src, dst, L.SCOPE_BOTH_E)
good, ref, t1 = [], {}, {}
for r in roots:
    d = one.bfs(r, n, L.SCOPE_BOTH_E, seed_is_dense=True, stats=True)
    if one.stats()["reached"] * 4 >= n:
        good.append(r)
        one.bfs(r, n, L.SCOPE_BOTH_E, seed_is_dense=True, fetch=False)
        ref[r] = d
        t1[r] = one.stats()["last_kernel_ms"]
        print(f"one-GPU root {r}: kernel {t1[r]:.3f} ms, levels {one.stats()['levels']}", flush=True)
    if len(good) == nroots:
        break
del one
st = torch.cuda.Stream()
tp = {}
with torch.cuda.stream(st):
    lay = local_layout(src, dst, n, 0, n)
    eng = Engine(stream=st.cuda_stream, host_threads=16).load_partition(n, 0, n, src, dst, L.SCOPE_BOTH_E, layout=lay)
    be = HipPartBackend(eng, n, 0, n)
    x = NativeExchange.rccl(0, comm=InProcessGroup(1).comm(0))
    for r in good:
        distributed_bfs_native(be, r, n, x, fetch=False, stats=False, **AB)            # warm
        torch.cuda.synchronize()
        t = time.perf_counter()
        distributed_bfs_native(be, r, n, x, fetch=False, stats=False, **AB)
        torch.cuda.synchronize()
        ms = (time.perf_counter() - t) * 1e3
        tp[r] = eng.stats()["last_kernel_ms"]
        d, _, lv = distributed_bfs_native(be, r, n, x, fetch=True, stats=False, **AB)
        print(f"partitioned world 1 root {r}: wall {ms:.3f} ms, kernel {tp[r]:.3f} ms, levels {lv}, "
              f"equal one-GPU {bool(np.array_equal(d, ref[r]))}", flush=True)
print(f"sum one-GPU {sum(t1.values()):.3f} ms, partitioned {sum(tp.values()):.3f} ms, "
      f"ratio {sum(t1.values()) / sum(tp.values()):.3f}", flush=True)

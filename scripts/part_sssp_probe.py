#!/usr/bin/env python3
"""Partitioned weighted delta SSSP at world 1 over RCCL (the native loop bench.py runs at N > 1,
tgo_part_sssp_run) next to the one-GPU device loop on the same RMAT graph: kernel ms per root,
phases, and whether the distances agree.  Run under rocprofv3 --kernel-trace to read the
per-phase protocol.  usage: part_sssp_probe.py [scale] [roots]"""
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
from titan_amd import Engine, pick_roots, rmat_edges  # noqa: E402
from titan_amd import _lib as L  # noqa: E402
from titan_amd.distributed import (HipPartBackend, InProcessGroup, NativeExchange,  # noqa: E402
                                   distributed_sssp_native, local_layout)

scale = int(sys.argv[1]) if len(sys.argv) > 1 else 24
nroots = int(sys.argv[2]) if len(sys.argv) > 2 else 2
n = 1 << scale
src, dst, w = rmat_edges(scale, 16, seed=0x54495441, weights=True, device=0)
roots = pick_roots(n, src, dst, 64, seed=7)
one = Engine(host_threads=16).load_edges(n, src, dst, L.SCOPE_IN_E, weight=w, apply_cap=True)
good = []
for r in roots:
    one.sssp(int(r), n, L.SCOPE_IN_E, mode=L.SSSP_DELTA, seed_is_dense=True, stats=True, fetch=False)
    if one.stats()["reached"] * 4 >= n:
        good.append(int(r))
    if len(good) == nroots:
        break
ref = {}
for r in good:
    ref[r] = one.sssp(r, n, L.SCOPE_IN_E, mode=L.SSSP_DELTA, seed_is_dense=True)
    print(f"one-GPU root {r}: kernel {one.stats()['last_kernel_ms']:.2f} ms, phases {one.stats()['levels']}", flush=True)
del one
st = torch.cuda.Stream()
with torch.cuda.stream(st):
    lay = local_layout(src, dst, n, 0, n)
    eng = Engine(stream=st.cuda_stream, host_threads=16).load_partition(n, 0, n, src, dst, L.SCOPE_IN_E, weight=w,
                                                                        apply_cap=True, layout=lay)
    be = HipPartBackend(eng, n, 0, n)
    x = NativeExchange.rccl(0, comm=InProcessGroup(1).comm(0))
    for r in good:
        distributed_sssp_native(be, r, x, fetch=False, stats=False)            # warm
        torch.cuda.synchronize()
        t = time.perf_counter()
        d, _, ph = distributed_sssp_native(be, r, x, fetch=True, stats=False)
        torch.cuda.synchronize()
        ms = (time.perf_counter() - t) * 1e3
        print(f"partitioned world 1 root {r}: wall {ms:.2f} ms, kernel {eng.stats()['last_kernel_ms']:.2f} ms, phases {ph}, "
              f"equal one-GPU {bool(np.array_equal(d, ref[r]))}", flush=True)

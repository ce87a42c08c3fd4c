#!/usr/bin/env python3
"""Dev probe: one-GPU vs partitioned (world size 1, RCCL) BFS on RMAT bothE with the same
roots — 64-source sweep and single-source per-root wall times, plus the partitioned
driver's per-level host time split.  usage: MASTER_ADDR=127.0.0.1 MASTER_PORT=29514
part_bfs_probe.py [scale]"""
import os
import sys
import time

import numpy as np
import torch
import torch.distributed as dist

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from titan_amd import Engine, pick_roots, rmat_edges  # noqa: E402
from titan_amd import _lib as L  # noqa: E402
from titan_amd import distributed as D  # noqa: E402

scale = int(sys.argv[1]) if len(sys.argv) > 1 else 24
n = 1 << scale
torch.cuda.set_device(0)
dist.init_process_group("nccl", rank=0, world_size=1, device_id=torch.device("cuda", 0))
src, dst, _ = rmat_edges(scale, 16, seed=0x54495441)
roots = [int(r) for r in pick_roots(n, src, dst, 64, seed=7)]
lay = D.local_layout(src, dst, n, 0, n)
st = D.exchange_stream()
be = D.HipPartBackend(Engine(stream=st, host_threads=16).load_partition(n, 0, n, src, dst, L.SCOPE_BOTH_E,
                                                                       apply_cap=False, layout=lay), n, 0, n,
                      device_counts=True)
one = Engine(host_threads=16).load_edges(n, src, dst, L.SCOPE_BOTH_E, apply_cap=False)


def timed(fn, reps=3):
    ts = []
    for _ in range(reps):
        torch.cuda.synchronize()
        t = time.perf_counter()
        fn()
        torch.cuda.synchronize()
        ts.append(time.perf_counter() - t)
    return float(np.median(ts)) * 1e3


print(f"msbfs sweep  one-GPU {timed(lambda: one.bfs_multi(roots, n, L.SCOPE_BOTH_E, seed_is_dense=True, fetch=False)):8.2f} ms"
      f"   partitioned {timed(lambda: D.distributed_msbfs(be, roots, n, stats=False)):8.2f} ms", flush=True)
t1 = np.mean([timed(lambda r=r: one.bfs(r, n, L.SCOPE_BOTH_E, seed_is_dense=True, fetch=False), 2) for r in roots[:16]])
t2 = np.mean([timed(lambda r=r: D.distributed_bfs(be, r, n, fetch=False, stats=False), 2) for r in roots[:16]])
print(f"single-source one-GPU {t1:8.3f} ms/root   partitioned {t2:8.3f} ms/root", flush=True)
one.bfs(roots[0], n, L.SCOPE_BOTH_E, seed_is_dense=True, stats=True, fetch=False)
print("one-GPU levels", one.stats()["levels"], flush=True)
_, _, lv = D.distributed_bfs(be, roots[0], n, fetch=False, stats=False)
print("partitioned levels", lv, flush=True)
_, _, lv = D.distributed_msbfs(be, roots, n, stats=False)
print("partitioned ms levels", lv, flush=True)
dist.destroy_process_group()

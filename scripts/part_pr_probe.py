#!/usr/bin/env python3
"""Dev probe: partitioned PageRank at world size 1 (RCCL), RMAT-24 inE, per-update time of
the exchange variants.  usage: MASTER_ADDR=127.0.0.1 MASTER_PORT=29513 part_pr_probe.py [scale]"""
import os
import sys
import time

import numpy as np
import torch
import torch.distributed as dist

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from titan_amd import Engine, rmat_edges  # noqa: E402
from titan_amd import _lib as L  # noqa: E402
from titan_amd.distributed import (HipPartBackend, distributed_pagerank, exchange_stream, local_layout,  # noqa: E402
                                   pagerank_layout)

scale = int(sys.argv[1]) if len(sys.argv) > 1 else 24
n = 1 << scale
torch.cuda.set_device(0)
dist.init_process_group("nccl", rank=0, world_size=1, device_id=torch.device("cuda", 0))
src, dst, _ = rmat_edges(scale, 16, seed=0x54495441)
lay = local_layout(src, dst, n, 0, n)
st = exchange_stream()
be = HipPartBackend(Engine(stream=st, host_threads=16).load_partition(n, 0, n, src, dst, L.SCOPE_IN_E, apply_cap=True,
                                                                     layout=lay), n, 0, n)
one = Engine(host_threads=16).load_edges(n, src, dst, L.SCOPE_IN_E, apply_cap=True)
blocked = pagerank_layout(be)
print("layout", blocked, flush=True)
iters = 20
for name, kw in (("plain", {"layout": (0, n)}), ("blocked-sync", {"layout": blocked, "overlap": False}),
                 ("blocked-overlap", {"layout": blocked, "overlap": True})):
    if name == "plain":
        os.environ["TGO_PR_BLOCKED"] = "0"
        be.pr_layout(1, blocked[1])           # switch the ctx to the plain layout
        os.environ.pop("TGO_PR_BLOCKED")
    else:
        be.pr_layout(1, blocked[1])
    ts = []
    for rep in range(4):
        torch.cuda.synchronize()
        t = time.perf_counter()
        pr = distributed_pagerank(be, 0.85, n, iters, fetch=rep == 3, **kw)
        torch.cuda.synchronize()
        ts.append(time.perf_counter() - t)
    ref = one.pagerank(0.85, n, iters)
    print(f"{name:16s} {np.median(ts[1:]) / (iters - 1) * 1e3:7.3f} ms/update   L1 vs one-GPU "
          f"{np.abs(pr - ref)[np.isfinite(ref)].sum():.2e}", flush=True)
t = []
for rep in range(4):
    t0 = time.perf_counter()
    one.pagerank(0.85, n, iters, fetch=False)
    t.append(time.perf_counter() - t0)
print(f"{'one-GPU':16s} {np.median(t[1:]) / (iters - 1) * 1e3:7.3f} ms/update", flush=True)
dist.destroy_process_group()

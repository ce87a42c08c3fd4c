#!/usr/bin/env python3
"""Consistency of a large assembled graph (RMAT-27 bothE: 2^31 entries per list): every row
sorted, OUT and IN lists transposes of each other (degree counts both ways), entry totals;
with "host" also array-identical to the host assembly (TGO_HOST_ASSEMBLY=1).
usage: python scripts/asm_check.py [scale] [host]"""
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
from titan_amd import Engine, rmat_edges  # noqa: E402
from titan_amd import _lib as L  # noqa: E402

scale = int(sys.argv[1]) if len(sys.argv) > 1 else 27
cmp_host = len(sys.argv) > 2 and sys.argv[2] == "host"
n = 1 << scale
src, dst, _ = rmat_edges(scale, 16, seed=0x54495441)
m = len(src)


def check(eng, tag):
    ok = True
    g = [eng.graph_csr(0), eng.graph_csr(1)]
    for d, c in enumerate(g):
        ok &= len(c["adj"]) == m and c["off"][-1] == m
        starts = np.zeros(m, bool)
        starts[c["off"][:-1][c["off"][:-1] < m]] = True
        dif = np.diff(c["adj"].astype(np.int64))
        ok &= bool(np.all((dif >= 0) | starts[1:]))
        print(f"[{tag}] list {d}: entries {len(c['adj'])}, rows sorted {bool(np.all((dif >= 0) | starts[1:]))}", flush=True)
        del dif, starts
    for d in (0, 1):
        cnt = np.bincount(g[d]["adj"], minlength=n)
        lens = np.diff(g[1 - d]["off"])
        same = bool(np.array_equal(cnt, lens))
        print(f"[{tag}] degrees of list {1 - d} == neighbour counts of list {d}: {same} "
              f"(mismatched rows {int(np.sum(cnt != lens))})", flush=True)
        ok &= same
    return ok, g


t = time.perf_counter()
dev = Engine(host_threads=16).load_edges(n, src, dst, L.SCOPE_BOTH_E, apply_cap=False)
print(f"device assembly load {time.perf_counter() - t:.1f} s", flush=True)
ok, gd = check(dev, "device")
pd = dev.graph_perm()
del dev
if cmp_host:
    os.environ["TGO_HOST_ASSEMBLY"] = "1"
    t = time.perf_counter()
    host = Engine(host_threads=16).load_edges(n, src, dst, L.SCOPE_BOTH_E, apply_cap=False)
    print(f"host assembly load {time.perf_counter() - t:.1f} s", flush=True)
    okh, gh = check(host, "host")
    same = bool(np.array_equal(pd, host.graph_perm())) and all(
        np.array_equal(gd[d][f], gh[d][f]) for d in (0, 1) for f in ("off", "adj"))
    print(f"device == host: {same}", flush=True)
    ok &= okh and same
print("CONSISTENT" if ok else "INCONSISTENT", flush=True)
sys.exit(0 if ok else 1)

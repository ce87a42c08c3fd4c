#!/usr/bin/env python3
"""The metric's scale-27 single-GPU anchor (BASELINE.json: "scale-27 (1/2/4/8 GPU)"):
RMAT-27 (n = 2^27, 2^31 input edges: 2^31 entries per direction, past int32 entry counts) on
ONE MI355X.  Loads the bothE BFS graph and the capped inE PageRank graph, runs the bench's
64-source sweep and PageRank(20), and checks full-size properties:
  * every one of the 64 multi-source BFS seeds equals its own single-source run (bit-exact);
  * PageRank(20) twice: bitwise identical ranks; sum of ranks in (0, 1];
prints one JSON line (timings, GTEPS, ms/update, load times, checks).
usage: python scripts/scale27_check.py [scale] [roots_checked]"""
import json
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
from titan_amd import Engine, pick_roots, rmat_edges  # noqa: E402
from titan_amd import _lib as L  # noqa: E402


def log(msg):
    print(f"[scale27] {msg}", file=sys.stderr, flush=True)


scale = int(sys.argv[1]) if len(sys.argv) > 1 else 27
nchk = int(sys.argv[2]) if len(sys.argv) > 2 else 64
n = 1 << scale
out = {"workload": f"rmat{scale}-msbfs64-bothE+pagerank20 (one GPU)", "scale": scale, "vertices": n}
t0 = time.perf_counter()
src, dst, _ = rmat_edges(scale, 16, seed=0x54495441)
out["edges"] = int(len(src))
out["gen_s"] = round(time.perf_counter() - t0, 1)
roots = [int(r) for r in pick_roots(n, src, dst, 64, seed=7)]
log(f"generated {len(src)} edges in {out['gen_s']} s")
t0 = time.perf_counter()
bfs = Engine(host_threads=16).load_edges(n, src, dst, L.SCOPE_BOTH_E, apply_cap=False)
st = bfs.stats()
out["load_bothE_s"] = round(time.perf_counter() - t0, 1)
out["bothE_entries"] = [int(st["out_entries"]), int(st["in_entries"])]
log(f"bothE loaded in {out['load_bothE_s']} s: {out['bothE_entries']} entries, {st['device_bytes'] / 2**30:.1f} GiB")
bfs.bfs_multi(roots, n, L.SCOPE_BOTH_E, seed_is_dense=True, stats=True, fetch=False)
_, mR = bfs.multi_stats(len(roots))
sw = []
for _ in range(3):
    bfs.bfs_multi(roots, n, L.SCOPE_BOTH_E, seed_is_dense=True, fetch=False)
    sw.append(bfs.stats()["last_kernel_ms"])
out["msbfs_sweep_ms"] = round(min(sw), 3)
out["msbfs_gteps"] = round(float(np.sum(mR)) / 2.0 / (min(sw) / 1e3) / 1e9, 1)
out["msbfs_levels"] = int(bfs.stats()["levels"])
log(f"sweep {out['msbfs_sweep_ms']} ms, {out['msbfs_gteps']} GTEPS")
import ctypes as C  # noqa: E402
ms = np.empty(n, np.int64)
ok, ss_ms = 0, []
for i in range(nchk):
    bfs.lib.tgo_copy_multi_distances(bfs.ctx, i, L.ptr(ms, C.c_int64))
    d = bfs.bfs(roots[i], n, L.SCOPE_BOTH_E, seed_is_dense=True)
    ss_ms.append(bfs.stats()["last_kernel_ms"])
    ok += int(np.array_equal(ms, d))
out["msbfs_seeds_equal_single_source"] = f"{ok}/{nchk}"
out["single_source_gteps_hmean"] = round(nchk / float(np.sum(np.array(ss_ms) / 1e3 / (mR[:nchk] / 2.0))) / 1e9, 1)
log(f"seeds equal: {ok}/{nchk}")
del bfs, ms
t0 = time.perf_counter()
pr = Engine(host_threads=16).load_edges(n, src, dst, L.SCOPE_IN_E, apply_cap=True)
out["load_inE_s"] = round(time.perf_counter() - t0, 1)
out["inE_truncated_rows"] = int(pr.stats()["truncated_results"])
del src, dst
log(f"inE loaded in {out['load_inE_s']} s, {out['inE_truncated_rows']} truncated rows")
a = pr.pagerank(0.85, n, 20)
t1 = pr.stats()["last_kernel_ms"]
b = pr.pagerank(0.85, n, 20)
t2 = pr.stats()["last_kernel_ms"]
out["pagerank_ms_per_update"] = round(min(t1, t2) / 19, 4)
out["pagerank_bitwise_reproducible"] = bool(np.array_equal(a, b))
fin = np.isfinite(a)
out["pagerank_sum"] = float(a[fin].sum())
out["pagerank_finite"] = int(fin.sum())
log(f"pagerank {out['pagerank_ms_per_update']} ms/update, bitwise {out['pagerank_bitwise_reproducible']}")
del pr, a, b
# configs[4]'s program at scale 27 on one GPU: weighted capped inE delta-stepping (the bench's
# sssp leg: roots whose reach is the giant component); the device-driven loop holds a scale-27
# queue since the 35-bit counter field (TGO_TRACE=1 prints "(device loop, ... piles)")
os.environ["TGO_TRACE"] = "1"
src, dst, w = rmat_edges(scale, 16, seed=0x54495441, weights=True)
t0 = time.perf_counter()
sp = Engine(host_threads=16).load_edges(n, src, dst, L.SCOPE_IN_E, weight=w, apply_cap=True)
out["load_weighted_inE_s"] = round(time.perf_counter() - t0, 1)
del src, dst, w
runs = []
for r in roots:
    d = sp.sssp(int(r), n, L.SCOPE_IN_E, mode=L.SSSP_DELTA, seed_is_dense=True, stats=True)
    st = sp.stats()
    if st["reached"] * 4 < n:
        continue
    sp.sssp(int(r), n, L.SCOPE_IN_E, mode=L.SSSP_DELTA, seed_is_dense=True, stats=True, fetch=False)
    st2 = sp.stats()
    runs.append({"root": int(r), "reached": int(st["reached"]), "reached_entries": int(st["reached_entries"]),
                 "relaxed_entries": int(st["relaxed_entries"]), "phases": int(st2["levels"]),
                 "ms": round(st2["last_kernel_ms"], 3),
                 "gteps": round(st["reached_entries"] / (st2["last_kernel_ms"] / 1e3) / 1e9, 2),
                 "repeat_equal": bool(np.array_equal(d, sp.sssp(int(r), n, L.SCOPE_IN_E, mode=L.SSSP_DELTA,
                                                                 seed_is_dense=True)))})
    log(f"sssp root {r}: {runs[-1]}")
    if len(runs) == 2:
        break
out["sssp_delta"] = runs
print(json.dumps(out), flush=True)
ok_all = ok == nchk and out["pagerank_bitwise_reproducible"] and 0 < out["pagerank_sum"] <= 1.0 + 1e-9 and \
    len(runs) == 2 and all(x["repeat_equal"] for x in runs)
sys.exit(0 if ok_all else 1)

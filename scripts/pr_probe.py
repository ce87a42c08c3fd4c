#!/usr/bin/env python3
"""PageRank gather variants on the bench graph (RMAT scale 24, inE, parity cap): device
ms per rank update for each TGO_PR_* setting, and whether the ranks stay bitwise equal to
the default path.  Diagnostic ranges (TGO_PR_DIAG=lo:hi) skip the gathers of sources
outside [lo, hi) — their ranks are wrong by design; they only attribute time.
usage: python scripts/pr_probe.py [scale] [iters]"""
import json
import os
import sys

import numpy as np

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
from titan_amd import Engine, rmat_edges  # noqa: E402
from titan_amd import _lib as L  # noqa: E402

scale = int(sys.argv[1]) if len(sys.argv) > 1 else 24
iters = int(sys.argv[2]) if len(sys.argv) > 2 else 20
n = 1 << scale
src, dst, _ = rmat_edges(scale, 16, seed=0x54495441)
eng = None
loaded_with = None
KEYS = ("TGO_PR_BLOCKED", "TGO_PR_HOT", "TGO_PR_SEG", "TGO_PR_DIAG", "TGO_PR_PACK", "TGO_PR_CPACK", "TGO_PR_HOT_TILE", "TGO_PR_HOT_PIPE",
        "TGO_PR_FX", "TGO_PR_FX_E", "TGO_PR_FX_COLD", "TGO_PR_FX_CE", "TGO_PR_FX_CP", "TGO_PR_FX_DIAG", "TGO_PR_FX_FOLD",
        "TGO_PR_FX_HROWS", "TGO_PR_FX_SPLIT", "TGO_PR_FX_SPLIT_AT")
variants = [
    {},
    {"TGO_PR_BLOCKED": "0"},
    {"TGO_PR_CPACK": "0"},
    {"TGO_PR_PACK": "0", "TGO_PR_CPACK": "0"},
    {"TGO_PR_HOT": "262144", "TGO_PR_SEG": "262144"},
    {"TGO_PR_HOT": "262144", "TGO_PR_SEG": "524288"},
    {"TGO_PR_DIAG": "-2:-1"},                 # no gathers at all: index stream + finalize
    {},
]
RELOAD = ("TGO_PR_BLOCKED", "TGO_PR_HOT", "TGO_PR_SEG", "TGO_PR_PACK", "TGO_PR_CPACK", "TGO_PR_HOT_TILE", "TGO_PR_HOT_PIPE",
          "TGO_PR_FX", "TGO_PR_FX_E", "TGO_PR_FX_COLD", "TGO_PR_FX_CE", "TGO_PR_FX_CP", "TGO_PR_FX_HROWS", "TGO_PR_FX_SPLIT", "TGO_PR_FX_SPLIT_AT")   # read at load time
if os.environ.get("PR_PROBE_DEFAULT_ONLY"):       # one variant: the TGO_PR_* settings of the caller's environment
    variants = [{k: os.environ[k] for k in KEYS if k in os.environ}]
if os.environ.get("PR_PROBE_VARIANTS"):        # a JSON list of env dicts, e.g. '[{}, {"TGO_PR_SEG": "393216"}]'
    variants = json.loads(os.environ["PR_PROBE_VARIANTS"])
base = None
out = []
for v in variants:
    for k in KEYS:
        os.environ.pop(k, None)
    os.environ.update(v)
    key = tuple(os.environ.get(k) for k in RELOAD)
    if key != loaded_with:
        eng = None
        eng = Engine(host_threads=16).load_edges(n, src, dst, L.SCOPE_IN_E, apply_cap=True)
        loaded_with = key
        print(json.dumps({"load": dict(zip(RELOAD, key)), "load_ms": round(eng.stats()["load_ms"], 1),
                          "device_bytes": eng.stats()["device_bytes"]}), flush=True)
    eng.pagerank(0.85, n, iters, fetch=False)          # warm
    times = []
    for _ in range(3):
        eng.pagerank(0.85, n, iters, fetch=False)
        times.append(eng.stats()["last_kernel_ms"] / (iters - 1))
    pr = eng.pagerank(0.85, n, iters)
    again = eng.pagerank(0.85, n, iters)
    if base is None:
        base = pr
    fin = np.isfinite(base)
    rec = {"variant": v or "default", "ms_per_update": round(min(times), 4), "ms_all": [round(t, 4) for t in times],
           "reproducible": bool(np.array_equal(pr, again)),
           "bitwise_equal_default": bool(np.array_equal(pr, base)), "l1_vs_default": float(np.abs(pr[fin] - base[fin]).sum())}
    out.append(rec)
    print(json.dumps(rec), flush=True)
if os.environ.get("PR_PROBE_SAVE"):           # a digest of the ranks' bytes (bitwise comparison across runs)
    import hashlib
    with open(os.environ["PR_PROBE_SAVE"], "w") as f:
        f.write(hashlib.sha256(np.ascontiguousarray(base).tobytes()).hexdigest() + "\n")

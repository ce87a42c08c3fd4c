#!/usr/bin/env python3
"""configs[1] load probe: RMAT scale 20 as edgestore rows through tgo_load_rows (device
decode, device assembly), three loads; TGO_TRACE=1 prints the finish-load phases.
usage: python scripts/rows_probe.py [scale]"""
import os
import sys
import time

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
from titan_amd import Engine, Schema, rmat_edges, synth_rows  # noqa: E402
from titan_amd import _lib as L  # noqa: E402

scale = int(sys.argv[1]) if len(sys.argv) > 1 else 20
n = 1 << scale
src, dst, _ = rmat_edges(scale, 16, seed=0x54495441)
label = (1 << 6) | 21
rows = synth_rows(n, src, dst, None, label_id=label, threads=16)
schema = Schema([{"type_id": label, "multiplicity": 0}], [])
for i in range(3):
    t0 = time.perf_counter()
    eng = Engine(device=0, host_threads=16).load_rows(rows, schema, L.SCOPE_BOTH_E, batch_rows=10 * 1024)
    wall = (time.perf_counter() - t0) * 1e3
    print(f"load {i}: wall {wall:.1f} ms, engine_load_ms {eng.stats()['load_ms']:.1f}", flush=True)
    del eng

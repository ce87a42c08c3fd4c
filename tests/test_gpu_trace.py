"""GPU: program tracing (titan_amd/csrc/trace.hpp) — every BFS level, multi-source level,
PageRank update (and its two phases), DegreeCounter superstep and delta-stepping step batch
is a device span with GPU timestamps and its level / iteration argument; the loads are host
spans with their assembly phases; roctx ranges on top do not disturb the programs."""
import numpy as np
import pytest

from titan_amd import Engine, rmat_edges, trace
from titan_amd import _lib as L

pytestmark = pytest.mark.gpu


def test_program_spans(tmp_path):
    path = str(tmp_path / "trace.json")
    scale = 12
    n = 1 << scale
    src, dst, w = rmat_edges(scale, 16, seed=91, weights=True)
    trace.enable(path, roctx=True)
    trace.clear()
    try:
        with trace.span("job"):
            both = Engine().load_edges(n, src, dst, L.SCOPE_BOTH_E)
            d = both.bfs(int(src[0]), n, L.SCOPE_BOTH_E, seed_is_dense=True)
            levels = both.stats()["levels"]
            both.bfs_multi([int(src[0]), int(dst[3])], n, L.SCOPE_BOTH_E, seed_is_dense=True, fetch=False)
            ms_levels = both.stats()["levels"]
            ine = Engine().load_edges(n, src, dst, L.SCOPE_IN_E, weight=w)
            pr = ine.pagerank(0.85, n, 10)
            ine.walkcount(3)
            ine.sssp(int(src[0]), n, L.SCOPE_IN_E, mode=L.SSSP_DELTA, seed_is_dense=True)
        trace.flush()
    finally:
        trace.disable()
    assert np.isfinite(pr).all() and (d != L.DIST_ABSENT).sum() > 1
    ev = trace.load_events(path)
    by = {}
    for e in ev:
        by.setdefault(e["name"], []).append(e)
    bl = by["bfs.level"]
    assert sorted(e["args"]["level"] for e in bl) == list(range(levels))
    assert all(e["cat"] == "device" and e["dur"] > 0 for e in bl)
    assert len(by["msbfs.level"]) == ms_levels
    upd = by["pagerank.update"]
    assert sorted(e["args"]["iteration"] for e in upd) == list(range(2, 11))
    # the phases sit inside their update
    for ph in by.get("pagerank.hot_phase", []):
        u = next(x for x in upd if x["args"]["iteration"] == ph["args"]["iteration"])
        assert u["ts"] - 1.0 <= ph["ts"] and ph["ts"] + ph["dur"] <= u["ts"] + u["dur"] + 1.0
    assert len(by["degree_counter.superstep"]) == 3
    assert len(by.get("sssp.delta_steps", [])) >= 1
    assert len(by["load.edges"]) == 2 and by["load.edges"][0]["cat"] == "host"
    assert any(k.startswith("assemble.") for k in by)
    job = by["job"][0]
    first = min(e["ts"] for e in ev if e["name"] != "job")
    assert job["ts"] <= first + 1.0                       # device spans land on the host timeline

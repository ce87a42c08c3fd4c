"""GPU: CSR assembly on the device (assemble.hip) against the host assembly (graph_build.cpp
assemble_from_edges) — array for array: the degree-grouped permutation, OUT / IN offsets,
neighbour ids, weights and column positions, the explicit push transpose of a cut load, and
the ScanMetrics counters.  Cases cover the untyped cut of single-direction scopes
(QueryContainer.java:28,122 at a small hard limit, so hubs are truncated and the transpose is
built), bothE (uncut), weights, TGO_LOAD_COLUMN_ORDER, caller Titan ids, duplicates and
self-loops (RMAT keeps them), isolated vertices and a vertex count that is not a power of 2."""
import numpy as np
import pytest

from titan_amd import Engine, rmat_edges
from titan_amd import _lib as L

pytestmark = pytest.mark.gpu


def _snapshot(eng):
    st = eng.stats()
    return {"perm": eng.graph_perm(), "out": eng.graph_csr(0), "in": eng.graph_csr(1), "push": eng.graph_csr(2),
            "counters": (st["num_vertices"], st["out_entries"], st["in_entries"], st["truncated_results"])}


def _load(monkeypatch, host, limit, **kw):
    if host:
        monkeypatch.setenv("TGO_HOST_ASSEMBLY", "1")
    else:
        monkeypatch.delenv("TGO_HOST_ASSEMBLY", raising=False)
    return _snapshot(Engine(hard_query_limit=limit).load_edges(**kw))


def _same(a, b):
    assert np.array_equal(a["perm"], b["perm"])
    assert a["counters"] == b["counters"]
    for k in ("out", "in", "push"):
        if a[k] is None or b[k] is None:
            assert a[k] is None and b[k] is None, k
            continue
        for f in ("off", "adj", "w", "col"):
            assert np.array_equal(a[k][f], b[k][f]), (k, f)


CASES = [
    # (name, scale, scope, cap, weights, column_order, titan_ids, limit)
    ("bothE", 12, L.SCOPE_BOTH_E, False, False, False, False, 100000),
    ("inE-cut", 12, L.SCOPE_IN_E, True, False, False, False, 40),
    ("outE-cut-weighted", 12, L.SCOPE_OUT_E, True, True, False, False, 33),
    ("inE-weighted-columns", 11, L.SCOPE_IN_E, True, True, True, True, 25),
    ("bothE-weighted-columns", 11, L.SCOPE_BOTH_E, True, True, True, False, 25),
    ("inE-uncut", 12, L.SCOPE_IN_E, False, True, False, True, 100000),
]


@pytest.mark.parametrize("name,scale,scope,cap,weights,cols,tids,limit", CASES, ids=[c[0] for c in CASES])
def test_device_assembly_equals_host(monkeypatch, name, scale, scope, cap, weights, cols, tids, limit):
    src, dst, w = rmat_edges(scale, 16, seed=61, weights=True)
    n = (1 << scale) + 37                       # isolated tail, not a power of two
    kw = dict(n=n, src=src, dst=dst, scope=scope, apply_cap=cap, column_order=cols)
    if weights:
        kw["weight"] = w
    if tids:
        kw["titan_ids"] = ((np.arange(n, dtype=np.int64) * 3 + 5) << 3) | 0
    host = _load(monkeypatch, True, limit, **kw)
    dev = _load(monkeypatch, False, limit, **kw)
    if cap and scope != L.SCOPE_BOTH_E:
        assert host["counters"][3] > 0 and host["push"] is not None    # the cut happened: transpose built
    _same(host, dev)


def test_device_assembly_at_bench_size(monkeypatch):
    """configs[2]'s PageRank graph (RMAT-24, inE, the real 100 000 cap: 25 truncated rows)
    and the bench BFS graph (bothE): device and host assembly array-identical."""
    scale = 24
    n = 1 << scale
    src, dst, _ = rmat_edges(scale, 16, seed=0x54495441)
    for scope, cap in ((L.SCOPE_IN_E, True), (L.SCOPE_BOTH_E, False)):
        kw = dict(n=n, src=src, dst=dst, scope=scope, apply_cap=cap)
        host = _load(monkeypatch, True, 100000, **kw)
        dev = _load(monkeypatch, False, 100000, **kw)
        _same(host, dev)
        if cap:
            assert dev["counters"][3] == 25
        del host, dev


def test_device_assembly_rejects_bad_input(monkeypatch):
    monkeypatch.delenv("TGO_HOST_ASSEMBLY", raising=False)
    from titan_amd.engine import TitanException
    with pytest.raises(TitanException):
        Engine().load_edges(8, np.array([0, 9], np.int32), np.array([1, 2], np.int32), L.SCOPE_BOTH_E)
    with pytest.raises(TitanException):
        Engine().load_edges(4, np.array([0], np.int32), np.array([1], np.int32), L.SCOPE_BOTH_E,
                            titan_ids=np.array([8, 16, 16, 24], np.int64))
    # no edges at all: every vertex isolated
    e = Engine().load_edges(70, np.zeros(0, np.int32), np.zeros(0, np.int32), L.SCOPE_IN_E)
    g = e.graph_csr(1)
    assert len(g["adj"]) == 0 and np.all(g["off"] == 0)
    assert np.array_equal(np.sort(e.graph_perm()), np.arange(70))


# ---------------------------------------------------------------- row loads (tgo_load_rows)
def _rows_both(monkeypatch, rows, sd, scope, limit, **kw):
    from titan_amd import Schema
    out = []
    for host in ("1", "0"):
        monkeypatch.setenv("TGO_HOST_ASSEMBLY", host)
        out.append(_snapshot(Engine(hard_query_limit=limit).load_rows(rows, Schema.from_dict(sd), scope, **kw)))
    monkeypatch.delenv("TGO_HOST_ASSEMBLY")
    return out


@pytest.mark.parametrize("scope", [L.SCOPE_IN_E, L.SCOPE_OUT_E, L.SCOPE_BOTH_E])
@pytest.mark.parametrize("cols", [False, True])
def test_device_row_assembly_equals_host(monkeypatch, scope, cols):
    """Edgestore rows (ghost rows, schema rows, a small cap so hub rows are cut, weights in
    the signature): device row assembly == host assemble_from_rows, array for array."""
    import sys
    import os
    sys.path.insert(0, os.path.dirname(__file__))
    from test_gpu_decode import rmat_rows
    rows, vids, sd, wkey, n = rmat_rows(with_w=True)
    h, d = _rows_both(monkeypatch, rows, sd, scope, 25, weight_key=wkey, batch_rows=77, column_order=cols)
    _same(h, d)
    if scope != L.SCOPE_BOTH_E:
        assert h["counters"][3] > 0


def test_device_row_assembly_typed_scopes(monkeypatch):
    """Typed scopes over DESC sort keys and SIMPLE labels (uncapped), weights: device == host."""
    import random
    import edgestore as es
    import fulgora as fr
    lib = fr.load()
    knows, likes = es.user_edge_label(1), es.user_edge_label(2)
    w, ks = lib.fr_schema_id(0, 1), lib.fr_schema_id(0, 2)
    pkeys = [(w, 3), (ks, 10)]
    sd = {"edge_types": [{"type_id": knows, "multiplicity": 0, "sort_key": [ks, w], "order": "DESC"},
                         {"type_id": likes, "multiplicity": 1, "signature": [ks, w]}],
          "property_keys": [list(p) for p in pkeys]}
    osch = fr.OracleSchema(sd["edge_types"], pkeys)
    rnd = random.Random(5)
    n = 300
    edges = [(rnd.randrange(n), rnd.randrange(n), rnd.choice([knows, likes]),
              [(w, rnd.randint(1, 30)), (ks, rnd.choice([0, 5, -8, 1234]))]) for _ in range(4000)]
    rows, vids = es.build_rows(es.GraphSpec(n=n, edges=edges), osch)
    for scope in (L.SCOPE_IN_E, L.SCOPE_OUT_E):
        for labels in ((), (knows,), (likes,)):
            h, d = _rows_both(monkeypatch, rows, sd, scope, 20, labels=labels, weight_key=w)
            _same(h, d)


def test_vertex_cut_rows_keep_the_host_assembly(monkeypatch):
    """Representative rows of vertex cuts fold on the host (graph_build.cpp): the device
    switch must not change that load (same arrays either way)."""
    import sys
    import os
    sys.path.insert(0, os.path.dirname(__file__))
    from conftest import load_fixture
    rows, vids, sd, npz = load_fixture("partition_groups")
    h, d = _rows_both(monkeypatch, rows, sd, L.SCOPE_BOTH_E, 100000, batch_rows=5)
    _same(h, d)


# ---------------------------------------------------------------- PageRank layout (pr_layout.hip)
@pytest.mark.parametrize("scale,hot,seg,tile", [(14, "1024", "512", None), (14, "600", "333", "8192"), (20, None, None, None)])
def test_device_pagerank_layout_bitwise(monkeypatch, scale, hot, seg, tile):
    """The cache-blocked PageRank layout built on the device (hot CSR, cold pieces, blocks,
    source-sorted packing of hot tiles and cold blocks) equals the host build: with the slot
    tiles (TGO_PR_FX=0) every sum runs in the same fixed order, so the ranks are bitwise
    identical.  The default device layout (fixed-point super-tiles and cold piece tiles, exact
    tile sums) is reproducible and within 1e-14 relative L1 of the slot form; both match the
    oracle."""
    import fulgora as fr
    for k, v in (("TGO_PR_HOT", hot), ("TGO_PR_SEG", seg), ("TGO_PR_HOT_TILE", tile)):
        if v is None:
            monkeypatch.delenv(k, raising=False)
        else:
            monkeypatch.setenv(k, v)
    n = 1 << scale
    src, dst, _ = rmat_edges(scale, 16, seed=71)
    res = []
    for host, fx in (("1", "0"), ("0", "0"), ("0", "1")):
        monkeypatch.setenv("TGO_HOST_ASSEMBLY", host)
        monkeypatch.setenv("TGO_PR_FX", fx)
        eng = Engine(hard_query_limit=300).load_edges(n, src, dst, L.SCOPE_IN_E, apply_cap=True)
        res.append(eng.pagerank(0.85, n, 12))
        if fx == "1":
            assert np.array_equal(res[-1], eng.pagerank(0.85, n, 12))      # exact sums: reproducible
    monkeypatch.delenv("TGO_HOST_ASSEMBLY")
    monkeypatch.delenv("TGO_PR_FX")
    assert np.array_equal(res[0], res[1])
    fin = np.isfinite(res[0])
    assert np.array_equal(np.isfinite(res[2]), fin)
    assert np.abs(res[2][fin] - res[0][fin]).sum() <= 1e-14 * np.abs(res[0][fin]).sum()
    if scale <= 14:
        opr, _ = fr.OracleGraph.from_edges(n, src, dst, hard_limit=300).pagerank(0.85, n, 12)
        fin = np.isfinite(opr)
        assert np.abs(res[1][fin] - opr[fin]).sum() <= 1e-6
        assert np.abs(res[2][fin] - opr[fin]).sum() <= 1e-6


PART_CASES = [
    # (name, scope, cap, weights, layout, limit)
    ("bothE", L.SCOPE_BOTH_E, False, False, False, 100000),
    ("bothE-layout", L.SCOPE_BOTH_E, False, False, True, 100000),
    ("inE-cut-layout", L.SCOPE_IN_E, True, False, True, 40),
    ("outE-cut-weighted", L.SCOPE_OUT_E, True, True, False, 33),
    ("inE-cut-weighted-layout", L.SCOPE_IN_E, True, True, True, 25),
    ("inE-weighted-uncut-layout", L.SCOPE_IN_E, False, True, True, 100000),
]


@pytest.mark.parametrize("name,scope,cap,weights,layout,limit", PART_CASES, ids=[c[0] for c in PART_CASES])
def test_device_partition_assembly_equals_host(monkeypatch, name, scope, cap, weights, layout, limit):
    """tgo_load_partition: the owned rows of a global edge list assembled on the device
    (assemble_partition_device) equal the host assembly array for array — offsets, global
    neighbour ids in column order, the cut, weights, the layout permutation — for every rank of
    a 3-way split with unequal 64-aligned ranges."""
    from titan_amd.distributed import local_layout
    scale = 12
    src, dst, w = rmat_edges(scale, 16, seed=67, weights=True)
    n = 1 << scale
    bounds = [0, 1344, 2688, n]
    lay = None
    if layout:
        lay = np.concatenate([local_layout(src, dst, n, bounds[r], bounds[r + 1]) for r in range(3)])
    for r in range(3):
        lo, hi = bounds[r], bounds[r + 1]
        snaps = []
        for host in (True, False):
            if host:
                monkeypatch.setenv("TGO_HOST_ASSEMBLY", "1")
            else:
                monkeypatch.delenv("TGO_HOST_ASSEMBLY", raising=False)
            eng = Engine(hard_query_limit=limit).load_partition(n, lo, hi, src, dst, scope,
                                                                 weight=w if weights else None, apply_cap=cap,
                                                                 layout=lay)
            snaps.append(_snapshot(eng))
        if cap:
            assert snaps[0]["counters"][3] > 0                 # rows were cut
        _same(snaps[0], snaps[1])

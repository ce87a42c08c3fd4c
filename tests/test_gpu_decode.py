"""GPU: the device row decoder (decode.hip) against the host decoder on the
same rows — the staging both produce is loaded and must give the same graph: ids, counters
(ghosts, truncated lists, skipped rows, vertex cuts) and traversal results; malformed rows
fail the same way.  TGO_HOST_DECODE=1 selects the host decoder (read on every call)."""
import random

import numpy as np
import pytest

import fulgora as fr
from conftest import load_fixture
from titan_amd import Engine, Schema, TitanException, rmat_edges
from titan_amd import _lib as L

pytestmark = pytest.mark.gpu
OUT, IN, BOTH = L.SCOPE_OUT_E, L.SCOPE_IN_E, L.SCOPE_BOTH_E
STAT_KEYS = ("num_vertices", "out_entries", "in_entries", "ghost_vertices", "truncated_results", "skipped_rows",
             "partitioned_vertices", "partition_rows", "ghost_partition_rows")


def load_both(monkeypatch, rows, sd, scope, limit=100000, **kw):
    out = []
    for host in ("1", "0"):
        monkeypatch.setenv("TGO_HOST_DECODE", host)
        out.append(Engine(hard_query_limit=limit).load_rows(rows, Schema.from_dict(sd), scope, **kw))
    monkeypatch.delenv("TGO_HOST_DECODE")
    return out


def assert_same(h, d, seeds, scope, n, weighted=False):
    for k in STAT_KEYS:
        assert h.stats()[k] == d.stats()[k], k
    assert np.array_equal(h.vertex_ids(), d.vertex_ids())
    for s in seeds:
        assert np.array_equal(h.bfs(int(s), n, scope), d.bfs(int(s), n, scope))
        if weighted:
            assert np.array_equal(h.sssp(int(s), 6, scope), d.sssp(int(s), 6, scope))


def rmat_rows(with_w=False, ghosts=True):
    import edgestore as es
    scale = 9
    src, dst, w = rmat_edges(scale, 8, seed=41, weights=True)
    n = 1 << scale
    knows = es.user_edge_label(1)
    wkey = (1 << 6) | 5
    sd = {"edge_types": [{"type_id": knows, "multiplicity": 0, "signature": [wkey] if with_w else []}],
          "property_keys": [[wkey, 3]]}
    osch = fr.OracleSchema(sd["edge_types"], [(wkey, 3)])
    edges = [(int(a), int(b), knows, [(wkey, int(x))] if with_w else []) for a, b, x in zip(src, dst, w)]
    spec = es.GraphSpec(n=n, edges=edges, schema_rows=3,
                        ghost_rows=[(es.vertex_id(n + 7), [(0, es.vertex_id(2), knows), (1, es.vertex_id(9), knows)])]
                        if ghosts else [])
    rows, vids = es.build_rows(spec, osch)
    return rows, vids, sd, wkey, n


@pytest.mark.parametrize("scope", [IN, OUT, BOTH])
@pytest.mark.parametrize("batch", [None, 77])
def test_rmat_rows_device_equals_host(monkeypatch, scope, batch):
    rows, vids, sd, wkey, n = rmat_rows(with_w=True)
    h, d = load_both(monkeypatch, rows, sd, scope, limit=25, weight_key=wkey, batch_rows=batch)
    if scope != BOTH:
        assert d.stats()["truncated_results"] > 0
    assert d.stats()["ghost_vertices"] == 1 and d.stats()["skipped_rows"] == 3     # the schema rows
    assert_same(h, d, vids[:4], scope, n, weighted=True)


def test_gotg_and_vertex_cuts_device_equals_host(monkeypatch):
    for name in ("gotg", "partition_groups"):
        rows, vids, sd, npz = load_fixture(name)
        for scope in (IN, BOTH):
            h, d = load_both(monkeypatch, rows, sd, scope, batch_rows=5)
            assert_same(h, d, vids[:3], scope, 12)
            if scope == IN:
                assert np.array_equal(h.walkcount(2), d.walkcount(2))


def test_typed_scope_and_sort_keys_device_equals_host(monkeypatch):
    import edgestore as es
    lib = fr.load()
    knows, likes = es.user_edge_label(1), es.user_edge_label(2)
    w, ks = lib.fr_schema_id(0, 1), lib.fr_schema_id(0, 2)
    pkeys = [(w, 3), (ks, 10)]
    sd = {"edge_types": [{"type_id": knows, "multiplicity": 0, "sort_key": [ks, w], "order": "DESC"},
                         {"type_id": likes, "multiplicity": 1, "signature": [ks, w]}],
          "property_keys": [list(p) for p in pkeys]}
    osch = fr.OracleSchema(sd["edge_types"], pkeys)
    rnd = random.Random(3)
    n = 300
    edges = [(rnd.randrange(n), rnd.randrange(n), rnd.choice([knows, likes]),
              [(w, rnd.randint(1, 30)), (ks, rnd.choice([0, 5, -8, 1234]))]) for _ in range(4000)]
    rows, vids = es.build_rows(es.GraphSpec(n=n, edges=edges), osch)
    for scope in (IN, OUT):
        for labels in ((), (knows,), (likes,)):
            h, d = load_both(monkeypatch, rows, sd, scope, limit=20, labels=labels, weight_key=w)
            assert_same(h, d, vids[:3], scope, n, weighted=True)


def test_malformed_rows_fail_alike(monkeypatch):
    rows, vids, sd, wkey, n = rmat_rows(ghosts=False)
    bad = type(rows)(rows.keys.copy(), rows.entry_begin.copy(), rows.byte_begin.copy(), rows.data.copy(),
                     rows.limit_valpos.copy())
    # corrupt the first user-edge entry of row 3: its relation-type byte names no known label
    r = next(i for i in range(rows.nrows) if rows.entry_begin[i + 1] - rows.entry_begin[i] >= 3)
    e1 = int(bad.entry_begin[r]) + 1
    start = int(bad.limit_valpos[e1 - 1]) >> 32
    bad.data[int(bad.byte_begin[r]) + start] = 0x7E
    codes = []
    for host in ("1", "0"):
        monkeypatch.setenv("TGO_HOST_DECODE", host)
        with pytest.raises(TitanException) as e:
            Engine().load_rows(bad, Schema.from_dict(sd), BOTH)
        codes.append(e.value.code)
    assert codes[0] == codes[1] == L.TGO_E_CODEC

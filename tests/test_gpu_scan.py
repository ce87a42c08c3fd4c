"""GPU: rows reach the engine through the scan contract — StandardScanner running the
CSR-collecting job (VertexJobConverter's queries: VERTEX_EXISTS_QUERY first, then the scope's
user-edge slice with the QueryContainer limit) — and the loaded graph equals a direct load of
the same rows: ids, ghost / truncated counters, traversal results."""
import numpy as np
import pytest

import fulgora as fr
from conftest import load_fixture
from titan_amd import Engine, Schema, rmat_edges
from titan_amd import _lib as L
from titan_amd.scan import InMemoryStore, scan_into_engine

pytestmark = pytest.mark.gpu
OUT, IN, BOTH = L.SCOPE_OUT_E, L.SCOPE_IN_E, L.SCOPE_BOTH_E


def by_id(ids, vals):
    return dict(zip((int(i) for i in ids), (int(v) for v in vals)))


@pytest.mark.parametrize("procs,block", [(1, 10000), (3, 17)])
@pytest.mark.parametrize("scope", [IN, OUT, BOTH])
def test_scan_equals_direct_load(scope, procs, block):
    import edgestore as es
    scale = 9
    src, dst, _ = rmat_edges(scale, 8, seed=99)
    n = 1 << scale
    knows = es.user_edge_label(1)
    sd = {"edge_types": [{"type_id": knows, "multiplicity": 0}], "property_keys": []}
    osch = fr.OracleSchema(sd["edge_types"], [])
    spec = es.GraphSpec(n=n, edges=[(int(a), int(b), knows, []) for a, b in zip(src, dst)],
                        ghost_rows=[(es.vertex_id(n + 5), [(0, es.vertex_id(3), knows)])], schema_rows=2)
    rows, vids = es.build_rows(spec, osch)
    direct = Engine(hard_query_limit=30).load_rows(rows, Schema.from_dict(sd), scope)
    scanned = Engine(hard_query_limit=30)
    m = scan_into_engine(scanned, InMemoryStore.from_rows(rows), Schema.from_dict(sd), scope, hard_limit=30,
                         num_processors=procs, work_block_size=block)
    assert m.get("failure") == 0
    sd_, ss_ = direct.stats(), scanned.stats()
    for k in ("num_vertices", "out_entries", "in_entries", "ghost_vertices", "truncated_results", "skipped_rows"):
        assert sd_[k] == ss_[k], k
    if scope != BOTH:
        assert ss_["truncated_results"] > 0          # the store applied the slice limit
    ids_d, ids_s = direct.vertex_ids(), scanned.vertex_ids()
    assert sorted(ids_d) == sorted(ids_s)
    for r in vids[:3]:
        assert by_id(ids_d, direct.bfs(int(r), n, scope)) == by_id(ids_s, scanned.bfs(int(r), n, scope))
    if scope == IN:
        assert by_id(ids_d, direct.walkcount(3)) == by_id(ids_s, scanned.walkcount(3))


def test_scan_gotg_ghost_and_typed_scope():
    rows, vids, sd, npz = load_fixture("gotg")
    names = list(npz["names"])
    for scope, seed, key in ((IN, "saturn", "bfs_in_saturn"), (BOTH, "jupiter", "bfs_both_jupiter")):
        eng = Engine()
        scan_into_engine(eng, InMemoryStore.from_rows(rows), Schema.from_dict(sd), scope, num_processors=2,
                         work_block_size=3)
        d = eng.bfs(int(vids[names.index(seed)]), 12, scope)
        got = by_id(eng.vertex_ids(), d)
        assert [-1 if got[int(v)] == L.DIST_ABSENT else got[int(v)] for v in vids] == [int(x) for x in npz[key]]
        assert eng.stats()["ghost_vertices"] == 1 and eng.stats()["skipped_rows"] == 1

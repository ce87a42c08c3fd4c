"""CPU: the product-side synthetic edgestore writer (tgo_synth_rows) and the oracle's capped
edge-list load, both pinned against independent restatements.

* tgo_synth_rows (titan_amd/csrc/synth_rows.cpp) must write the same bytes as the oracle's
  encoder driven by tests/edgestore.py (EdgeSerializer.writeRelation,
  EdgeSerializer.java:222-315; StaticArrayEntryList layout, StaticArrayEntryList.java:15-50).
* fr_load_edges_capped (oracle) must equal rows capped by plain numpy
  (QueryContainer.java:28,122: the user-edge slice cut in column order, OUT entries first).
* Rows written by tgo_synth_rows and decoded by the oracle's row path
  (VertexJobConverter.process, VertexJobConverter.java:109-129) give the same programs as the
  oracle's edge-list path.
"""
import numpy as np
import pytest

import edgestore as es
import fulgora as fr
from titan_amd import rmat_edges, synth_rows
from titan_amd import _lib as L

IN, OUT, BOTH = L.SCOPE_IN_E, L.SCOPE_OUT_E, L.SCOPE_BOTH_E


def oracle_encoded_rows(n, src, dst, w, pb=5):
    knows = es.user_edge_label(1)
    wkey = es.user_property_key(1)
    if w is None:
        sd = {"edge_types": [{"type_id": knows, "multiplicity": 0}], "property_keys": []}
        edges = [(int(a), int(b), knows, []) for a, b in zip(src, dst)]
    else:
        sd = {"edge_types": [{"type_id": knows, "multiplicity": 0, "signature": [wkey]}], "property_keys": [[wkey, 3]]}
        edges = [(int(a), int(b), knows, [(wkey, int(x))]) for a, b, x in zip(src, dst, w)]
    osch = fr.OracleSchema(sd["edge_types"], [tuple(x) for x in sd["property_keys"]])
    rows, vids = es.build_rows(es.GraphSpec(n=n, edges=edges), osch, pb=pb)
    return rows, vids, sd, osch, knows, wkey


@pytest.mark.parametrize("weighted", [False, True])
@pytest.mark.parametrize("scale,ef", [(7, 4), (10, 2)])
def test_synth_rows_match_oracle_encoder_bytes(weighted, scale, ef):
    n = 1 << scale
    src, dst, w = rmat_edges(scale, ef, seed=3, weights=True)
    # negative and large weights exercise the zig-zag varint lengths
    w = (w.astype(np.int64) * 9973 - 1_200_000).astype(np.int32)
    rows, vids, sd, osch, knows, wkey = oracle_encoded_rows(n, src, dst, w if weighted else None)
    got = synth_rows(n, src, dst, w if weighted else None, label_id=knows)
    for f in ("keys", "entry_begin", "byte_begin", "limit_valpos", "data"):
        assert np.array_equal(getattr(rows, f), getattr(got, f)), f


def test_synth_rows_other_partition_bits_and_loops():
    n = 200
    src = np.array([0, 5, 5, 199, 7, 7, 7], np.int32)          # duplicates and self-loops kept
    dst = np.array([0, 9, 9, 0, 7, 150, 3], np.int32)
    rows, *_ = oracle_encoded_rows(n, src, dst, None, pb=3)
    got = synth_rows(n, src, dst, None, partition_bits=3)
    for f in ("keys", "entry_begin", "byte_begin", "limit_valpos", "data"):
        assert np.array_equal(getattr(rows, f), getattr(got, f)), f


def test_synth_rows_rejects_bad_input():
    from titan_amd import TitanException
    with pytest.raises(TitanException):
        synth_rows(4, np.array([0], np.int32), np.array([4], np.int32))       # endpoint out of range
    with pytest.raises(TitanException):
        synth_rows(4, np.array([0], np.int32), np.array([1], np.int32), label_id=(1 << 6) | 5)   # a property key id


def numpy_capped(n, src, dst, limit):
    """Rows of (src, dst) as the commit path writes them, each cut at `limit` entries in
    column order (OUT entries, then IN entries, each by (neighbour, edge index))."""
    m = len(src)
    eidx = np.arange(m)
    o = np.lexsort((eidx, dst, src))
    i = np.lexsort((eidx, src, dst))
    owner = np.concatenate([src[o], dst[i]]).astype(np.int64)
    other = np.concatenate([dst[o], src[i]]).astype(np.int64)
    dirn = np.concatenate([np.zeros(m, np.int64), np.ones(m, np.int64)])
    order = np.lexsort((np.arange(2 * m), dirn, owner))      # per row: OUT run then IN run
    owner, other, dirn = owner[order], other[order], dirn[order]
    deg = np.bincount(owner, minlength=n)
    off = np.zeros(n + 1, np.int64)
    off[1:] = np.cumsum(deg)
    pos = np.arange(2 * m) - off[owner]
    keep = pos < limit
    cnt = np.minimum(deg, limit)
    noff = np.zeros(n + 1, np.int64)
    noff[1:] = np.cumsum(cnt)
    outs = np.bincount(owner[keep & (dirn == 0)], minlength=n)
    mid = noff[:-1] + outs
    return noff, mid, other[keep].astype(np.int32), int((deg >= limit).sum())


@pytest.mark.parametrize("limit", [7, 40, 10 ** 9])
def test_oracle_capped_edge_load_matches_numpy(limit):
    scale = 10
    n = 1 << scale
    src, dst, _ = rmat_edges(scale, 8, seed=21)
    ids = (np.arange(n, dtype=np.int64) + 1) << 3
    off, mid, adj, trunc = numpy_capped(n, src, dst, limit)
    ref = fr.OracleGraph.from_adjacency(ids, off, mid, adj)
    og = fr.OracleGraph.from_edges(n, src, dst, hard_limit=limit)
    assert og.stats.truncated_results == trunc
    eo, em, ea, _ = og.export()
    assert np.array_equal(eo, off) and np.array_equal(em, mid) and np.array_equal(ea, adj)
    for r in (0, 17, 500):
        assert np.array_equal(og.shortest_distance(int(ids[r]), n, IN)[0], ref.shortest_distance(int(ids[r]), n, IN)[0])
    assert np.array_equal(og.pagerank(0.85, n, 6)[0], ref.pagerank(0.85, n, 6)[0], equal_nan=True)


def test_oracle_resolve_keeps_results():
    scale = 10
    n = 1 << scale
    src, dst, w = rmat_edges(scale, 8, seed=5, weights=True)
    a = fr.OracleGraph.from_edges(n, src, dst, w)
    b = fr.OracleGraph.from_edges(n, src, dst, w).resolve(threads=4)
    seed = int(((np.arange(n) + 1) << 3)[3])
    for scope in (IN, OUT, BOTH):
        assert np.array_equal(a.shortest_distance(seed, 9, scope, weighted=True)[0],
                              b.shortest_distance(seed, 9, scope, weighted=True, threads=4)[0])
    assert np.array_equal(a.pagerank(0.85, n, 8)[0], b.pagerank(0.85, n, 8, threads=4)[0], equal_nan=True)
    assert np.array_equal(a.degree_counter(3)[0], b.degree_counter(3, threads=4)[0])


def test_synth_rows_decode_like_edge_lists():
    """Oracle row path over tgo_synth_rows == oracle edge-list path (ids mapped)."""
    scale = 9
    n = 1 << scale
    src, dst, w = rmat_edges(scale, 8, seed=8, weights=True)
    knows = es.user_edge_label(1)
    wkey = es.user_property_key(1)
    sd = {"edge_types": [{"type_id": knows, "multiplicity": 0, "signature": [wkey]}], "property_keys": [[wkey, 3]]}
    osch = fr.OracleSchema(sd["edge_types"], [tuple(x) for x in sd["property_keys"]])
    rows = synth_rows(n, src, dst, w, label_id=knows)
    vid = np.array([es.vertex_id(i) for i in range(n)], np.int64)
    for scope, limit in ((IN, 30), (BOTH, 30), (OUT, 10 ** 6)):
        og_rows = fr.OracleGraph.from_rows(rows, osch, scope, hard_limit=limit, weight_key=wkey)
        cap = limit if scope != BOTH else 0
        og_edges = fr.OracleGraph.from_edges(n, src, dst, w, titan_ids=vid, hard_limit=cap)
        assert og_rows.stats.truncated_results == og_edges.stats.truncated_results
        pos = {int(v): i for i, v in enumerate(og_rows.vertex_ids())}
        perm = np.array([pos[int(v)] for v in vid])
        for r in (1, 100, 300):
            a = og_rows.shortest_distance(int(vid[r]), n, scope, weighted=True)[0][perm]
            b = og_edges.shortest_distance(int(vid[r]), n, scope, weighted=True)[0]
            assert np.array_equal(a, b)

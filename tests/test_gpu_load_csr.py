"""GPU: tgo_load_csr — a caller-assembled adjacency, the rows as a CSR-collecting
scan job holds them after VertexJobConverter (VertexJobConverter.java:109-129).  Loading the
rows of an edge list this way gives the same device graph as tgo_load_edges, array for array;
rows whose OUT and IN lists are not transposes of each other (a cut applied by the scan) get
the explicit push transpose and the reference's per-row semantics (checked against the oracle
loaded from the same rows); malformed input fails like the other loads."""
import os
import sys

import numpy as np
import pytest

from titan_amd import Engine, rmat_edges, pick_roots
from titan_amd import _lib as L
from titan_amd.engine import TitanException

sys.path.insert(0, os.path.dirname(__file__))
from test_gpu_assembly import _snapshot, _same  # noqa: E402
from test_gpu_parity import numpy_adjacency  # noqa: E402

import fulgora as fr  # noqa: E402

pytestmark = pytest.mark.gpu


def _split(off, mid, adj, ww):
    """Row-wise OUT / IN CSRs of the oracle's adjacency (per row [off, mid) OUT, [mid, off+1) IN)."""
    n = len(off) - 1
    outdeg = mid - off[:-1]
    indeg = off[1:] - mid
    row = np.repeat(np.arange(n), (off[1:] - off[:-1]).astype(np.int64))
    is_out = np.arange(len(adj)) < mid[row]
    oo = np.zeros(n + 1, np.int64)
    oo[1:] = np.cumsum(outdeg)
    io = np.zeros(n + 1, np.int64)
    io[1:] = np.cumsum(indeg)
    ow = iw = None
    if ww is not None:
        ow, iw = ww[is_out], ww[~is_out]
    return oo, adj[is_out], ow, io, adj[~is_out], iw


def _cut(off, mid, adj, ww, keep):
    """The adjacency with every row's OUT list cut to its first `keep` entries (a preload cut
    on one direction only: the lists are no longer transposes of each other)."""
    n = len(off) - 1
    outdeg = np.minimum(mid - off[:-1], keep)
    indeg = off[1:] - mid
    row = np.repeat(np.arange(n), (off[1:] - off[:-1]).astype(np.int64))
    pos = np.arange(len(adj)) - off[row]
    sel = (pos < outdeg[row]) | (np.arange(len(adj)) >= mid[row])
    noff = np.zeros(n + 1, np.int64)
    noff[1:] = np.cumsum(outdeg + indeg)
    nmid = noff[:-1] + outdeg
    return noff, nmid, adj[sel], None if ww is None else ww[sel]


@pytest.mark.parametrize("scope,weighted,cols", [(L.SCOPE_BOTH_E, False, False), (L.SCOPE_IN_E, True, False),
                                                 (L.SCOPE_OUT_E, True, True)])
def test_csr_load_equals_edge_load(monkeypatch, scope, weighted, cols):
    monkeypatch.delenv("TGO_HOST_ASSEMBLY", raising=False)
    scale = 12
    src, dst, w = rmat_edges(scale, 16, seed=83, weights=True)
    n = (1 << scale) + 19                         # isolated tail
    ids = ((np.arange(n, dtype=np.int64) * 5 + 3) << 3)
    off, mid, adj, ww = numpy_adjacency(n, src, dst, w if weighted else None)
    oo, oi, ow, io, ii, iw = _split(off, mid, adj, ww)
    a = _snapshot(Engine().load_edges(n, src, dst, scope, weight=w if weighted else None, titan_ids=ids,
                                      apply_cap=False, column_order=cols))
    b = _snapshot(Engine().load_csr(n, oo, oi, io, ii, scope, out_w=ow, in_w=iw, titan_ids=ids, column_order=cols))
    _same(a, b)


def test_csr_load_cut_rows_match_the_oracle(monkeypatch):
    """OUT lists cut to 6 entries: inE (pull over OUT rows, push over the explicit transpose)
    BFS, weighted delta SSSP and PageRank against the oracle over the same rows; device and
    host assembly array-identical."""
    scale = 11
    src, dst, w = rmat_edges(scale, 16, seed=29, weights=True)
    n = 1 << scale
    ids = ((np.arange(n, dtype=np.int64) + 1) << 3)
    off, mid, adj, ww = _cut(*numpy_adjacency(n, src, dst, w), keep=6)
    oo, oi, ow, io, ii, iw = _split(off, mid, adj, ww)
    snaps = []
    for host in ("1", "0"):
        monkeypatch.setenv("TGO_HOST_ASSEMBLY", host)
        snaps.append(_snapshot(Engine().load_csr(n, oo, oi, io, ii, L.SCOPE_IN_E, out_w=ow, in_w=iw, titan_ids=ids)))
    monkeypatch.delenv("TGO_HOST_ASSEMBLY")
    _same(snaps[0], snaps[1])
    assert snaps[1]["push"] is not None                 # the lists are asymmetric: transpose built
    oracle = fr.OracleGraph.from_adjacency(ids, off, mid, adj, ww)
    eng = Engine().load_csr(n, oo, oi, io, ii, L.SCOPE_IN_E, out_w=ow, in_w=iw, titan_ids=ids)
    for r in pick_roots(n, src, dst, 3, seed=5):
        d = eng.sssp(int(r), n, L.SCOPE_IN_E, mode=L.SSSP_DELTA, seed_is_dense=True)
        od, _ = oracle.shortest_distance(int(ids[r]), n, L.SCOPE_IN_E, weighted=True)
        assert np.array_equal(d, od)
        b = eng.bfs(int(r), 5, L.SCOPE_IN_E, seed_is_dense=True)
        ob, _ = oracle.shortest_distance(int(ids[r]), 5, L.SCOPE_IN_E)
        assert np.array_equal(b, ob)
    pr = eng.pagerank(0.85, n, 10)
    opr, _ = oracle.pagerank(0.85, n, 10)
    fin = np.isfinite(opr)
    assert np.array_equal(np.isfinite(pr), fin)
    # the cut OUT lists make edgeCount small, so the ranks grow far beyond 1: relative L1
    assert np.abs(pr[fin] - opr[fin]).sum() <= 1e-12 * np.abs(opr[fin]).sum()


def test_csr_load_rejects_bad_input():
    z = np.zeros(5, np.int64)
    e = np.zeros(0, np.int32)
    with pytest.raises(TitanException):                  # decreasing offsets
        Engine().load_csr(4, np.array([0, 2, 1, 2, 2]), np.array([1, 2], np.int32), z, e, L.SCOPE_BOTH_E)
    with pytest.raises(TitanException):                  # neighbour index out of range
        Engine().load_csr(4, np.array([0, 1, 1, 1, 1]), np.array([7], np.int32), z, e, L.SCOPE_BOTH_E)
    with pytest.raises(TitanException):                  # titan ids not increasing
        Engine().load_csr(4, z, e, z, e, L.SCOPE_BOTH_E, titan_ids=np.array([8, 16, 16, 24]))
    with pytest.raises(TitanException):                  # a weight array missing
        _missing_weight()
    g = Engine().load_csr(4, z, e, z, e, L.SCOPE_BOTH_E)    # no entries: every vertex isolated
    assert g.stats()["num_vertices"] == 4 and g.stats()["out_entries"] == 0


def _missing_weight():
    import ctypes as C
    lib = L.load()
    eng = Engine()
    opts, keep = eng._opts(L.SCOPE_BOTH_E, False, (), 1, 0)
    oo = np.array([0, 1, 1], np.int64)
    io = np.array([0, 0, 1], np.int64)
    oi = np.array([1], np.int32)
    ii = np.array([0], np.int32)
    ow = np.array([4], np.int32)
    rc = lib.tgo_load_csr(eng.ctx, 2, None, L.ptr(oo, C.c_int64), L.ptr(oi, C.c_int32), L.ptr(ow, C.c_int32),
                          L.ptr(io, C.c_int64), L.ptr(ii, C.c_int32), None, C.byref(opts))
    if rc:
        raise TitanException(rc, "missing in_w")

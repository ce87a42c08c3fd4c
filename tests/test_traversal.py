"""TraversalVertexProgram k-hop traversals (titan_amd/traversal.py) on CPU: the program driven
through the oracle double (OracleEngine: fr_gather merges the bulks) against a sparse-matrix
evaluation of the same step sequence in wrapping int64, and the k-walk closed form of
OLAPTest's DegreeCounter for both()^k.  The device run: tests/test_gpu_traversal.py."""
import numpy as np
import pytest

import fulgora as fr
from generic_programs import OracleEngine
from titan_amd import FulgoraMemory, TraversalVertexProgram, rmat_edges
from titan_amd import _lib as L
from titan_amd.generic import preload_scope, run_generic


def step_matrix_eval(n, src, dst, ids, steps, seeds):
    """Bulks after the steps: out moves tail -> head along every edge, in head -> tail, both
    either way (a self-loop is one OUT and one IN entry of its vertex: both() takes it twice)."""
    pos = {int(v): i for i, v in enumerate(ids)}
    tid = (np.arange(n, dtype=np.int64) + 1) << 3            # OracleGraph.from_edges' Titan ids
    rs = np.array([pos[int(tid[s])] for s in src])
    rd = np.array([pos[int(tid[d])] for d in dst])
    b = np.zeros(len(ids), np.int64)
    if seeds is None:
        b[:] = 1
    else:
        for s in seeds:
            if int(s) in pos:
                b[pos[int(s)]] += 1
    with np.errstate(over="ignore"):
        for st in steps:
            nb = np.zeros_like(b)
            if st in ("out", "both"):
                np.add.at(nb, rd, b[rs])
            if st in ("in", "both"):
                np.add.at(nb, rs, b[rd])
            b = nb
    return b


@pytest.fixture(scope="module")
def small():
    n = 1 << 9
    src, dst, _ = rmat_edges(9, 6, seed=23)
    return n, src, dst, fr.OracleGraph.from_edges(n, src, dst)


@pytest.mark.parametrize("steps", [["out"], ["in", "in"], ["both", "out", "in"], ["out"] * 6, ["both"] * 9])
def test_traversal_bulks_match_matrix_evaluation(small, steps):
    n, src, dst, o = small
    eng = OracleEngine(o)
    ids = eng.vertex_ids()
    for seeds in (None, ids[[0, 5, 5, 77]]):
        p = TraversalVertexProgram(steps, seeds)
        mem = FulgoraMemory(p.memory_compute_keys)
        verts = run_generic(eng, p, mem)
        mem.complete()
        got, present = verts.property("traversers")
        exp = step_matrix_eval(n, src, dst, ids, steps, seeds)
        assert np.array_equal(np.where(present, got, 0), exp), (steps, seeds is None)
        assert np.array_equal(present, exp != 0)
        assert mem.get("count") == int(exp.sum(dtype=np.int64))
        assert mem.getIteration() == len(steps)


def test_in_k_equals_degree_counter_walks(small):
    """in()^k from every vertex: the k-walk counts of OLAPTest.DegreeCounter (DEG_MSG = inE:
    each vertex sums its out-neighbours' previous counts; the oracle's fr_degree_counter,
    pinned by the OLAPTest closed forms in tests/test_oracle.py)."""
    n, src, dst, o = small
    for k in (1, 2, 3, 4):
        p = TraversalVertexProgram(["in"] * k)
        mem = FulgoraMemory(p.memory_compute_keys)
        verts = run_generic(OracleEngine(o), p, mem)
        got, present = verts.property("traversers")
        walks, _ = o.degree_counter(k)
        assert np.array_equal(np.where(present, got, 0), walks.astype(np.int64)), k


def test_preload_is_the_star_graph_and_step_validation():
    p = TraversalVertexProgram(["out", "in"])
    assert preload_scope(p, probe_memory_iterations=3) == L.SCOPE_BOTH_E
    with pytest.raises(ValueError):
        TraversalVertexProgram(["out", "sideways"])

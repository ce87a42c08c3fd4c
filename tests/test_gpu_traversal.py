"""GPU: TraversalVertexProgram k-hop traversals (titan_amd/traversal.py) submitted through the
TitanGraphComputer mirror on the star-graph (bothE) preload: bulks and count() equal to the
same program driven through the oracle double (fr_gather), which tests/test_traversal.py pins
against a sparse-matrix evaluation and OLAPTest's DegreeCounter walk counts — and in()^k equal
to the device's own tgo_walkcount (DegreeCounter) where no int wraps."""
import numpy as np
import pytest

import fulgora as fr
from generic_programs import OracleEngine
from titan_amd import FulgoraMemory, GpuGraph, TraversalVertexProgram, rmat_edges
from titan_amd.generic import run_generic

pytestmark = pytest.mark.gpu


def reorder(ids_from, values, ids_to):
    pos = {int(v): i for i, v in enumerate(ids_from)}
    return np.array([values[pos[int(v)]] for v in ids_to])


@pytest.fixture(scope="module")
def rmat():
    n = 1 << 12
    src, dst, _ = rmat_edges(12, 8, seed=41)
    return n, src, dst, fr.OracleGraph.from_edges(n, src, dst, hard_limit=100000)


@pytest.mark.parametrize("steps,seeded", [(["out", "out"], False), (["both", "in", "out"], True),
                                          (["in"] * 5, False), (["both"] * 7, True)])
def test_traversal_program_matches_oracle(rmat, steps, seeded):
    n, src, dst, o = rmat
    ids = o.vertex_ids()
    seeds = ids[[1, 2, 2, 300, 4000]] if seeded else None
    graph = GpuGraph(edges=(n, src, dst, None))
    result = graph.compute().program(TraversalVertexProgram(steps, seeds)).submit().get()
    p = TraversalVertexProgram(steps, seeds)
    mem = FulgoraMemory(p.memory_compute_keys)
    verts = run_generic(OracleEngine(o), p, mem)
    mem.complete()
    exp, ep = verts.property("traversers")
    rids, (got, gp) = result.vertex_properties["traversers"][0], result.vertex_properties["traversers"][1]
    assert np.array_equal(reorder(rids, gp, verts.ids), ep)
    assert np.array_equal(reorder(rids, np.where(gp, got, 0), verts.ids), np.where(ep, exp, 0))
    assert result.memory().get("count") == mem.get("count")
    assert result.memory().getIteration() == len(steps) == mem.getIteration()


def test_in_k_equals_device_walkcount(rmat):
    n, src, dst, o = rmat
    graph = GpuGraph(edges=(n, src, dst, None))
    for k in (1, 2, 3):
        result = graph.compute().program(TraversalVertexProgram(["in"] * k)).submit().get()
        rids, (got, gp) = result.vertex_properties["traversers"][0], result.vertex_properties["traversers"][1]
        walks, _ = o.degree_counter(k)
        b = reorder(rids, np.where(gp, got, 0), o.vertex_ids())
        assert np.array_equal(b, walks.astype(np.int64)), k

"""TraversalVertexProgram's k-hop traversals on the GPU path.

TinkerPop's TraversalVertexProgram runs a Gremlin traversal on the computer: traversers sit
at vertices with a bulk (a long count of the identical traversers merged there), and every
vertex step moves each traverser along the incident edges of its vertex.  Titan's only part
in it is the preload: the whole star graph of every vertex, BOTH directions, every label
(VertexProgramScanJob.getQueries, :101-107) — because a traverser may take any incident edge.
An untyped BOTH query is "fitted" and keeps NO_LIMIT (QueryContainer.java:122;
BasicVertexCentricQueryBuilder.java:418-431), so the star preload is uncapped: the 100 000-entry
hard limit cuts only single-direction untyped scopes.

Restated here for the traversals that are pure vertex steps, ``g.V([seeds]).out().in()
.both()...`` followed by ``count()`` (the k-hop / path-count queries Gremlin OLAP is run for):
one superstep per step; a step is a Local message scope (``out()``: Local(outE), the traverser
moves from the edge's tail to its head; ``in()``: Local(inE); ``both()``: Local(bothE)) whose
messages are the bulks, merged at the receiving vertex by SUM — Java long addition, wrapping,
as Traverser bulks do.  The device does the merging (tgo_gather, identity edge function,
int64 SUM); the preload is the star graph (``preload = bothE``), so every step direction
reads the same loaded lists.

Parity: TinkerPop's own tests for TraversalVertexProgram live in the absent gremlin-test jar
(SURVEY.md §8c), so the bulks are pinned instead by (i) the closed forms the walk counts of
OLAPTest's DegreeCounter obey — ``in()`` k times from every vertex gives its k-walk counts
(DEG_MSG = inE, OLAPTest.java:334-416; tgo_walkcount, int wrap aside) — and (ii) a
sparse-matrix evaluation of the same step sequence (tests/test_traversal.py, tests/test_gpu_traversal.py).  Steps with label filters,
filters, side effects and paths are TinkerPop's machinery and are not restated.
"""
from __future__ import annotations

import numpy as np

from . import _lib as L
from .generic import GenericVertexProgram, MessageScope

STEP_SCOPES = {"out": "outE", "in": "inE", "both": "bothE"}


def _wrap_sum(a) -> int:
    """Java long sum of int64 values (wrapping)."""
    return int(np.asarray(a, np.int64).sum(dtype=np.int64))


class TraversalVertexProgram(GenericVertexProgram):
    """``g.V([seeds]).<step>()...<step>().count()`` with vertex steps out / in / both.

    Element compute key ``traversers``: the bulk at each vertex after the last step (present
    where it is non-zero).  Memory ``count``: the traversal's count(), the sum of the bulks."""
    value_type = L.VAL_INT64
    combiner = L.COMBINE_SUM
    compute_keys = ("traversers",)
    memory_compute_keys = ("count",)
    preload = L.SCOPE_BOTH_E            # the star graph (VertexProgramScanJob.java:101-107)

    def __init__(self, steps, seeds=None):
        steps = list(steps)
        bad = [s for s in steps if s not in STEP_SCOPES]
        if bad:
            raise ValueError(f"vertex steps must be out, in or both: {bad}")
        self.steps = steps
        self.seeds = None if seeds is None else np.asarray(seeds, np.int64)
        self._scopes = [MessageScope.Local(STEP_SCOPES[s]) for s in steps]

    def getMessageScopes(self, memory):  # noqa: N802
        it = memory.getIteration()
        return [self._scopes[it]] if it < len(self.steps) else []

    def _finish(self, v, bulk, memory):
        v.set_property("traversers", bulk, bulk != 0)
        memory.incr("count", _wrap_sum(bulk))

    def execute(self, v, messenger, memory):
        it = memory.getIteration()
        if it == 0:
            bulk = np.zeros(v.n, np.int64)
            if self.seeds is None:
                bulk[:] = 1                      # g.V(): one traverser per vertex
            else:                                # g.V(ids): one per listed id (repeats add up)
                pos = {int(x): i for i, x in enumerate(v.ids)}
                for s in self.seeds:
                    i = pos.get(int(s))
                    if i is not None:
                        bulk[i] += 1
        else:
            got, has = messenger.receive(self._scopes[it - 1])
            bulk = np.where(has, got, 0).astype(np.int64)
        if it < len(self.steps):
            messenger.send(self._scopes[it], bulk, bulk != 0)
        else:
            self._finish(v, bulk, memory)

    def terminate(self, memory):
        return memory.getIteration() >= len(self.steps)

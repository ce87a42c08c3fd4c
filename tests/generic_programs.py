"""Test helpers: vectorised vertex programs for the generic GPU path, and an engine double
over the CPU oracle so the same programs run through Fulgora's restated primitives.

The double (OracleEngine) is test infrastructure: it answers the four calls run_generic makes
(vertex_ids / gather / combine_global / dense_ids) with oracle/fulgora_ref.c's fr_gather and
fr_combine_global, the restatements of VertexMemoryHandler.receiveMessages and
VertexState.addMessage.
"""
import numpy as np

import fulgora as fr
from titan_amd import GenericVertexProgram, MessageScope
from titan_amd import _lib as L


class OracleEngine:
    def __init__(self, oracle: fr.OracleGraph, pb=5):
        self.o = oracle
        self.n = oracle.n
        self._ids = oracle.vertex_ids()
        self._pos = {int(v): i for i, v in enumerate(self._ids)}
        self.pb = pb

    def vertex_ids(self):
        return self._ids

    def gather(self, scope, value_type, combiner, edge_fn, msg, has):
        h = np.ones(self.n, bool) if has is None else has
        return self.o.gather(scope, value_type, combiner, edge_fn, msg, h)

    def gather_lists(self, scope, value_type, edge_fn, msg, has):
        h = np.ones(self.n, bool) if has is None else has
        return self.o.gather_lists(scope, value_type, edge_fn, msg, h)

    def set_edge_program(self, ops, iconsts=None, fconsts=None):
        fr.set_edge_program(ops, iconsts, fconsts)

    def combine_global(self, value_type, combiner, targets, values):
        return fr.combine_global(self.n, value_type, combiner, targets, values)

    def dense_ids(self, titan_ids):
        lib = fr.load()
        out = np.empty(len(titan_ids), np.int64)
        for i, v in enumerate(titan_ids):
            v = int(v)
            if lib.fr_is_partitioned(v, self.pb):
                v = lib.fr_canonical_vertex_id(v, self.pb)
            out[i] = self._pos.get(v, -1)
        return out


class ConnectedComponents(GenericVertexProgram):
    """Weakly connected components by MIN label propagation over bothE: label = smallest
    Titan id reachable.  Memory: `changes` accumulates (incr) the label changes of every
    superstep — FulgoraMemory never clears the current map — and the run stops when a
    superstep adds none; `any` ORs whether anything ever changed."""
    value_type = L.VAL_INT64
    combiner = L.COMBINE_MIN
    compute_keys = ("cc",)
    memory_compute_keys = ("changes", "any")
    SCOPE = MessageScope.Local("bothE")

    def __init__(self):
        self._last = -1

    def getMessageScopes(self, memory):  # noqa: N802
        return [self.SCOPE]

    def execute(self, v, messenger, memory):
        if memory.isInitialIteration():
            v.set_property("cc", v.ids.copy())
            messenger.send(self.SCOPE, v.ids)
            memory.incr("changes", 0)
            memory.or_("any", False)
            return
        cur, _ = v.property("cc")
        got, has = messenger.receive(self.SCOPE)
        better = has & (got < cur)
        v.set_property("cc", np.where(better, got, cur), better)
        messenger.send(self.SCOPE, np.where(better, got, cur), better)
        memory.incr("changes", int(better.sum()))
        memory.or_("any", bool(better.any()))

    def terminate(self, memory):
        total = memory.get("changes")
        done = memory.getIteration() > 0 and total == self._last
        self._last = total
        return done


class GenericPageRank(GenericVertexProgram):
    """PageRankVertexProgram (tmain/olap/PageRankVertexProgram.java:75-100) written against
    the vectorised API: inE scope in iteration 0, outE afterwards, SUM of fp64 messages."""
    value_type = L.VAL_FP64
    combiner = L.COMBINE_SUM
    compute_keys = ("pr", "edges")
    IN = MessageScope.Local("inE")
    OUT = MessageScope.Local("outE")

    def __init__(self, alpha, vertex_count, iterations):
        self.alpha, self.N, self.iterations = alpha, float(vertex_count), iterations

    def getMessageScopes(self, memory):  # noqa: N802
        return [self.IN] if memory.isInitialIteration() else [self.OUT]

    def execute(self, v, messenger, memory):
        if memory.isInitialIteration():
            messenger.send(self.IN, np.ones(v.n))
            return
        if memory.getIteration() == 1:
            ec, _ = messenger.receive(self.IN)
            v.set_property("edges", ec)
            pr = np.full(v.n, 1.0 / self.N)
        else:
            s, _ = messenger.receive(self.OUT)
            pr = self.alpha * s + (1.0 - self.alpha) / self.N
        v.set_property("pr", pr)
        with np.errstate(divide="ignore"):
            messenger.send(self.OUT, pr / v.property("edges")[0])

    def terminate(self, memory):
        return memory.getIteration() >= self.iterations


class GlobalDegreeSum(GenericVertexProgram):
    """Global scope: every vertex sends its (weighted) in-degree sum to `buckets` hub vertices
    chosen by id; the hubs store the SUM they received (in send order) and MAX of the totals
    goes to memory."""
    value_type = L.VAL_INT64
    combiner = L.COMBINE_SUM
    compute_keys = ("inbox",)
    memory_compute_keys = ("total", "best")
    LOCAL = MessageScope.Local("inE", "add_weight")
    GLOBAL = MessageScope.Global()
    weight_property = "w"

    def __init__(self, hub_ids):
        self.hubs = np.asarray(hub_ids, np.int64)

    def getMessageScopes(self, memory):  # noqa: N802
        return [self.LOCAL] if memory.getIteration() == 0 else [self.GLOBAL]

    def execute(self, v, messenger, memory):
        it = memory.getIteration()
        if it == 0:
            messenger.send(self.LOCAL, np.zeros(v.n, np.int64))      # receivers get the weights
        elif it == 1:
            s, has = messenger.receive(self.LOCAL)
            s = np.where(has, s, 0)
            targets = self.hubs[v.ids % len(self.hubs)]
            messenger.send_global(self.GLOBAL, targets, s)
            memory.incr("total", int(s.sum()))
        else:
            inbox, has = messenger.receive(self.GLOBAL)
            v.set_property("inbox", inbox, has)
            memory.set("best", int(inbox[has].max()) if has.any() else 0)

    def terminate(self, memory):
        return memory.getIteration() >= 2


class FirstLastCount(GenericVertexProgram):
    """No combiner: iteration 0 every vertex sends (its Titan id mod 1000) on inE with the edge
    function sub_weight; iteration 1 each vertex keeps the first and the last message of its
    stream and their count (order-sensitive: the stream order is the reference's)."""
    value_type = L.VAL_INT64
    combiner = None
    compute_keys = ("first", "last", "count")
    weight_property = "w"
    SCOPE = MessageScope.Local("inE", "sub_weight")

    def getMessageScopes(self, memory):  # noqa: N802
        return [self.SCOPE] if memory.getIteration() == 0 else []

    def execute(self, v, messenger, memory):
        if memory.getIteration() == 0:
            messenger.send(self.SCOPE, np.asarray(v.ids, np.int64) % 1000)
            return
        lists = messenger.receive(self.SCOPE)
        cnt = lists.counts()
        has = cnt > 0
        first = np.zeros(v.n, np.int64)
        last = np.zeros(v.n, np.int64)
        first[has] = lists.values[lists.offsets[:-1][has]]
        last[has] = lists.values[lists.offsets[1:][has] - 1]
        v.set_property("first", first, has)
        v.set_property("last", last, has)
        v.set_property("count", cnt.astype(np.int64))

    def terminate(self, memory):
        return memory.getIteration() >= 1


class GlobalNoCombiner(GenericVertexProgram):
    """No combiner, a Global scope: every vertex sends 3 x its index to one target (a
    permutation when unique, else two senders share each target -> the job fails)."""
    value_type = L.VAL_INT64
    combiner = None
    compute_keys = ("inbox",)
    SCOPE = MessageScope.Global()

    def __init__(self, ids, unique=True):
        self.ids = np.asarray(ids, np.int64)
        self.unique = unique

    def getMessageScopes(self, memory):  # noqa: N802
        return [self.SCOPE] if memory.getIteration() == 0 else []

    def execute(self, v, messenger, memory):
        n = v.n
        if memory.getIteration() == 0:
            tgt = self.ids[::-1] if self.unique else self.ids[np.arange(n) // 2]
            messenger.send_global(self.SCOPE, tgt, 3 * np.arange(n, dtype=np.int64))
            return
        inbox, has = messenger.receive(self.SCOPE)
        v.set_property("inbox", inbox, has)

    def terminate(self, memory):
        return memory.getIteration() >= 1

"""Generic vertex programs on the GPU path.

A program the engine does not implement natively runs Fulgora's superstep loop
(FulgoraGraphComputer.submit, FulgoraGraphComputer.java:140-189) here on the host, with its
``execute`` written over whole per-vertex vectors instead of one vertex at a time, while the
message traffic — what Fulgora spends its supersteps on — is combined on the device:

* ``MessageScope.Local(incident, edge_fn)`` receives run ``tgo_gather``: every vertex folds
  ``edge_fn(msg[u], e)`` over its reversed incident entries with the program's combiner
  (VertexMemoryHandler.receiveMessages, VertexMemoryHandler.java:77-93; FulgoraUtil.java:57);
* ``MessageScope.Global`` sends run ``tgo_combine_global``: messages to explicit targets fold
  into the target in send order (VertexState.addMessage, VertexState.java:63-78);
* ``FulgoraMemory`` restates the global memory: ``incr/and/or/set`` write the current map,
  ``get`` reads the previous one, ``completeSubRound`` copies current -> previous and
  ``complete`` steps the iteration back (FulgoraMemory.java:21-131).

Messages are double-buffered exactly as VertexState does (sent in iteration i, read in i+1;
VertexState.java:55-89), and the scopes a vertex may receive on are the ones the program
declared for the previous iteration (FulgoraVertexMemory.nextIteration/completeIteration).
With a combiner the receive returns the combined message per vertex.  Without one
(``combiner = None``) a Local receive returns every vertex's message stream itself
(``MessageLists``, ``tgo_gather_lists``) in the order the reference's stream yields it, the
row's column order, for the program to reduce however it likes; a Global scope then delivers
at most one message per target, and two messages meeting at a target (or at a vertex cut)
fail the job as FulgoraUtil's ThrowingCombiner does (FulgoraUtil.java:80-91).

Edge functions are "message op w" over the load's weight property (any 32-bit numeric key:
Byte, Short, Integer, Character, Boolean, Float): identity, +1, + - * / min max of w — or any
arithmetic composition of the message ``M``, the weight ``W`` and constants written as an
``EdgeExpr`` (``MessageScope.Local("inE", M * 2 + W)``): compiled to a postfix program
(tgo_set_edge_program) that the device evaluates per entry in Java arithmetic.
TinkerPop's TraversalVertexProgram (Gremlin OLAP traversals, BOTH preload at
VertexProgramScanJob.java:101-107) is restated for vertex-step traversals in
titan_amd/traversal.py (a program with ``preload = bothE``); its own tests live in the absent
gremlin-test jar, so it is pinned against walk-count closed forms instead.
"""
from __future__ import annotations

import numpy as np

from . import _lib as L

EDGE_FNS = {"identity": L.EDGE_IDENTITY, "add_one": L.EDGE_ADD_ONE, "add_weight": L.EDGE_ADD_WEIGHT,
            "mul_weight": L.EDGE_MUL_WEIGHT, "sub_weight": L.EDGE_SUB_WEIGHT, "min_weight": L.EDGE_MIN_WEIGHT,
            "max_weight": L.EDGE_MAX_WEIGHT, "div_weight": L.EDGE_DIV_WEIGHT}
INCIDENT = {"outE": L.SCOPE_OUT_E, "inE": L.SCOPE_IN_E, "bothE": L.SCOPE_BOTH_E}


class EdgeExpr:
    """An edge function (m, e) -> message as an arithmetic expression over the message ``M``,
    the weight ``W`` = e.value(weight) and constants, in Java semantics for the message type
    (long: wrapping + - *, truncating / and %, / 0 throws; double: IEEE, Math.min / max / abs).
    ``compile()`` gives the postfix program of include/titan_gpu_olap.h tgo_edge_program.
    Python ints and floats mix in: ``M * 2 + W``, ``(M - 1).min(W)``, ``abs(-M)``."""

    def __init__(self, op, args=(), value=None):
        self.op, self.args, self.value = op, tuple(args), value

    @staticmethod
    def lift(x):
        if isinstance(x, EdgeExpr):
            return x
        if isinstance(x, bool) or not isinstance(x, (int, float)):
            raise TypeError(f"edge expression operand must be an EdgeExpr, int or float: {x!r}")
        return EdgeExpr(L.OP_CONST, value=x)

    def _bin(self, op, other, swap=False):
        o = EdgeExpr.lift(other)
        return EdgeExpr(op, (o, self) if swap else (self, o))

    def __add__(self, o): return self._bin(L.OP_ADD, o)
    def __radd__(self, o): return self._bin(L.OP_ADD, o, True)
    def __sub__(self, o): return self._bin(L.OP_SUB, o)
    def __rsub__(self, o): return self._bin(L.OP_SUB, o, True)
    def __mul__(self, o): return self._bin(L.OP_MUL, o)
    def __rmul__(self, o): return self._bin(L.OP_MUL, o, True)
    def __truediv__(self, o): return self._bin(L.OP_DIV, o)        # Java / (long: truncating)
    def __rtruediv__(self, o): return self._bin(L.OP_DIV, o, True)
    def __mod__(self, o): return self._bin(L.OP_REM, o)            # Java %
    def __rmod__(self, o): return self._bin(L.OP_REM, o, True)
    def __neg__(self): return EdgeExpr(L.OP_NEG, (self,))
    def __abs__(self): return EdgeExpr(L.OP_ABS, (self,))
    def min(self, o): return self._bin(L.OP_MIN, o)                # Math.min
    def max(self, o): return self._bin(L.OP_MAX, o)                # Math.max

    def compile(self):
        """(ops, long constants, double constants); a constant that is not integral gives no
        long form (the program then runs on double messages only)."""
        ops, consts = [], []

        def emit(e):
            for a in e.args:
                emit(a)
            if e.op == L.OP_CONST:
                v = e.value
                if isinstance(v, int) and not -(1 << 63) <= v < (1 << 63):
                    raise ValueError(f"edge expression constant out of long range: {v}")
                # the same constant: same type and, for floats, the same bits (0.0 is not -0.0)
                same = (lambda c: c == v) if isinstance(v, int) else (lambda c: float(c).hex() == float(v).hex())
                i = next((k for k, c in enumerate(consts) if type(c) is type(v) and same(c)), None)
                if i is None:
                    consts.append(v)
                    i = len(consts) - 1
                ops.append(L.OP_CONST | (i << 8))
            else:
                ops.append(e.op)
        emit(self)
        if len(ops) > L.EDGE_PROGRAM_MAX_OPS or len(consts) > L.EDGE_PROGRAM_MAX_CONSTS:
            raise ValueError(f"edge expression too large: {len(ops)} ops, {len(consts)} constants")
        integral = all(isinstance(c, int) for c in consts)
        ic = [int(c) for c in consts] if integral else None
        fc = [float(c) for c in consts]
        return ops, ic, fc

    def key(self):
        return (self.op, self.value, tuple(a.key() for a in self.args))

    def __eq__(self, o):
        return isinstance(o, EdgeExpr) and self.key() == o.key()

    def __hash__(self):
        return hash(self.key())

    def __repr__(self):
        names = {L.OP_ADD: "+", L.OP_SUB: "-", L.OP_MUL: "*", L.OP_DIV: "/", L.OP_REM: "%"}
        if self.op == L.OP_MSG:
            return "M"
        if self.op == L.OP_WEIGHT:
            return "W"
        if self.op == L.OP_CONST:
            return repr(self.value)
        if self.op in names:
            return f"({self.args[0]!r} {names[self.op]} {self.args[1]!r})"
        if self.op == L.OP_NEG:
            return f"-{self.args[0]!r}"
        if self.op == L.OP_ABS:
            return f"abs({self.args[0]!r})"
        return f"{self.args[0]!r}.{'min' if self.op == L.OP_MIN else 'max'}({self.args[1]!r})"


M = EdgeExpr(L.OP_MSG)      # the message the sender holds
W = EdgeExpr(L.OP_WEIGHT)   # e.value(weight) of the traversed edge


class MessageScope:
    class Local:
        """MessageScope.Local.of(__::<incident>, edgeFunction); edge_fn is a menu name or an
        EdgeExpr."""

        def __init__(self, incident="inE", edge_fn="identity"):
            if incident not in INCIDENT:
                raise ValueError(f"incident traversal must be outE, inE or bothE: {incident}")
            if not isinstance(edge_fn, EdgeExpr) and edge_fn not in EDGE_FNS:
                raise ValueError(f"unsupported edge function {edge_fn}")
            self.incident, self.edge_fn = incident, edge_fn

        def __eq__(self, o):
            return isinstance(o, MessageScope.Local) and (o.incident, o.edge_fn) == (self.incident, self.edge_fn)

        def __hash__(self):
            return hash(("local", self.incident, self.edge_fn))

        def __repr__(self):
            return f"Local({self.incident}, {self.edge_fn})"

    class Global:
        """MessageScope.Global: every Global scope is one inbox (FulgoraVertexMemory.normalizeScope)."""

        def __eq__(self, o):
            return isinstance(o, MessageScope.Global)

        def __hash__(self):
            return hash("global")

        def __repr__(self):
            return "Global"


class MemoryException(KeyError):
    pass


class FulgoraMemory:
    """core/graphdb/olap/computer/FulgoraMemory.java:21-131."""

    def __init__(self, memory_keys=()):
        self.memory_keys = set(memory_keys)
        self.previous, self.current = {}, {}
        self._iteration = 0
        self._runtime = 0

    def keys(self):
        return set(self.previous)

    def incrIteration(self):  # noqa: N802
        self._iteration += 1

    def setIteration(self, it):  # noqa: N802
        self._iteration = it

    def getIteration(self):  # noqa: N802
        return self._iteration

    def setRuntime(self, rt):  # noqa: N802
        self._runtime = rt

    def getRuntime(self):  # noqa: N802
        return self._runtime

    def isInitialIteration(self):  # noqa: N802
        return self._iteration == 0

    def complete(self):                       # :73-76
        self._iteration -= 1
        self.previous = self.current

    def completeSubRound(self):  # noqa: N802  :78-81
        self.previous = dict(self.current)

    def exists(self, key):
        return key in self.previous

    def get(self, key):
        if key not in self.previous:
            raise MemoryException(f"The memory does not have a value for provided key: {key}")
        return self.previous[key]

    def _check(self, key, value):
        if key not in self.memory_keys:
            raise ValueError(f"The provided key is not a memory compute key: {key}")
        if value is None:
            raise ValueError("Memory values can not be null")

    def incr(self, key, delta):
        self._check(key, delta)
        v = self.current.get(key)
        self.current[key] = int(delta) if v is None else int(delta) + v

    def and_(self, key, b):
        self._check(key, b)
        v = self.current.get(key)
        self.current[key] = bool(b) if v is None else (bool(b) and v)

    def or_(self, key, b):
        self._check(key, b)
        v = self.current.get(key)
        self.current[key] = bool(b) if v is None else (bool(b) or v)

    def set(self, key, value):
        self._check(key, value)
        self.current[key] = value


class Vertices:
    """All executing vertices of one superstep: Titan ids (row order) and compute-key
    properties as (values, present) vectors (VertexState properties, immediate writes)."""

    def __init__(self, ids, compute_keys):
        self.ids = ids
        self.n = len(ids)
        self._props = {k: None for k in compute_keys}

    def property(self, key):
        """(values, present) — present False where the property was never set."""
        if key not in self._props:
            raise KeyError(f"not an element compute key: {key}")
        return self._props[key]

    def set_property(self, key, values, present=None):
        if key not in self._props:
            raise KeyError(f"not an element compute key: {key}")
        values = np.asarray(values)
        present = np.ones(self.n, bool) if present is None else np.asarray(present, bool)
        old = self._props[key]
        if old is None:
            self._props[key] = (values.copy(), present.copy())
        else:                                 # only the vertices that set it change
            ov, op = old
            nv = ov.copy()
            nv[present] = values[present]
            self._props[key] = (nv, op | present)


class MessageLists:
    """A combiner-less Local receive: every vertex's message stream (row order), the values
    of vertex i in ``values[offsets[i]:offsets[i+1]]`` in the order the reference's
    receiveMessages stream yields them (VertexMemoryHandler.java:83-92)."""

    def __init__(self, offsets, values):
        self.offsets = np.asarray(offsets, np.int64)
        self.values = np.asarray(values)

    def __len__(self):
        return len(self.offsets) - 1

    def of(self, i):
        return self.values[self.offsets[i]:self.offsets[i + 1]]

    def counts(self):
        return np.diff(self.offsets)

    def has(self):
        return self.counts() > 0

    def reduce(self, ufunc):
        """ufunc folded over each vertex's stream in stream order -> (values, has)."""
        n = len(self)
        cnt = self.counts()
        out = np.zeros(n, self.values.dtype)
        nz = cnt > 0
        if nz.any():
            out[nz] = ufunc.reduceat(self.values, self.offsets[:-1][nz])
        return out, nz


class Messenger:
    """Messenger of one superstep: receive() combines the previous superstep's messages of a
    scope on the device; send() records this superstep's messages."""

    def __init__(self, engine, program, previous, current_scopes):
        self._e = engine
        self._p = program
        self._prev = previous           # scope -> (values, has) as sent last superstep
        self._scopes = set(current_scopes)
        self.sent = {}                  # Local scope -> (values, has); Global -> [(targets, values)]

    def receive(self, scope):
        """(combined values, has-message mask) per vertex for `scope`."""
        n = self._e.n
        zero = np.zeros(n, np.int64 if self._p.value_type == L.VAL_INT64 else np.float64)
        if scope not in self._prev:
            return zero, np.zeros(n, bool)
        vals, has = self._prev[scope]
        if isinstance(scope, MessageScope.Global):
            return vals, has
        fn = EDGE_FNS.get(scope.edge_fn) if not isinstance(scope.edge_fn, EdgeExpr) else L.EDGE_PROGRAM
        if fn == L.EDGE_PROGRAM:
            self._e.set_edge_program(*scope.edge_fn.compile())
        if self._p.combiner is None:
            return MessageLists(*self._e.gather_lists(INCIDENT[scope.incident], self._p.value_type, fn, vals, has))
        return self._e.gather(INCIDENT[scope.incident], self._p.value_type, self._p.combiner, fn, vals, has)

    def send(self, scope, values, has=None):
        """Local scope: every vertex with has[v] sends values[v] (setMessage on the sender,
        VertexMemoryHandler.java:106-108).  Global scope: use send_global."""
        if scope not in self._scopes:
            raise ValueError(f"Provided scope was not declared in the VertexProgram: {scope}")
        if isinstance(scope, MessageScope.Global):
            raise TypeError("Global messages name their targets: use send_global(scope, targets, values)")
        n = self._e.n
        has = np.ones(n, bool) if has is None else np.asarray(has, bool)
        old = self.sent.get(scope)
        if old is None:
            self.sent[scope] = (np.array(values, copy=True), has.copy())
        else:                           # a later send replaces the earlier message (setMessage)
            ov, oh = old
            nv = ov.copy()
            nv[has] = np.asarray(values)[has]
            self.sent[scope] = (nv, oh | has)

    def send_global(self, scope, target_ids, values):
        """Messages to explicit vertices (Titan ids; vertex cuts canonicalised, unknown ids
        dropped), combined per target in send order."""
        if scope not in self._scopes:
            raise ValueError(f"Provided scope was not declared in the VertexProgram: {scope}")
        self.sent.setdefault(MessageScope.Global(), []).append((np.asarray(target_ids, np.int64), np.asarray(values)))

    def finish(self):
        """completeIteration: this superstep's messages become the next one's previous."""
        out = {}
        for scope, v in self.sent.items():
            if isinstance(scope, MessageScope.Global):
                tid = np.concatenate([t for t, _ in v]) if v else np.zeros(0, np.int64)
                val = np.concatenate([x for _, x in v]) if v else np.zeros(0)
                dense = self._e.dense_ids(tid)
                keep = dense >= 0
                comb = self._p.combiner
                if comb is None:
                    # no combiner: VertexState.addMessage combines a second message to one
                    # target with FulgoraUtil's ThrowingCombiner (:80-91)
                    t = dense[keep]
                    if len(t) != len(np.unique(t)):
                        from .engine import TitanException
                        raise TitanException(L.TGO_E_PROGRAM, "The VertexProgram needs to define a message combiner "
                                                              "in order to preserve memory and handle partitioned vertices")
                    comb = L.COMBINE_SUM
                out[scope] = self._e.combine_global(self._p.value_type, comb, dense[keep], val[keep])
            else:
                out[scope] = v
        return out


class GenericVertexProgram:
    """Base of vectorised vertex programs (TinkerPop VertexProgram, one call per superstep
    over all vertices).  Subclasses set value_type / combiner and override the hooks."""
    value_type = L.VAL_INT64
    combiner = L.COMBINE_SUM            # None: receive() hands Local streams over as MessageLists
    compute_keys: tuple = ()
    memory_compute_keys: tuple = ()
    weight_property = None              # property read by add_weight / mul_weight edge functions
    # getPreferredPersist: the mode submit() uses when resultMode is not set; NOTHING keeps
    # the results in memory / MapReduce (subclasses may prefer VERTEX_PROPERTIES)
    preferred_persist = None            # None = Persist.NOTHING

    def setup(self, memory):
        pass

    def getMessageScopes(self, memory):  # noqa: N802
        return []

    def execute(self, vertices: Vertices, messenger: Messenger, memory: FulgoraMemory):
        raise NotImplementedError("GenericVertexProgram.execute must be overridden")

    def terminate(self, memory) -> bool:
        return True


def preload_scope(program, probe_memory_iterations=1):
    """The single preload a program's Local scopes need: their common direction, or bothE when
    they differ (VertexProgramScanJob.getQueries adds one slice per scope, :109-119).  A program
    that fixes its preload (``preload``, e.g. TraversalVertexProgram's whole star graph,
    VertexProgramScanJob.java:101-107) gets that."""
    if getattr(program, "preload", None) is not None:
        return program.preload
    dirs = set()
    mem = FulgoraMemory(program.memory_compute_keys)
    for it in range(probe_memory_iterations):
        mem.setIteration(it)
        for s in program.getMessageScopes(mem):
            if isinstance(s, MessageScope.Local):
                dirs.add(INCIDENT[s.incident])
    if len(dirs) == 1:
        return dirs.pop()
    return L.SCOPE_BOTH_E


def run_generic(engine, program: GenericVertexProgram, memory: FulgoraMemory):
    """FulgoraGraphComputer.submit's superstep loop (:140-189) over one loaded engine.
    Returns the final Vertices (compute-key properties)."""
    ids = engine.vertex_ids()
    verts = Vertices(ids, program.compute_keys)
    program.setup(memory)
    memory.completeSubRound()
    previous = {}
    while True:
        scopes = list(program.getMessageScopes(memory))          # vertexMemory.nextIteration
        messenger = Messenger(engine, program, previous, scopes)
        program.execute(verts, messenger, memory)
        previous = messenger.finish()                            # vertexMemory.completeIteration
        memory.completeSubRound()
        try:
            if program.terminate(memory):
                break
        finally:
            memory.incrIteration()
            memory.completeSubRound()
    return verts


class ComputeKeyMapReduce:
    """Emits (vertex id, value) of one compute key for every vertex where it is set — the
    shape of PageRankMapReduce / ShortestDistanceMapReduce (map :45-50)."""

    def __init__(self, compute_key, memory_key):
        self.compute_key = compute_key
        self.memory_key = memory_key

    def emit_generic(self, verts: Vertices):
        from .computer import KeyValue
        p = verts.property(self.compute_key)
        if p is None:
            return []
        vals, present = p
        return [KeyValue(int(i), v.item()) for i, v, ok in zip(verts.ids, vals, present) if ok]

"""Host-side mirror of Titan's GraphComputer API for the OLAP path.

Same names, argument meaning and error behaviour as the reference, so the parity tests
read like OLAPTest:

    computer = graph.compute()                          # TitanBlueprintsGraph.java:133-146
    computer.resultMode(TitanGraphComputer.ResultMode.NONE)
    computer.workers(4)                                 # FulgoraGraphComputer.java:96-100
    computer.program(PageRankVertexProgram.build().iterations(10).vertexCount(n)
                     .dampingFactor(0.85).create(graph))
    computer.mapReduce(PageRankMapReduce.build().create())
    result = computer.submit().get()                    # FulgoraGraphComputer.java:117-311
    ranks = result.memory().get(PageRankMapReduce.DEFAULT_MEMORY_KEY)

What runs underneath is the HIP engine (titan_amd/engine.py -> libtitan_gpu_olap.so):
the graph's edgestore rows are decoded once per message-scope (the reference preloads the
reversed-scope slice every superstep, VertexProgramScanJob.getQueries :99-120) and each
program is one tgo_* call.  Failures surface as ExecutionException from get(), wrapping a
TitanException (OLAPTest.vertexProgramExceptionPropagatesToCaller, :222-239).
"""
from __future__ import annotations

import enum
import threading
from concurrent.futures import Future, ThreadPoolExecutor
from dataclasses import dataclass

import numpy as np

from . import _lib as L
from .engine import Engine, Schema, TitanException
from .generic import FulgoraMemory, GenericVertexProgram, preload_scope, run_generic

SCOPE_NAMES = {"outE": L.SCOPE_OUT_E, "inE": L.SCOPE_IN_E, "bothE": L.SCOPE_BOTH_E}


class ExecutionException(Exception):
    """java.util.concurrent.ExecutionException: raised by Future.get() on failure."""


class ComputerFuture:
    def __init__(self, fut: Future):
        self._f = fut

    def get(self, timeout=None):
        try:
            return self._f.result(timeout)
        except ExecutionException:
            raise
        except Exception as e:  # noqa: BLE001 - mirror CompletableFuture semantics
            raise ExecutionException(e) from e

    def done(self):
        return self._f.done()


@dataclass(frozen=True)
class KeyValue:
    key: int
    value: object

    def getKey(self):  # noqa: N802 - reference naming
        return self.key

    def getValue(self):  # noqa: N802
        return self.value


class Memory:
    """FulgoraMemory after complete(): iteration reports T (FulgoraMemory.java:73-76)."""

    def __init__(self, iteration, runtime_ms, values):
        self._it = iteration
        self._rt = runtime_ms
        self._values = values

    def getIteration(self):  # noqa: N802
        return self._it

    def getRuntime(self):  # noqa: N802
        return self._rt

    def exists(self, key):
        return key in self._values

    def get(self, key):
        if key not in self._values:
            raise KeyError(f"The memory does not have a value for provided key: {key}")
        v = self._values[key]
        return iter(v) if isinstance(v, list) else v

    def keys(self):
        return set(self._values)


# ----------------------------------------------------------------------------- write-back
def _relation_type_header(key_id: int) -> bytes:
    """IDHandler.writeRelationType(keyId, PROPERTY_DIR) for a user property key (:88-94): prefix
    0b010, then VariableLong.writePositiveWithPrefix(count << 1) (VariableLong.java:139-164)."""
    v = (key_id >> 6) << 1
    delta = 5
    first = 2 << delta
    vl = max(1, v.bit_length())
    mod = vl % 7
    if mod <= delta - 1:
        off = vl - mod
        first |= v >> off
        v &= (1 << off) - 1
        vl -= mod
    else:
        vl += 7 - mod
    if vl > 0:
        first |= 1 << (delta - 1)
    out = [first]
    while vl > 0:
        vl -= 7
        out.append(((v >> vl) & 0x7F) | (0x80 if vl == 0 else 0))
    return bytes(out)


def _row_key(vid: int, pb: int) -> int:
    """IDManager.getKey (IDManager.java:461-473), as a signed 64-bit long."""
    part = (vid >> 3) & ((1 << pb) - 1) if pb else 0
    key = ((part << (64 - pb)) if pb else 0) | ((vid >> (3 + pb)) << 3) | (vid & 7)
    return key - (1 << 64) if key >= (1 << 63) else key


def _row_entries(rows, r):
    base = int(rows.byte_begin[r])
    out, start = [], 0
    for e in range(int(rows.entry_begin[r]), int(rows.entry_begin[r + 1])):
        lv = int(rows.limit_valpos[e])
        end, vpos = lv >> 32, lv & 0x7FFFFFFF
        out.append((bytes(rows.data[base + start:base + end]), vpos))
        start = end
    return out


def merge_rows(store, mutations):
    """Apply result rows to a row store the way the backend applies mutations: per row key the
    entries are merged in column byte order and an entry whose column equals an existing one
    replaces it (single cardinality: the column is the property key alone)."""
    from .engine import Rows
    rows = {int(k): _row_entries(store, r) for r, k in enumerate(store.keys)}
    for r, k in enumerate(mutations.keys):
        cur = {e[0][:e[1]]: e for e in rows.get(int(k), [])}
        for e in _row_entries(mutations, r):
            cur[e[0][:e[1]]] = e
        rows[int(k)] = sorted(cur.values(), key=lambda e: e[0][:e[1]])
    keys = sorted(rows, key=lambda k: k & ((1 << 64) - 1))       # unsigned key order
    data, lv, eb, bb = bytearray(), [], [0], [0]
    for k in keys:
        start = len(data)
        for b, vpos in rows[k]:
            data += b
            lv.append(((len(data) - start) << 32) | vpos)
        eb.append(len(lv))
        bb.append(len(data))
    return Rows(np.asarray(keys, np.int64), np.asarray(eb, np.int64), np.asarray(bb, np.int64),
                np.frombuffer(bytes(data) or b"\0", np.uint8).copy(), np.asarray(lv or [0], np.int64))


def read_property(rows, vid: int, key_id: int, datatype: int, pb: int = 5):
    """The value of a SINGLE-cardinality property on a vertex's row (EdgeSerializer.parseRelation
    property branch :112-126), or None."""
    key = _row_key(vid, pb)
    idx = np.nonzero(rows.keys == key)[0]
    if len(idx) == 0:
        return None
    hdr = _relation_type_header(key_id)
    for b, vpos in _row_entries(rows, int(idx[0])):
        if b[:vpos] != hdr:
            continue
        if datatype == L.DT_OBJECT:
            # generic key: the value's class registration, then its serializer, no null flag
            # (StandardSerializer.readClassAndObject :247-252; Long 13, Double 20, Integer 12)
            cls = b[vpos] & 0x7F
            if b[vpos] == 0x80:
                return None
            datatype = {13: L.DT_LONG, 20: L.DT_DOUBLE, 12: L.DT_INTEGER}.get(cls)
            if datatype is None or not b[vpos] & 0x80:
                raise TitanException(L.TGO_E_UNSUPPORTED, f"generic value class {b[vpos]}")
        elif b[vpos] == 0xFF:
            return None
        v = b[vpos + 1:]
        if datatype == L.DT_LONG:
            return int.from_bytes(v[:8], "big") - (1 << 63)
        if datatype == L.DT_DOUBLE:
            return float(np.frombuffer(v[:8][::-1], np.float64)[0])
        if datatype == L.DT_INTEGER:
            u, i = 0, 0
            while True:
                u = (u << 7) | (v[i] & 0x7F)
                if v[i] & 0x80:
                    break
                i += 1
            return -(u >> 1) if u & 1 else u >> 1
        raise TitanException(L.TGO_E_UNSUPPORTED, f"datatype {datatype}")
    return None


class LocalTxGraph:
    """ResultMode LOCALTX: the graph seen through a new, uncommitted transaction that holds the
    computed properties (FulgoraGraphComputer.java:296-305, ResultGraph.NEW)."""

    def __init__(self, graph, mutations):
        self.graph = graph
        self.mutations = mutations

    def read_property(self, vid, key_id, datatype):
        v = read_property(self.mutations, vid, key_id, datatype, self.graph.partition_bits)
        return v if v is not None else self.graph.read_property(vid, key_id, datatype)


class ComputerResult:
    def __init__(self, graph, memory: Memory, vertex_properties):
        self._graph = graph
        self._memory = memory
        self.vertex_properties = vertex_properties   # compute key -> (titan_ids, values)

    def memory(self):
        return self._memory

    def graph(self):
        return self._graph


# ----------------------------------------------------------------------------- programs
class ResultGraph(enum.Enum):          # GraphComputer.ResultGraph
    ORIGINAL = 0
    NEW = 1


class Persist(enum.Enum):              # GraphComputer.Persist
    NOTHING = 0
    VERTEX_PROPERTIES = 1
    EDGES = 2


class VertexProgram:
    scope_name = "bothE"
    compute_keys: tuple = ()
    # getPreferredResultGraph / getPreferredPersist: what submit() uses when resultMode was
    # not set (FulgoraGraphComputer.java:133-135, GraphComputerHelper.getPersistState)
    preferred_result_graph = ResultGraph.ORIGINAL
    preferred_persist = Persist.VERTEX_PROPERTIES


class ShortestDistanceVertexProgram(VertexProgram):
    """tmain/olap/ShortestDistanceVertexProgram.java: Local(inE, m + e.value(weight))."""
    DISTANCE = "titan.shortestDistanceVertexProgram.distance"
    compute_keys = (DISTANCE,)

    def __init__(self, seed, max_depth, weight_property="distance", scope="inE", weighted=True, mode=L.SSSP_HOP_BOUNDED):
        self.seed = seed
        self.max_depth = max_depth
        self.weight_property = weight_property
        self.scope_name = scope
        self.weighted = weighted
        self.mode = mode

    class Builder:
        def __init__(self):
            self._seed = None
            self._max_depth = None
            self._weight = "distance"
            self._scope = "inE"
            self._weighted = True
            self._mode = L.SSSP_HOP_BOUNDED

        def seed(self, s):
            self._seed = int(s)
            return self

        def maxDepth(self, d):  # noqa: N802
            self._max_depth = int(d)
            return self

        def weightProperty(self, name):  # noqa: N802
            self._weight = name
            return self

        def scope(self, name):
            self._scope = name
            return self

        def unitWeight(self):  # noqa: N802 - BFS / k-hop: edge function m -> m + 1
            self._weighted = False
            return self

        def deltaStepping(self):  # noqa: N802
            """Converged shortest distances by delta-stepping (TGO_SSSP_DELTA) instead of
            maxDepth Jacobi supersteps.  Equal to ShortestDistanceVertexProgram's result only
            when every shortest path has at most maxDepth hops: the reference stops after
            maxDepth supersteps (ShortestDistanceVertexProgram.java:128-130) and leaves longer
            paths at their bounded distance; this mode does not check the hop count.  Use the
            default (hop-bounded) mode for exact reference semantics at small maxDepth."""
            self._mode = L.SSSP_DELTA
            return self

        def create(self, graph=None):
            if self._seed is None or self._max_depth is None:
                raise ValueError("seed and maxDepth are required (configuration.getInt(MAX_DEPTH))")
            return ShortestDistanceVertexProgram(self._seed, self._max_depth, self._weight, self._scope,
                                                 self._weighted, self._mode)

    @staticmethod
    def build():
        return ShortestDistanceVertexProgram.Builder()


class PageRankVertexProgram(VertexProgram):
    """tmain/olap/PageRankVertexProgram.java:45-100 (scopes outE + inE)."""
    PAGE_RANK = "titan.pageRank.pageRank"
    OUTGOING_EDGE_COUNT = "titan.pageRank.edgeCount"
    compute_keys = (PAGE_RANK, OUTGOING_EDGE_COUNT)
    scope_name = "inE"

    def __init__(self, alpha=0.85, max_iterations=10, vertex_count=1):
        self.alpha = alpha
        self.max_iterations = max_iterations
        self.vertex_count = vertex_count

    class Builder:
        def __init__(self):
            self._a, self._it, self._n = 0.85, 10, 1          # loadState defaults (:52-54)

        def vertexCount(self, n):  # noqa: N802
            self._n = int(n)
            return self

        def dampingFactor(self, a):  # noqa: N802
            self._a = float(a)
            return self

        def iterations(self, k):
            self._it = int(k)
            return self

        def create(self, graph=None):
            return PageRankVertexProgram(self._a, self._it, self._n)

    @staticmethod
    def build():
        return PageRankVertexProgram.Builder()


class DegreeCounter(VertexProgram):
    """tmain/olap/OLAPTest.java:334-416 — k-walk counts over inE, Java int wrap."""
    DEGREE = "degree"
    compute_keys = (DEGREE,)
    scope_name = "inE"
    preferred_result_graph = ResultGraph.NEW          # OLAPTest.java:391-398

    def __init__(self, length=1):
        if length <= 0:
            raise ValueError("length must be > 0")      # Preconditions.checkArgument(length>0)
        self.length = length


# ----------------------------------------------------------------------------- map-reduces
class MapReduce:
    memory_key = ""


class PageRankMapReduce(MapReduce):
    DEFAULT_MEMORY_KEY = "pageRank"     # PageRankMapReduce.java:19

    def __init__(self, key=DEFAULT_MEMORY_KEY):
        self.memory_key = key

    class Builder:
        def __init__(self):
            self._k = PageRankMapReduce.DEFAULT_MEMORY_KEY

        def memoryKey(self, k):  # noqa: N802
            self._k = k
            return self

        def create(self):
            return PageRankMapReduce(self._k)

    @staticmethod
    def build():
        return PageRankMapReduce.Builder()

    def emit(self, ids, props):
        pr = props.get(PageRankVertexProgram.PAGE_RANK)
        if pr is None:
            return []
        # map() emits only vertices where the property is present (:45-50)
        return [KeyValue(int(i), float(v)) for i, v in zip(ids, pr) if not np.isnan(v)]


class ShortestDistanceMapReduce(MapReduce):
    DEFAULT_MEMORY_KEY = "shortestDistance"   # ShortestDistanceMapReduce.java:16

    def __init__(self, key=DEFAULT_MEMORY_KEY):
        self.memory_key = key

    class Builder:
        def __init__(self):
            self._k = ShortestDistanceMapReduce.DEFAULT_MEMORY_KEY

        def memoryKey(self, k):  # noqa: N802
            self._k = k
            return self

        def create(self):
            return ShortestDistanceMapReduce(self._k)

    @staticmethod
    def build():
        return ShortestDistanceMapReduce.Builder()

    def emit(self, ids, props):
        d = props.get(ShortestDistanceVertexProgram.DISTANCE)
        if d is None:
            return []
        return [KeyValue(int(i), int(v)) for i, v in zip(ids, d) if v != L.DIST_ABSENT]


class DegreeMapper(MapReduce):
    DEGREE_RESULT = "degrees"                 # OLAPTest.java:420
    memory_key = DEGREE_RESULT

    def emit(self, ids, props):
        d = props.get(DegreeCounter.DEGREE)
        return {int(i): int(v) for i, v in zip(ids, d)} if d is not None else {}


# ----------------------------------------------------------------------------- graph / computer
class GpuGraph:
    """An edgestore snapshot: rows (as a scan returns them) + schema.  The engine preloads
    the slice each message scope needs, once, and keeps it resident on the device."""

    def __init__(self, rows=None, schema=None, edges=None, device=0, partition_bits=5, hard_query_limit=100000,
                 apply_cap=True, property_keys=None, relation_id_base=1 << 40):
        self.rows = rows
        # compute-key name -> (PropertyKey schema id, tgo datatype): the typed keys write-back uses
        self.property_keys = dict(property_keys or {})
        self._next_relation_id = relation_id_base     # the IDAuthority block result writes draw from
        self._schema_dict = schema if isinstance(schema, dict) else None
        self.schema = schema if (schema is None or isinstance(schema, Schema)) else Schema.from_dict(schema)
        self.edges = edges       # (n, src, dst, weight) decoded-adjacency input
        self.device = device
        self.partition_bits = partition_bits
        self.hard_query_limit = hard_query_limit
        self.apply_cap = apply_cap
        self._engines = {}
        self._lock = threading.Lock()

    def compute(self):
        return GpuGraphComputer(self)

    def property_key(self, name):
        """(schema id, tgo datatype) of a compute key; a key the graph has no schema for is
        created the way getOrCreatePropertyKey does with the default schema maker: a generic
        key, dataType(Object.class) (DefaultSchemaMaker.java:46-48), whose values carry their
        class.  Ids continue after the largest schema id in use."""
        with self._lock:
            k = self.property_keys.get(name)
            if k is None:
                used = [int(i) >> 6 for i, _ in self.property_keys.values()]
                if self._schema_dict is not None:
                    used += [int(t["type_id"]) >> 6 for t in self._schema_dict.get("edge_types", [])]
                    used += [int(p[0]) >> 6 for p in self._schema_dict.get("property_keys", [])]
                k = (((max(used, default=0) + 1) << 6) | 5, L.DT_OBJECT)     # IDManager: UserPropertyKey
                self.property_keys[name] = k
            return k

    def reserve_relation_ids(self, count):
        with self._lock:
            base = self._next_relation_id
            self._next_relation_id += max(1, count)
            return base

    def persist(self, mutations):
        """Commit result rows to the store (VertexPropertyWriter's batched transactions)."""
        if self.rows is None:
            raise TitanException(L.TGO_E_UNSUPPORTED, "write-back needs an edgestore-backed graph")
        with self._lock:
            self.rows = merge_rows(self.rows, mutations)

    def read_property(self, vid, key_id, datatype):
        return None if self.rows is None else read_property(self.rows, vid, key_id, datatype, self.partition_bits)

    def engine_for(self, scope: int, weight_key: int = 0, column_order: bool = False) -> Engine:
        key = (scope, weight_key, column_order)
        with self._lock:
            if key not in self._engines:
                eng = Engine(self.device, self.partition_bits, hard_query_limit=self.hard_query_limit)
                if self.rows is not None:
                    eng.load_rows(self.rows, self.schema, scope, apply_cap=self.apply_cap, weight_key=weight_key,
                                  column_order=column_order)
                else:
                    n, src, dst, w = self.edges
                    eng.load_edges(n, src, dst, scope, weight=w if weight_key else None, apply_cap=self.apply_cap,
                                   column_order=column_order)
                self._engines[key] = eng
            return self._engines[key]


class TitanGraphComputer:
    class ResultMode(enum.Enum):          # core/TitanGraphComputer.java:10-31
        NONE = 0
        PERSIST = 1
        LOCALTX = 2


_POOL = ThreadPoolExecutor(max_workers=4, thread_name_prefix="tgo-submit")


class GpuGraphComputer(TitanGraphComputer):
    """Drop-in for FulgoraGraphComputer on the OLAP path."""

    def __init__(self, graph: GpuGraph):
        self.graph = graph
        self._program = None
        self._map_reduces = []
        self._workers = 1
        self._mode = None                # unset: the program's preference (see _result_mode)
        self._executed = False
        self.weight_keys = {}            # weight property name -> key id (schema lookup)

    def workers(self, threads: int):
        if threads <= 0:
            raise ValueError(f"Invalid number of threads: {threads}")
        self._workers = threads
        return self

    def resultMode(self, mode):  # noqa: N802
        """core/TitanGraphComputer.java:10-37.  NONE: results only in memory / MapReduce.
        PERSIST: the compute keys are written back to the graph (FulgoraGraphComputer.java:
        248-295, ResultGraph.ORIGINAL + Persist.VERTEX_PROPERTIES).  LOCALTX: they are held by a
        new uncommitted transaction returned as the result graph (:296-305)."""
        self._mode = TitanGraphComputer.ResultMode(mode)
        return self

    # compute key name -> (tgo result kind, slot) for the natively run programs
    _RESULT_KEYS = {ShortestDistanceVertexProgram: (L.RESULT_DISTANCE, (ShortestDistanceVertexProgram.DISTANCE,)),
                    PageRankVertexProgram: (L.RESULT_PAGERANK, (PageRankVertexProgram.PAGE_RANK,
                                                                PageRankVertexProgram.OUTGOING_EDGE_COUNT)),
                    DegreeCounter: (L.RESULT_DEGREE, (DegreeCounter.DEGREE,))}

    def _result_mode(self):
        """resultMode if set, else the program's preferred (ResultGraph, Persist) as Fulgora
        takes them (FulgoraGraphComputer.java:133-135): PageRank and ShortestDistance persist
        into the original graph, DegreeCounter into a new one (LOCALTX); no program: NONE.
        (whether the mode was explicit, the mode)"""
        if self._mode is not None:
            return True, self._mode
        p = self._program
        if p is None or getattr(p, "preferred_persist", None) in (None, Persist.NOTHING):
            return False, TitanGraphComputer.ResultMode.NONE
        if getattr(p, "preferred_result_graph", ResultGraph.ORIGINAL) == ResultGraph.NEW:
            return False, TitanGraphComputer.ResultMode.LOCALTX
        return False, TitanGraphComputer.ResultMode.PERSIST

    def _write_back(self, eng):
        """Encode the last program's compute keys on the device (tgo_result_rows) and persist
        them (PERSIST) or hand them to a local transaction (LOCALTX)."""
        explicit, mode = self._result_mode()
        if mode == TitanGraphComputer.ResultMode.NONE:
            return self.graph
        if self.graph.rows is None and not explicit:
            # a graph given as an already-decoded adjacency has no store to write into: the
            # program's preference cannot apply (an explicit PERSIST / LOCALTX still fails)
            return self.graph
        spec = self._RESULT_KEYS.get(type(self._program))
        if spec is None:
            raise TitanException(L.TGO_E_UNSUPPORTED, f"write-back of {type(self._program).__name__} compute keys")
        kind, names = spec
        keys = [self.graph.property_key(k) for k in names]
        base = self.graph.reserve_relation_ids(eng.n * len(keys))
        rows = eng.result_rows(kind, [k for k, _ in keys], [d for _, d in keys], base)
        if mode == TitanGraphComputer.ResultMode.PERSIST:
            self.graph.persist(rows)
            return self.graph
        return LocalTxGraph(self.graph, rows)

    def program(self, program: VertexProgram):
        if self._program is not None:
            raise RuntimeError("A vertex program has already been set")
        self._program = program
        return self

    def mapReduce(self, mr: MapReduce):  # noqa: N802
        self._map_reduces.append(mr)
        return self

    def submit(self) -> ComputerFuture:
        if self._executed:
            raise RuntimeError("This computer has already executed a vertex program")
        self._executed = True
        if self._program is None and not self._map_reduces:
            raise RuntimeError("The computer has no vertex program or map reducers to execute")
        return ComputerFuture(_POOL.submit(self._run))

    def _run(self):
        import time
        t0 = time.perf_counter()
        p = self._program
        props = {}
        iteration = 0
        if isinstance(p, GenericVertexProgram):
            return self._run_generic(p, t0)
        if isinstance(p, ShortestDistanceVertexProgram):
            scope = SCOPE_NAMES[p.scope_name]
            wk = 0
            if p.weighted:
                wk = self.weight_keys.get(p.weight_property, 0)
                if wk == 0:
                    raise TitanException(L.TGO_E_INVALID, f"weight property '{p.weight_property}' has no key id")
            eng = self.graph.engine_for(scope, wk)
            if p.weighted or p.mode == L.SSSP_DELTA:
                d = eng.sssp(p.seed, p.max_depth, scope, mode=p.mode)
            else:
                d = eng.bfs(p.seed, p.max_depth, scope)
            props[ShortestDistanceVertexProgram.DISTANCE] = d
            iteration = p.max_depth
            ids = eng.vertex_ids()
        elif isinstance(p, PageRankVertexProgram):
            eng = self.graph.engine_for(L.SCOPE_IN_E)
            props[PageRankVertexProgram.PAGE_RANK] = eng.pagerank(p.alpha, p.vertex_count, p.max_iterations)
            iteration = p.max_iterations
            ids = eng.vertex_ids()
        elif isinstance(p, DegreeCounter):
            eng = self.graph.engine_for(L.SCOPE_IN_E)
            props[DegreeCounter.DEGREE] = eng.walkcount(p.length)
            iteration = p.length
            ids = eng.vertex_ids()
        else:
            raise TitanException(L.TGO_E_UNSUPPORTED, f"vertex program {type(p).__name__} is not supported on the GPU path")
        values = {}
        for mr in self._map_reduces:
            values[mr.memory_key] = mr.emit(ids, props)
        result_graph = self._write_back(eng)
        rt = (time.perf_counter() - t0) * 1000.0
        vprops = {k: (ids, v) for k, v in props.items()}
        return ComputerResult(result_graph, Memory(iteration, rt, values), vprops)

    def _run_generic(self, p, t0):
        """Vectorised program: Fulgora's superstep loop on the host, messages combined on the
        device (titan_amd/generic.py)."""
        import time
        scope = preload_scope(p, probe_memory_iterations=3)
        wk = 0
        if p.weight_property is not None:
            wk = self.weight_keys.get(p.weight_property, 0)
            if wk == 0:
                raise TitanException(L.TGO_E_INVALID, f"weight property '{p.weight_property}' has no key id")
        # a combiner-less program reads message streams: keep the column order for them
        eng = self.graph.engine_for(scope, wk, column_order=p.combiner is None)
        memory = FulgoraMemory(tuple(p.memory_compute_keys) + tuple(mr.memory_key for mr in self._map_reduces))
        verts = run_generic(eng, p, memory)
        memory.setRuntime((time.perf_counter() - t0) * 1000.0)
        memory.complete()
        values = dict(memory.previous)
        for mr in self._map_reduces:
            values[mr.memory_key] = mr.emit_generic(verts)
        vprops = {k: (verts.ids, v) for k, v in verts._props.items() if v is not None}
        result_graph = self._write_back_generic(eng, verts)
        return ComputerResult(result_graph, Memory(memory.getIteration(), memory.getRuntime(), values), vprops)

    def _write_back_generic(self, eng, verts):
        """A generic program's element compute keys written back like Fulgora writes every
        vertex's mutable properties (FulgoraGraphComputer.java:248-305): one SINGLE-cardinality
        entry per vertex holding the key, encoded on the device (tgo_result_rows_values).
        int64 values go to a Long / Integer key, fp64 values to a Double key; a key without a
        schema becomes a generic key (getOrCreatePropertyKey)."""
        explicit, mode = self._result_mode()
        if mode == TitanGraphComputer.ResultMode.NONE or (self.graph.rows is None and not explicit):
            return self.graph
        merged = None
        for name in self._program.compute_keys:
            prop = verts.property(name)
            if prop is None:
                continue
            vals, present = prop
            vals = np.asarray(vals)
            if vals.dtype.kind in "iu":
                vt, ok = L.VAL_INT64, (L.DT_LONG, L.DT_INTEGER, L.DT_OBJECT)
            elif vals.dtype.kind == "f":
                vt, ok = L.VAL_FP64, (L.DT_DOUBLE, L.DT_OBJECT)
            else:
                raise TitanException(L.TGO_E_UNSUPPORTED, f"compute key {name}: values of dtype {vals.dtype}")
            key, dt = self.graph.property_key(name)
            if dt not in ok:
                raise TitanException(L.TGO_E_INVALID, f"compute key {name}: its PropertyKey datatype {dt} does not "
                                                      f"hold {vals.dtype} values")
            base = self.graph.reserve_relation_ids(int(np.count_nonzero(present)))
            rows = eng.result_rows_values(key, dt, vt, vals, present, base)
            merged = rows if merged is None else merge_rows(merged, rows)
        if merged is None:
            return self.graph
        if mode == TitanGraphComputer.ResultMode.PERSIST:
            self.graph.persist(merged)
            return self.graph
        return LocalTxGraph(self.graph, merged)

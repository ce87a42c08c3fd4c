"""The scan SPI of the GPU path, host side.

Restates the reference's scan contract so the engine's row intake runs under the same rules
the Java host uses (`java/.../olap/gpu/CsrCollectingScanJob.java` over the unchanged
`StandardScanner`):

* `SliceQuery` — [start, end) over unsigned column bytes, optional limit
  (diskstorage/keycolumnvalue/SliceQuery.java:60-104);
* `ScanJob` — the job SPI: workerIterationStart / workerIterationEnd / process / getQueries /
  getKeyFilter / clone (diskstorage/keycolumnvalue/scan/ScanJob.java:17-130);
* `StandardScanner.execute` — StandardScannerExecutor.run (:85-188): the first of several
  queries must be grounded (start = one 0x00 byte, end = all 0xFF), one key stream per query
  filtered by the job's key filter, rows emitted in key order for every key the grounding
  query returns, each query's entries (or an empty list) per row, processors that clone the
  job every `workBlockSize` rows (:235-288), SUCCESS / FAILURE metrics;
* `CsrCollectingScanJob` — VertexJobConverter's queries (VERTEX_EXISTS_QUERY first, then the
  program scope's user-edge slice with the QueryContainer limit; VertexJobConverter.java:39,
  140-152) whose `process` appends each row in StaticArrayEntryList form and hands full work
  blocks to `tgo_load_rows`.

The store here is an in-memory ordered key-column-value map (what a backend's getKeys +
getSlice return); nothing in this module touches the device except `tgo_load_rows`.
"""
from __future__ import annotations

import bisect
import threading
from collections import defaultdict

import numpy as np

from . import _lib as L
from .engine import Engine, Rows, TitanException


def _ukey(b: bytes):
    return b                                     # bytes compare unsigned-lexicographically


class SliceQuery:
    """SliceQuery.java: columns c with start <= c < end (unsigned byte order), at most `limit`."""

    def __init__(self, start: bytes, end: bytes, limit: int | None = None):
        self.start, self.end, self.limit = bytes(start), bytes(end), limit

    def setLimit(self, limit):  # noqa: N802
        return SliceQuery(self.start, self.end, limit)

    def hasLimit(self):  # noqa: N802
        return self.limit is not None

    def __eq__(self, o):
        return isinstance(o, SliceQuery) and (self.start, self.end, self.limit) == (o.start, o.end, o.limit)

    def __hash__(self):
        return hash((self.start, self.end, self.limit))

    def __repr__(self):
        return f"SliceQuery({self.start.hex()}, {self.end.hex()}, limit={self.limit})"


def zero_buffer(n):
    return b"\x00" * n


def one_buffer(n):
    return b"\xff" * n


class InMemoryStore:
    """Ordered key -> [(column, value)] (columns sorted); getSlice as a backend answers it."""

    def __init__(self):
        self.rows = {}

    def put(self, key: bytes, entries):
        self.rows[bytes(key)] = sorted((bytes(c), bytes(v)) for c, v in entries)

    @classmethod
    def from_rows(cls, rows: Rows):
        """From the tgo_rows layout (8-byte big-endian keys, (limit << 32 | valuePos))."""
        s = cls()
        for r in range(rows.nrows):
            key = int(rows.keys[r]).to_bytes(8, "big", signed=True)
            base, start, ents = int(rows.byte_begin[r]), 0, []
            for e in range(int(rows.entry_begin[r]), int(rows.entry_begin[r + 1])):
                lv = int(rows.limit_valpos[e])
                end, vpos = lv >> 32, lv & 0x7FFFFFFF
                b = bytes(rows.data[base + start:base + end])
                ents.append((b[:vpos], b[vpos:]))
                start = end
            s.rows[key] = ents
        return s

    def keys(self):
        return sorted(self.rows, key=_ukey)

    def get_slice(self, key: bytes, q: SliceQuery):
        cols = self.rows.get(key, [])
        lo = bisect.bisect_left(cols, (q.start, b""))
        out = []
        for c, v in cols[lo:]:
            if c >= q.end or (q.limit is not None and len(out) >= q.limit):
                break
            out.append((c, v))
        return out


class ScanMetrics:
    SUCCESS, FAILURE = "success", "failure"

    def __init__(self):
        self._lock = threading.Lock()
        self.custom = defaultdict(int)
        self.metric = defaultdict(int)

    def incrementCustom(self, name, delta=1):  # noqa: N802
        with self._lock:
            self.custom[name] += delta

    def getCustom(self, name):  # noqa: N802
        return self.custom.get(name, 0)

    def increment(self, metric):
        with self._lock:
            self.metric[metric] += 1

    def get(self, metric):
        return self.metric.get(metric, 0)


class ScanJob:
    """ScanJob.java:17-130 (the methods the executor calls)."""

    def workerIterationStart(self, config, graph_config, metrics):  # noqa: N802
        pass

    def workerIterationEnd(self, metrics):  # noqa: N802
        pass

    def process(self, key: bytes, entries: dict, metrics: ScanMetrics):
        raise NotImplementedError

    def getQueries(self):  # noqa: N802
        raise NotImplementedError

    def getKeyFilter(self):  # noqa: N802
        return lambda key: True

    def clone(self):
        raise NotImplementedError


class ScanException(TitanException):
    pass


class StandardScanner:
    """StandardScanner.Builder + StandardScannerExecutor.run over an InMemoryStore."""

    def __init__(self, store: InMemoryStore):
        self.store = store

    def execute(self, job: ScanJob, config=None, graph_config=None, num_processors=1, work_block_size=10000):
        metrics = ScanMetrics()
        job.workerIterationStart(config, graph_config, metrics)
        try:
            queries = list(job.getQueries())
            if not queries:
                raise ScanException(L.TGO_E_INVALID, f"Must at least specify one query for job: {job}")
            if len(queries) > 1:             # :92-101 the first query grounds the scan
                g = queries[0]
                if g.start != zero_buffer(1):
                    raise ScanException(L.TGO_E_INVALID, f"Expected start of first query to be a single 0s: {g.start.hex()}")
                if g.end != one_buffer(len(g.end)):
                    raise ScanException(L.TGO_E_INVALID, f"Expected end of first query to be all 1s: {g.end.hex()}")
            keyfilter = job.getKeyFilter()
            # one data puller per query: the keys with entries in that slice, key-filtered
            # (KCVSUtil.getKeys + DataPuller), as (key, entries) in key order
            streams = []
            for q in queries:
                res = {}
                for k in self.store.keys():
                    if not keyfilter(k):
                        continue
                    ents = self.store.get_slice(k, q)
                    if ents:
                        res[k] = ents
                streams.append(res)
        finally:
            job.workerIterationEnd(metrics)
        # merge join on the grounding query (:123-152)
        rows = []
        for k in sorted(streams[0], key=_ukey):
            rows.append((k, {q: streams[i].get(k, []) for i, q in enumerate(queries)}))
        # processors: contiguous shares of the row queue, a fresh job clone per work block
        lock = threading.Lock()
        it = iter(rows)

        def processor():
            pjob = job.clone()
            pjob.workerIterationStart(config, graph_config, metrics)
            done = 0
            try:
                while True:
                    with lock:
                        row = next(it, None)
                    if row is None:
                        break
                    if done >= work_block_size:
                        pjob.workerIterationEnd(metrics)
                        pjob = pjob.clone()
                        pjob.workerIterationStart(config, graph_config, metrics)
                        done = 0
                    try:
                        pjob.process(row[0], row[1], metrics)
                        metrics.increment(ScanMetrics.SUCCESS)
                    except Exception:
                        metrics.increment(ScanMetrics.FAILURE)
                    done += 1
            finally:
                pjob.workerIterationEnd(metrics)

        threads = [threading.Thread(target=processor) for _ in range(max(1, num_processors))]
        for t in threads:
            t.start()
        for t in threads:
            t.join()
        return metrics


# ----------------------------------------------------------------------------- CSR collector
VERTEX_EXISTS_QUERY = SliceQuery(zero_buffer(1), one_buffer(4), 1)     # VertexJobConverter.java:39
USER_EDGE_SLICE = (b"\x60", b"\x80")                                    # user edge labels (IDHandler prefix 011)


class CsrCollectingScanJob(ScanJob):
    """The GPU path's VertexScanJob stand-in: asks for VertexJobConverter's queries and feeds
    every processor's rows to tgo_load_rows one work block at a time (the engine decodes,
    filters ghosts and counts truncated lists exactly as VertexJobConverter.process does)."""

    def __init__(self, engine: Engine, schema, scope, hard_limit=100000, apply_cap=True, labels=(), weight_key=0,
                 _shared=None):
        self.engine, self.schema, self.scope = engine, schema, scope
        self.hard_limit, self.apply_cap, self.labels, self.weight_key = hard_limit, apply_cap, tuple(labels), weight_key
        self._shared = _shared if _shared is not None else {"lock": threading.Lock()}
        self._block = []

    def getQueries(self):  # noqa: N802
        fitted = self.scope == L.SCOPE_BOTH_E or len(self.labels) > 0     # BasicVertexCentricQueryBuilder :418-474
        limit = None if (fitted or not self.apply_cap) else self.hard_limit
        return [VERTEX_EXISTS_QUERY, SliceQuery(*USER_EDGE_SLICE, limit)]

    def getKeyFilter(self):  # noqa: N802
        return lambda key: True             # the engine applies IDManager's key filter (Invisible ids)

    def clone(self):
        return CsrCollectingScanJob(self.engine, self.schema, self.scope, self.hard_limit, self.apply_cap, self.labels,
                                    self.weight_key, self._shared)

    def process(self, key, entries, metrics):
        q0, q1 = self.getQueries()
        ents = list(entries.get(q0, [])) + [e for e in entries.get(q1, []) if e not in entries.get(q0, [])]
        self._block.append((key, ents))

    def workerIterationEnd(self, metrics):  # noqa: N802
        if not self._block:
            return
        keys, eb, bb, data, lv = [], [0], [0], bytearray(), []
        for key, ents in self._block:
            start = len(data)
            for c, v in ents:
                data += c + v
                lv.append(((len(data) - start) << 32) | len(c))
            keys.append(int.from_bytes(key, "big", signed=True))
            eb.append(len(lv))
            bb.append(len(data))
        rows = Rows(np.asarray(keys, np.int64), np.asarray(eb, np.int64), np.asarray(bb, np.int64),
                    np.frombuffer(bytes(data) or b"\0", np.uint8).copy(), np.asarray(lv or [0], np.int64))
        self._block = []
        with self._shared["lock"]:          # one ctx is used by one thread at a time
            self.engine.append_rows(rows, self.schema, self.scope, apply_cap=self.apply_cap, labels=self.labels,
                                    weight_key=self.weight_key)


def scan_into_engine(engine: Engine, store: InMemoryStore, schema, scope, hard_limit=100000, apply_cap=True,
                     labels=(), weight_key=0, num_processors=1, work_block_size=10000):
    """One StandardScanner run of the CSR-collecting job, then tgo_finish_load."""
    job = CsrCollectingScanJob(engine, schema, scope, hard_limit, apply_cap, labels, weight_key)
    metrics = StandardScanner(store).execute(job, num_processors=num_processors, work_block_size=work_block_size)
    if metrics.get(ScanMetrics.FAILURE):
        raise ScanException(L.TGO_E_CODEC, f"Failed to process [{metrics.get(ScanMetrics.FAILURE)}] rows")
    engine.finish_rows()
    return metrics

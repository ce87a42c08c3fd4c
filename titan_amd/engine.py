"""Object wrapper over the C-ABI: one Engine = one tgo_ctx (one device)."""
from __future__ import annotations

import ctypes as C

import numpy as np

from . import _lib as L


class TitanException(RuntimeError):
    """Mirrors com.thinkaurelius.titan.core.TitanException (status + message of the C-ABI)."""

    def __init__(self, code: int, message: str):
        super().__init__(f"[{code}] {message}")
        self.code = code


def _check(lib, ctx, rc):
    if rc != L.TGO_OK:
        msg = lib.tgo_last_error(ctx).decode(errors="replace") if ctx else "tgo_create failed"
        raise TitanException(rc, msg)


class Schema:
    """Edge-label / property-key schema (what tx.getExistingRelationType resolves)."""

    def __init__(self, edge_types, property_keys):
        self._keep = []
        et = (L.EdgeType * max(1, len(edge_types)))()
        for i, t in enumerate(edge_types):
            sk = np.ascontiguousarray(t.get("sort_key", []), dtype=np.int64)
            sg = np.ascontiguousarray(t.get("signature", []), dtype=np.int64)
            self._keep += [sk, sg]
            et[i] = L.EdgeType(t["type_id"], t["multiplicity"], len(sk), L.ptr(sk, C.c_int64),
                               len(sg), 1 if t.get("order", "ASC") == "DESC" else 0, L.ptr(sg, C.c_int64))
        pk = (L.PropertyKey * max(1, len(property_keys)))()
        for i, (kid, dt) in enumerate(property_keys):
            pk[i] = L.PropertyKey(kid, dt)
        self._keep += [et, pk]
        self.c = L.Schema(len(edge_types), et, len(property_keys), pk)

    @classmethod
    def from_dict(cls, d):
        return cls(d["edge_types"], [tuple(x) for x in d["property_keys"]])


class Engine:
    def __init__(self, device: int = 0, partition_bits: int = 5, host_threads: int = 0,
                 hard_query_limit: int = 100000, stream: int = 0):
        """stream: a HIP stream handle the ctx runs on (stream-ordered with the caller's
        work); 0 = a ctx-owned stream (the handle of torch's default stream is also 0, so a
        caller that wants ordering with torch must run on a non-default stream)."""
        self.lib = L.load()
        o = L.Options()
        self.lib.tgo_default_options(C.byref(o))
        o.device = device
        o.partition_bits = partition_bits
        o.host_threads = host_threads
        o.hard_query_limit = hard_query_limit
        o.stream = stream or None
        self.stream = int(stream or 0)
        h = C.c_void_p()
        rc = self.lib.tgo_create(C.byref(o), C.byref(h))
        if rc != L.TGO_OK:
            raise TitanException(rc, "tgo_create failed: no usable gfx950 device "
                                     "(the engine has no CPU fallback)")
        self.ctx = h
        self.n = 0

    def close(self):
        if getattr(self, "ctx", None):
            self.lib.tgo_destroy(self.ctx)
            self.ctx = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    # ------------------------------------------------------------------ loads
    @staticmethod
    def _opts(scope, apply_cap, labels, weight_key, flags=0):
        lab = np.ascontiguousarray(labels, dtype=np.int64)
        o = L.LoadOpts(scope=scope, apply_cap=1 if apply_cap else 0, n_labels=len(lab), flags=flags,
                       label_ids=L.ptr(lab, C.c_int64) if len(lab) else None, weight_key=weight_key)
        return o, lab

    def load_rows(self, rows, schema: Schema, scope, apply_cap=True, labels=(), weight_key=0, batch_rows=None,
                  column_order=False):
        """Feed scanned rows (optionally in work blocks) and finish the load.  column_order:
        keep each entry's column position (gather_lists hands messages over in column order)."""
        opts, keep = self._opts(scope, apply_cap, labels, weight_key, L.LOAD_COLUMN_ORDER if column_order else 0)
        nrows = rows.nrows
        step = batch_rows or max(nrows, 1)
        for r0 in range(0, max(nrows, 1), step):
            r1 = min(nrows, r0 + step)
            eb = rows.entry_begin[r0:r1 + 1]
            bb = rows.byte_begin[r0:r1 + 1]
            keys = np.ascontiguousarray(rows.keys[r0:r1])
            eb0 = np.ascontiguousarray(eb - eb[0])
            bb0 = np.ascontiguousarray(bb - bb[0])
            data = np.ascontiguousarray(rows.data[bb[0]:max(bb[-1], bb[0] + 1)])
            lv = np.ascontiguousarray(rows.limit_valpos[eb[0]:max(eb[-1], eb[0] + 1)])
            cr = L.Rows(r1 - r0, L.ptr(keys, C.c_int64), L.ptr(eb0, C.c_int64), L.ptr(bb0, C.c_int64),
                        L.ptr(data, C.c_uint8), L.ptr(lv, C.c_int64))
            _check(self.lib, self.ctx, self.lib.tgo_load_rows(self.ctx, C.byref(cr), C.byref(schema.c), C.byref(opts)))
        _check(self.lib, self.ctx, self.lib.tgo_finish_load(self.ctx))
        self.n = self.lib.tgo_num_vertices(self.ctx)
        return self

    @staticmethod
    def _row_block(rows, r0, r1):
        """Rows [r0, r1) as a tgo_rows (offsets rebased) and the arrays it points into."""
        eb = rows.entry_begin[r0:r1 + 1]
        bb = rows.byte_begin[r0:r1 + 1]
        keys = np.ascontiguousarray(rows.keys[r0:r1], dtype=np.int64)
        eb0 = np.ascontiguousarray(eb - eb[0], dtype=np.int64)
        bb0 = np.ascontiguousarray(bb - bb[0], dtype=np.int64)
        data = np.ascontiguousarray(rows.data[bb[0]:max(bb[-1], bb[0] + 1)], dtype=np.uint8)
        lv = np.ascontiguousarray(rows.limit_valpos[eb[0]:max(eb[-1], eb[0] + 1)], dtype=np.int64)
        cr = L.Rows(r1 - r0, L.ptr(keys, C.c_int64), L.ptr(eb0, C.c_int64), L.ptr(bb0, C.c_int64),
                    L.ptr(data, C.c_uint8), L.ptr(lv, C.c_int64))
        return cr, (keys, eb0, bb0, data, lv)

    def append_rows(self, rows, schema: Schema, scope, apply_cap=True, labels=(), weight_key=0):
        """One work block of scanned rows (tgo_load_rows without finishing the load)."""
        opts, keep = self._opts(scope, apply_cap, labels, weight_key)
        keys = np.ascontiguousarray(rows.keys, dtype=np.int64)
        eb = np.ascontiguousarray(rows.entry_begin, dtype=np.int64)
        bb = np.ascontiguousarray(rows.byte_begin, dtype=np.int64)
        data = np.ascontiguousarray(rows.data, dtype=np.uint8)
        lv = np.ascontiguousarray(rows.limit_valpos, dtype=np.int64)
        cr = L.Rows(rows.nrows, L.ptr(keys, C.c_int64), L.ptr(eb, C.c_int64), L.ptr(bb, C.c_int64),
                    L.ptr(data, C.c_uint8), L.ptr(lv, C.c_int64))
        _check(self.lib, self.ctx, self.lib.tgo_load_rows(self.ctx, C.byref(cr), C.byref(schema.c), C.byref(opts)))
        return self

    def finish_rows(self):
        _check(self.lib, self.ctx, self.lib.tgo_finish_load(self.ctx))
        self.n = self.lib.tgo_num_vertices(self.ctx)
        return self

    def load_edges(self, n, src, dst, scope, weight=None, titan_ids=None, apply_cap=True, weight_key=0,
                   column_order=False):
        src = np.ascontiguousarray(src, dtype=np.int32)
        dst = np.ascontiguousarray(dst, dtype=np.int32)
        w = None if weight is None else np.ascontiguousarray(weight, dtype=np.int32)
        t = None if titan_ids is None else np.ascontiguousarray(titan_ids, dtype=np.int64)
        e = L.Edges(n, len(src), L.ptr(src, C.c_int32), L.ptr(dst, C.c_int32), L.ptr(w, C.c_int32),
                    L.ptr(t, C.c_int64))
        opts, keep = self._opts(scope, apply_cap, (), weight_key, L.LOAD_COLUMN_ORDER if column_order else 0)
        if w is not None and weight_key == 0:
            opts.weight_key = 1      # any non-zero key: the edge list carries the weights
        _check(self.lib, self.ctx, self.lib.tgo_load_edges(self.ctx, C.byref(e), C.byref(opts)))
        self.n = self.lib.tgo_num_vertices(self.ctx)
        return self

    def load_csr(self, n, out_off, out_idx, in_off, in_idx, scope, out_w=None, in_w=None, titan_ids=None,
                 weight_key=0, column_order=False):
        """A caller-assembled adjacency (tgo_load_csr): row v's OUT entries out_idx[out_off[v]:
        out_off[v+1]] and IN entries in_idx[in_off[v]:in_off[v+1]] (dense neighbour indices), the
        rows as preloaded (no cap applied again)."""
        oo = np.ascontiguousarray(out_off, dtype=np.int64)
        io = np.ascontiguousarray(in_off, dtype=np.int64)
        oi = np.ascontiguousarray(out_idx, dtype=np.int32)
        ii = np.ascontiguousarray(in_idx, dtype=np.int32)
        ow = None if out_w is None else np.ascontiguousarray(out_w, dtype=np.int32)
        iw = None if in_w is None else np.ascontiguousarray(in_w, dtype=np.int32)
        t = None if titan_ids is None else np.ascontiguousarray(titan_ids, dtype=np.int64)
        if len(oo) != n + 1 or len(io) != n + 1:
            raise ValueError("offsets must hold n + 1 entries")
        opts, keep = self._opts(scope, False, (), weight_key, L.LOAD_COLUMN_ORDER if column_order else 0)
        if (ow is not None or iw is not None) and weight_key == 0:
            opts.weight_key = 1      # any non-zero key: the lists carry the weights
        rc = self.lib.tgo_load_csr(self.ctx, n, L.ptr(t, C.c_int64), L.ptr(oo, C.c_int64), L.ptr(oi, C.c_int32),
                                   L.ptr(ow, C.c_int32), L.ptr(io, C.c_int64), L.ptr(ii, C.c_int32),
                                   L.ptr(iw, C.c_int32), C.byref(opts))
        _check(self.lib, self.ctx, rc)
        self.n = self.lib.tgo_num_vertices(self.ctx)
        return self

    # ------------------------------------------------------------------ 1-D partition (multi-GPU)
    def load_partition(self, n_global, lo, hi, src, dst, scope, weight=None, apply_cap=True, layout=None):
        """Rows of global vertices [lo, hi) (titan_gpu_olap_part.h); `layout` = the
        all-gathered tgo_part_layout slices (n_global int32) or None for identity ids."""
        src = np.ascontiguousarray(src, dtype=np.int32)
        dst = np.ascontiguousarray(dst, dtype=np.int32)
        w = None if weight is None else np.ascontiguousarray(weight, dtype=np.int32)
        e = L.Edges(n_global, len(src), L.ptr(src, C.c_int32), L.ptr(dst, C.c_int32), L.ptr(w, C.c_int32), None)
        opts, keep = self._opts(scope, apply_cap, (), 1 if w is not None else 0)
        if layout is None:
            rc = self.lib.tgo_load_partition(self.ctx, n_global, lo, hi, C.byref(e), C.byref(opts))
        else:
            lay = np.ascontiguousarray(layout, dtype=np.int32)
            if len(lay) != n_global:
                raise ValueError("layout must hold n_global entries")
            rc = self.lib.tgo_load_partition_layout(self.ctx, n_global, lo, hi, C.byref(e), C.byref(opts),
                                                    L.ptr(lay, C.c_int32))
        _check(self.lib, self.ctx, rc)
        self.n = self.lib.tgo_num_vertices(self.ctx)
        return self

    def load_partition_rows(self, exchange, rows, schema: Schema, scope, apply_cap=True, labels=(), weight_key=0,
                            layout=True, batch_rows=None):
        """This rank's rows of a row-range partition of the scan (tgo_load_partition_rows; a
        collective over `exchange`, a distributed.NativeExchange): the one-GPU decode and cut per
        row, global slot ids.  Returns (live rows here, slot size S, live rows of every rank):
        n_global = world * S, lo = rank * S; results are the first `live` entries of the rank's
        outputs, whose ids are vertex_ids()[:live].  batch_rows: stage the rows in work blocks
        (tgo_load_rows each) and finish with tgo_finish_partition_rows, as a scan hands them over."""
        if batch_rows:
            opts, keep = self._opts(scope, apply_cap, labels, weight_key)
            rc = L.TGO_OK
            for r0 in range(0, rows.nrows, batch_rows):
                cr, hold = self._row_block(rows, r0, min(rows.nrows, r0 + batch_rows))
                rc = self.lib.tgo_load_rows(self.ctx, C.byref(cr), C.byref(schema.c), C.byref(opts))
                if rc != L.TGO_OK:
                    break
            if rc != L.TGO_OK:       # the ranks still meet in the collective load: an empty one
                msg = self.lib.tgo_last_error(self.ctx).decode(errors="replace")
                cr, hold = self._row_block(rows, 0, 0)
                part = np.zeros(3, np.int64)
                self.lib.tgo_load_partition_rows(self.ctx, exchange.h, C.byref(cr), C.byref(schema.c), None, 0,
                                                 L.ptr(part, C.c_int64))
                raise TitanException(rc, msg)
            return self.finish_partition_rows(exchange, layout)
        opts, keep = self._opts(scope, apply_cap, labels, weight_key)
        keys = np.ascontiguousarray(rows.keys, dtype=np.int64)
        eb = np.ascontiguousarray(rows.entry_begin, dtype=np.int64)
        bb = np.ascontiguousarray(rows.byte_begin, dtype=np.int64)
        data = np.ascontiguousarray(rows.data if len(rows.data) else np.zeros(1, np.uint8), dtype=np.uint8)
        lv = np.ascontiguousarray(rows.limit_valpos if len(rows.limit_valpos) else np.zeros(1, np.int64), dtype=np.int64)
        cr = L.Rows(rows.nrows, L.ptr(keys, C.c_int64), L.ptr(eb, C.c_int64), L.ptr(bb, C.c_int64),
                    L.ptr(data, C.c_uint8), L.ptr(lv, C.c_int64))
        part = np.zeros(3, np.int64)
        _check(self.lib, self.ctx, self.lib.tgo_load_partition_rows(self.ctx, exchange.h, C.byref(cr), C.byref(schema.c),
                                                                    C.byref(opts), 1 if layout else 0,
                                                                    L.ptr(part, C.c_int64)))
        self.n = self.lib.tgo_num_vertices(self.ctx)
        return int(part[0]), int(part[1]), int(part[2])

    def finish_partition_rows(self, exchange, layout=True):
        """The collective finish of a partition from staged rows (tgo_finish_partition_rows)."""
        part = np.zeros(3, np.int64)
        _check(self.lib, self.ctx, self.lib.tgo_finish_partition_rows(self.ctx, exchange.h, 1 if layout else 0,
                                                                      L.ptr(part, C.c_int64)))
        self.n = self.lib.tgo_num_vertices(self.ctx)
        return int(part[0]), int(part[1]), int(part[2])

    def part_call(self, name, *args):
        _check(self.lib, self.ctx, getattr(self.lib, name)(self.ctx, *args))

    def vertex_ids(self):
        out = np.zeros(self.n, dtype=np.int64)
        _check(self.lib, self.ctx, self.lib.tgo_vertex_ids(self.ctx, L.ptr(out, C.c_int64)))
        return out

    def graph_csr(self, which):
        """The assembled device lists (which: 0 OUT, 1 IN, 2 push transpose) in internal ids:
        dict(off, adj, w, col) with w / col None when the load has none; None if absent."""
        nnz = C.c_int64()
        _check(self.lib, self.ctx, self.lib.tgo_graph_csr(self.ctx, which, C.byref(nnz), None, None, None, None))
        if nnz.value < 0:
            return None
        off = np.zeros(self.n + 1, np.int64)
        adj = np.zeros(nnz.value, np.int32)
        w = np.full(nnz.value, -7, np.int32)
        col = np.full(nnz.value, 0xFFFFFFFF, np.uint32)
        _check(self.lib, self.ctx, self.lib.tgo_graph_csr(self.ctx, which, C.byref(nnz), L.ptr(off, C.c_int64),
                                                          L.ptr(adj, C.c_int32), L.ptr(w, C.c_int32),
                                                          L.ptr(col, C.c_uint32)))
        return {"off": off, "adj": adj, "w": w, "col": col}

    def graph_perm(self):
        out = np.zeros(self.n, np.int32)
        _check(self.lib, self.ctx, self.lib.tgo_graph_perm(self.ctx, L.ptr(out, C.c_int32)))
        return out

    # ------------------------------------------------------------------ programs
    def bfs(self, seed, max_depth, scope, seed_is_dense=False, stats=False, fetch=True):
        a = L.BfsArgs(int(seed), 1 if seed_is_dense else 0, int(max_depth), scope, L.FLAG_STATS if stats else 0)
        out = np.zeros(self.n, dtype=np.int64) if fetch else None
        _check(self.lib, self.ctx, self.lib.tgo_bfs(self.ctx, C.byref(a), L.ptr(out, C.c_int64)))
        return out

    def bfs_multi(self, seeds, max_depth, scope, seed_is_dense=False, stats=False, fetch=True):
        """Multi-source BFS (<= 64 seeds): returns a (nseeds, n) int64 array (or None)."""
        sd = np.ascontiguousarray(seeds, dtype=np.int64)
        a = L.BfsArgs(0, 1 if seed_is_dense else 0, int(max_depth), scope, L.FLAG_STATS if stats else 0)
        out = np.zeros((len(sd), self.n), dtype=np.int64) if fetch else None
        _check(self.lib, self.ctx, self.lib.tgo_bfs_multi(self.ctx, L.ptr(sd, C.c_int64), len(sd), C.byref(a),
                                                          L.ptr(out, C.c_int64)))
        return out

    def set_tuning(self, key, value):
        """tgo_set_tuning: a traversal policy of this ctx (L.TUNE_MS_SPLIT: the multi-source
        source-split budget; < 0 restores the default).  Never changes a result."""
        _check(self.lib, self.ctx, self.lib.tgo_set_tuning(self.ctx, int(key), float(value)))
        return self

    def multi_stats(self, nseeds):
        r = np.zeros(nseeds, np.int64)
        e = np.zeros(nseeds, np.int64)
        _check(self.lib, self.ctx, self.lib.tgo_multi_stats(self.ctx, L.ptr(r, C.c_int64), L.ptr(e, C.c_int64)))
        return r, e

    def sssp(self, seed, max_depth, scope, mode=L.SSSP_HOP_BOUNDED, seed_is_dense=False, stats=False, fetch=True,
             delta=0):
        """ShortestDistanceVertexProgram.  HOP_BOUNDED: the reference's Jacobi supersteps
        0..max_depth exactly; DELTA: delta-stepping to the converged distances (bucket width
        `delta`, 0 = a quarter of the mean weight)."""
        a = L.SsspArgs(int(seed), 1 if seed_is_dense else 0, int(max_depth), scope, mode, int(delta),
                       L.FLAG_STATS if stats else 0, 0)
        out = np.zeros(self.n, dtype=np.int64) if fetch else None
        _check(self.lib, self.ctx, self.lib.tgo_sssp(self.ctx, C.byref(a), L.ptr(out, C.c_int64)))
        return out

    def pagerank(self, alpha, vertex_count, max_iterations, fetch=True):
        a = L.PrArgs(alpha, int(vertex_count), int(max_iterations), 0)
        out = np.zeros(self.n, dtype=np.float64) if fetch else None
        _check(self.lib, self.ctx, self.lib.tgo_pagerank(self.ctx, C.byref(a), L.ptr(out, C.c_double)))
        return out

    def walkcount(self, k, fetch=True):
        out = np.zeros(self.n, dtype=np.int32) if fetch else None
        _check(self.lib, self.ctx, self.lib.tgo_walkcount(self.ctx, int(k), L.ptr(out, C.c_int32)))
        return out

    def result_rows(self, kind, key_ids, datatypes, relation_id_base):
        """Edgestore entries of the last program's compute keys (tgo_result_rows): the rows
        ResultMode PERSIST writes back (FulgoraGraphComputer.java:248-305)."""
        k = list(key_ids) + [0] * (2 - len(key_ids))
        d = list(datatypes) + [0] * (2 - len(datatypes))
        a = L.ResultArgs(kind, 0, (C.c_int64 * 2)(*k), (C.c_int32 * 2)(*d), int(relation_id_base))
        sz = L.ResultSize()
        _check(self.lib, self.ctx, self.lib.tgo_result_rows(self.ctx, C.byref(a), C.byref(sz), None))
        keys = np.empty(max(sz.nrows, 1), np.int64)
        eb = np.empty(sz.nrows + 1, np.int64)
        bb = np.empty(sz.nrows + 1, np.int64)
        data = np.empty(max(sz.nbytes, 1), np.uint8)
        lv = np.empty(max(sz.nentries, 1), np.int64)
        buf = L.RowsBuf(L.ptr(keys, C.c_int64), L.ptr(eb, C.c_int64), L.ptr(bb, C.c_int64), L.ptr(data, C.c_uint8),
                        L.ptr(lv, C.c_int64))
        _check(self.lib, self.ctx, self.lib.tgo_result_rows(self.ctx, C.byref(a), C.byref(sz), C.byref(buf)))
        return Rows(keys[:sz.nrows], eb, bb, data[:sz.nbytes], lv[:sz.nentries])

    # ------------------------------------------------------------------ generic vertex programs
    @staticmethod
    def _vals(values, value_type):
        return np.ascontiguousarray(values, dtype=np.int64 if value_type == L.VAL_INT64 else np.float64)

    def gather(self, scope, value_type, combiner, edge_fn, msg, has=None):
        """MessageScope.Local receive with a combiner (tgo_gather): returns (combined values,
        has-message mask) per vertex in row order."""
        m = self._vals(msg, value_type)
        h = None if has is None else np.ascontiguousarray(has, dtype=np.uint8)
        out = np.empty(self.n, dtype=m.dtype)
        out_has = np.empty(self.n, dtype=np.uint8)
        a = L.GatherArgs(scope, value_type, combiner, edge_fn)
        _check(self.lib, self.ctx, self.lib.tgo_gather(self.ctx, C.byref(a), m.ctypes.data_as(C.c_void_p),
                                                       L.ptr(h, C.c_uint8), out.ctypes.data_as(C.c_void_p),
                                                       L.ptr(out_has, C.c_uint8)))
        return out, out_has.astype(bool)

    def set_edge_program(self, ops, iconsts=None, fconsts=None):
        """tgo_set_edge_program: the postfix program TGO_EDGE_PROGRAM gathers evaluate (None clears
        it).  ops: tgo_edge_op | const index << 8; iconsts / fconsts: the constants as Java long /
        double (None: the program does not run on that message type)."""
        if ops is None:
            _check(self.lib, self.ctx, self.lib.tgo_set_edge_program(self.ctx, None))
            return
        o = np.ascontiguousarray(ops, dtype=np.int32)
        ic = None if iconsts is None else np.ascontiguousarray(iconsts, dtype=np.int64)
        fc = None if fconsts is None else np.ascontiguousarray(fconsts, dtype=np.float64)
        nc = len(ic) if ic is not None else (len(fc) if fc is not None else 0)
        p = L.EdgeProgram(len(o), L.ptr(o, C.c_int32), nc, L.ptr(ic, C.c_int64), L.ptr(fc, C.c_double))
        _check(self.lib, self.ctx, self.lib.tgo_set_edge_program(self.ctx, C.byref(p)))

    def gather_lists(self, scope, value_type, edge_fn, msg, has=None):
        """MessageScope.Local receive WITHOUT a combiner (tgo_gather_lists): every vertex's
        message stream as (row offsets n+1, values) in the API's row order."""
        m = self._vals(msg, value_type)
        h = None if has is None else np.ascontiguousarray(has, dtype=np.uint8)
        off = np.zeros(self.n + 1, dtype=np.int64)
        a = L.GatherArgs(scope, value_type, 0, edge_fn)
        _check(self.lib, self.ctx, self.lib.tgo_gather_lists(self.ctx, C.byref(a), m.ctypes.data_as(C.c_void_p),
                                                             L.ptr(h, C.c_uint8), L.ptr(off, C.c_int64), None))
        vals = np.zeros(max(int(off[-1]), 1), dtype=m.dtype)
        if off[-1] > 0:
            _check(self.lib, self.ctx, self.lib.tgo_gather_lists(self.ctx, C.byref(a), m.ctypes.data_as(C.c_void_p),
                                                                 L.ptr(h, C.c_uint8), L.ptr(off, C.c_int64),
                                                                 vals.ctypes.data_as(C.c_void_p)))
        return off, vals[:int(off[-1])]

    def result_rows_values(self, key_id, datatype, value_type, values, present, relation_id_base):
        """Edgestore entries of a generic program's compute key (tgo_result_rows_values)."""
        v = self._vals(values, value_type)
        p = np.ascontiguousarray(present, dtype=np.uint8)
        a = L.ResultArgs(L.RESULT_VALUES, int(value_type), (C.c_int64 * 2)(int(key_id), 0), (C.c_int32 * 2)(int(datatype), 0),
                         int(relation_id_base))
        sz = L.ResultSize()
        vp = v.ctypes.data_as(C.c_void_p)
        _check(self.lib, self.ctx, self.lib.tgo_result_rows_values(self.ctx, C.byref(a), vp, L.ptr(p, C.c_uint8),
                                                                   C.byref(sz), None))
        keys = np.empty(max(sz.nrows, 1), np.int64)
        eb = np.empty(sz.nrows + 1, np.int64)
        bb = np.empty(sz.nrows + 1, np.int64)
        data = np.empty(max(sz.nbytes, 1), np.uint8)
        lv = np.empty(max(sz.nentries, 1), np.int64)
        buf = L.RowsBuf(L.ptr(keys, C.c_int64), L.ptr(eb, C.c_int64), L.ptr(bb, C.c_int64), L.ptr(data, C.c_uint8),
                        L.ptr(lv, C.c_int64))
        _check(self.lib, self.ctx, self.lib.tgo_result_rows_values(self.ctx, C.byref(a), vp, L.ptr(p, C.c_uint8),
                                                                   C.byref(sz), C.byref(buf)))
        return Rows(keys[:sz.nrows], eb, bb, data[:sz.nbytes], lv[:sz.nentries])

    def combine_global(self, value_type, combiner, targets, values):
        """MessageScope.Global: messages to dense row ids combined per target in send order."""
        t = np.ascontiguousarray(targets, dtype=np.int64)
        v = self._vals(values, value_type)
        out = np.empty(self.n, dtype=v.dtype)
        out_has = np.empty(self.n, dtype=np.uint8)
        _check(self.lib, self.ctx, self.lib.tgo_combine_global(self.ctx, value_type, combiner, len(t), L.ptr(t, C.c_int64),
                                                               v.ctypes.data_as(C.c_void_p),
                                                               out.ctypes.data_as(C.c_void_p), L.ptr(out_has, C.c_uint8)))
        return out, out_has.astype(bool)

    def dense_ids(self, titan_ids):
        ids = np.ascontiguousarray(titan_ids, dtype=np.int64)
        out = np.empty(len(ids), dtype=np.int64)
        _check(self.lib, self.ctx, self.lib.tgo_dense_ids(self.ctx, L.ptr(ids, C.c_int64), len(ids), L.ptr(out, C.c_int64)))
        return out

    def stats(self):
        s = L.Stats()
        _check(self.lib, self.ctx, self.lib.tgo_stats_get(self.ctx, C.byref(s)))
        return {f: getattr(s, f) for f, _ in L.Stats._fields_}

    def sync(self):
        _check(self.lib, self.ctx, self.lib.tgo_sync(self.ctx))


def rmat_edges(scale, edge_factor=16, seed=0x54495441, weights=False, threads=0, device=None):
    """Synthetic RMAT edge list (include/tgo_synth.h); device=k generates the same stream on
    GPU k (tgo_rmat_edges_device)."""
    lib = L.load()
    m = edge_factor << scale
    src = np.empty(m, dtype=np.int32)
    dst = np.empty(m, dtype=np.int32)
    w = np.empty(m, dtype=np.int32) if weights else None
    if device is not None:
        rc = lib.tgo_rmat_edges_device(scale, edge_factor, seed, 0, m, L.ptr(src, C.c_int32), L.ptr(dst, C.c_int32),
                                       L.ptr(w, C.c_int32), int(device))
    else:
        rc = lib.tgo_rmat_edges(scale, edge_factor, seed, 0, m, L.ptr(src, C.c_int32), L.ptr(dst, C.c_int32),
                                L.ptr(w, C.c_int32), threads)
    if rc:
        raise TitanException(rc, "tgo_rmat_edges failed")
    return src, dst, w


class Rows:
    """Scanned edgestore rows in the tgo_rows layout (StaticArrayEntryList per row)."""

    def __init__(self, keys, entry_begin, byte_begin, data, limit_valpos):
        self.keys, self.entry_begin, self.byte_begin = keys, entry_begin, byte_begin
        self.data, self.limit_valpos = data, limit_valpos

    @property
    def nrows(self):
        return len(self.keys)


USER_EDGE_LABEL_1 = (1 << 6) | 21     # IDManager.getSchemaId(UserEdgeLabel, 1)


def synth_rows(n, src, dst, weight=None, label_id=USER_EDGE_LABEL_1, partition_bits=5, threads=0):
    """Byte-exact edgestore rows of a directed edge list (include/tgo_synth.h)."""
    lib = L.load()
    src = np.ascontiguousarray(src, dtype=np.int32)
    dst = np.ascontiguousarray(dst, dtype=np.int32)
    w = None if weight is None else np.ascontiguousarray(weight, dtype=np.int32)
    sz = np.zeros(3, np.int64)
    args = (n, len(src), L.ptr(src, C.c_int32), L.ptr(dst, C.c_int32), L.ptr(w, C.c_int32), label_id,
            partition_bits, threads, L.ptr(sz, C.c_int64))
    rc = lib.tgo_synth_rows(*args, None, None, None, None, None)
    if rc:
        raise TitanException(rc, "tgo_synth_rows failed")
    nrows, nent, nbytes = (int(x) for x in sz)
    keys = np.empty(nrows, np.int64)
    eb = np.empty(nrows + 1, np.int64)
    bb = np.empty(nrows + 1, np.int64)
    data = np.empty(max(nbytes, 1), np.uint8)
    lv = np.empty(max(nent, 1), np.int64)
    rc = lib.tgo_synth_rows(*args, L.ptr(keys, C.c_int64), L.ptr(eb, C.c_int64), L.ptr(bb, C.c_int64),
                            L.ptr(data, C.c_uint8), L.ptr(lv, C.c_int64))
    if rc:
        raise TitanException(rc, "tgo_synth_rows failed")
    return Rows(keys, eb, bb, data[:nbytes], lv[:nent])


def pick_roots(n, src, dst, nroots=64, seed=7):
    lib = L.load()
    out = np.zeros(nroots, dtype=np.int64)
    rc = lib.tgo_pick_roots(n, len(src), L.ptr(src, C.c_int32), L.ptr(dst, C.c_int32), seed, nroots,
                            L.ptr(out, C.c_int64))
    if rc:
        raise TitanException(rc, "tgo_pick_roots failed")
    return out

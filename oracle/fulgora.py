"""ctypes binding of the CPU oracle (oracle/libfulgora_ref.so).

TEST INFRASTRUCTURE ONLY: imported by tests/, __graft_entry__.smoke() and bench.py's
cpu_baseline leg, always as the checker / the timed CPU baseline, never as the product.
"""
from __future__ import annotations

import ctypes as C
import os
import subprocess

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(_HERE, "libfulgora_ref.so")

FR_ABSENT = -(1 << 63)
_i64p = C.POINTER(C.c_int64)
_i32p = C.POINTER(C.c_int32)
_u8p = C.POINTER(C.c_uint8)


class FrBuf(C.Structure):
    _fields_ = [("p", _u8p), ("len", C.c_size_t), ("cap", C.c_size_t)]


class FrRows(C.Structure):
    _fields_ = [("nrows", C.c_int64), ("row_keys", _i64p), ("row_entry_begin", _i64p),
                ("row_byte_begin", _i64p), ("entry_bytes", _u8p), ("entry_limit_valpos", _i64p)]


class FrEdgeType(C.Structure):
    _fields_ = [("type_id", C.c_int64), ("multiplicity", C.c_int32), ("n_sort_key", C.c_int32),
                ("sort_key_ids", _i64p), ("n_signature", C.c_int32), ("sort_order", C.c_int32),
                ("signature_ids", _i64p)]


class FrPropertyKey(C.Structure):
    _fields_ = [("key_id", C.c_int64), ("datatype", C.c_int32)]


class FrSchema(C.Structure):
    _fields_ = [("n_edge_types", C.c_int32), ("edge_types", C.POINTER(FrEdgeType)),
                ("n_property_keys", C.c_int32), ("property_keys", C.POINTER(FrPropertyKey))]


class FrProp(C.Structure):
    _fields_ = [("key_id", C.c_int64), ("value", C.c_int64)]


class FrLoadOpts(C.Structure):
    _fields_ = [("scope", C.c_int32), ("apply_cap", C.c_int32), ("hard_query_limit", C.c_int64),
                ("n_labels", C.c_int32), ("label_ids", _i64p), ("weight_key", C.c_int64),
                ("partition_bits", C.c_int32)]


class FrLoadStats(C.Structure):
    _fields_ = [("ghost_vertices", C.c_int64), ("truncated_results", C.c_int64),
                ("skipped_rows", C.c_int64), ("num_entries", C.c_int64),
                ("partitioned_vertices", C.c_int64), ("partition_rows", C.c_int64),
                ("ghost_partition_rows", C.c_int64)]


_lib = None


def build() -> None:
    subprocess.run(["make", "-s", "-C", _HERE], check=True)


def load() -> C.CDLL:
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(LIB_PATH):
        build()
    lib = C.CDLL(LIB_PATH)
    P = C.POINTER
    vp = C.c_void_p
    sig = {
        "fr_buf_free": (None, [P(FrBuf)]),
        "fr_vl_write_positive": (None, [P(FrBuf), C.c_int64]),
        "fr_vl_read_positive": (C.c_int64, [_u8p, P(C.c_size_t)]),
        "fr_vl_write": (None, [P(FrBuf), C.c_int64]),
        "fr_vl_read": (C.c_int64, [_u8p, P(C.c_size_t)]),
        "fr_vl_write_positive_with_prefix": (None, [P(FrBuf), C.c_int64, C.c_int64, C.c_int]),
        "fr_vl_read_positive_with_prefix": (None, [_u8p, P(C.c_size_t), C.c_int, _i64p, _i64p]),
        "fr_vl_write_positive_backward": (None, [P(FrBuf), C.c_int64]),
        "fr_vl_read_positive_backward": (C.c_int64, [_u8p, P(C.c_size_t)]),
        "fr_vl_positive_length": (C.c_int, [C.c_int64]),
        "fr_vl_backward_length": (C.c_int, [C.c_int64]),
        "fr_schema_id": (C.c_int64, [C.c_int, C.c_int64]),
        "fr_vertex_id": (C.c_int64, [C.c_int64, C.c_int64, C.c_int]),
        "fr_key_of": (C.c_int64, [C.c_int64, C.c_int]),
        "fr_key_id": (C.c_int64, [C.c_int64, C.c_int]),
        "fr_is_invisible": (C.c_int, [C.c_int64]),
        "fr_partitioned_vertex_id": (C.c_int64, [C.c_int64, C.c_int64, C.c_int]),
        "fr_is_partitioned": (C.c_int, [C.c_int64, C.c_int]),
        "fr_canonical_vertex_id": (C.c_int64, [C.c_int64, C.c_int]),
        "fr_write_relation_type": (None, [P(FrBuf), C.c_int64, C.c_int, C.c_int, C.c_int]),
        "fr_read_relation_type": (C.c_int, [_u8p, P(C.c_size_t), _i64p, P(C.c_int), P(C.c_int)]),
        "fr_encode_edge": (C.c_int, [P(FrBuf), _i32p, P(FrSchema), C.c_int64, C.c_int, C.c_int64,
                                     C.c_int64, P(FrProp), C.c_int]),
        "fr_encode_vertex_exists": (C.c_int, [P(FrBuf), _i32p, C.c_int64]),
        "fr_write_value": (C.c_int, [P(FrBuf), C.c_int, C.c_int, C.c_int64, C.c_int]),
        "fr_encode_property_f64": (C.c_int, [P(FrBuf), _i32p, C.c_int64, C.c_double, C.c_int64]),
        "fr_string_of": (C.c_int, [C.c_int64, P(C.c_uint16)]),
        "fr_encode_property": (C.c_int, [P(FrBuf), _i32p, C.c_int64, C.c_int, C.c_int64, C.c_int64]),
        "fr_encode_property_generic": (C.c_int, [P(FrBuf), _i32p, C.c_int64, C.c_int, C.c_int64, C.c_int64]),
        "fr_decode_edge": (C.c_int, [_u8p, C.c_size_t, C.c_size_t, P(FrSchema), C.c_int64, _i64p,
                                     P(C.c_int), _i64p, _i64p, P(C.c_int), _i64p]),
        "fr_load_rows": (C.c_int, [P(FrRows), P(FrSchema), P(FrLoadOpts), P(vp), P(FrLoadStats)]),
        "fr_load_adjacency": (C.c_int, [C.c_int64, _i64p, _i64p, _i64p, _i32p, _i32p, P(vp)]),
        "fr_load_edges": (C.c_int, [C.c_int64, C.c_int64, _i32p, _i32p, _i32p, _i64p, P(vp)]),
        "fr_load_edges_capped": (C.c_int, [C.c_int64, C.c_int64, _i32p, _i32p, _i32p, _i64p, C.c_int64, _i64p,
                                           P(vp)]),
        "fr_resolve": (C.c_int, [vp, C.c_int]),
        "fr_free": (None, [vp]),
        "fr_num_vertices": (C.c_int64, [vp]),
        "fr_vertex_ids": (None, [vp, _i64p]),
        "fr_num_entries": (C.c_int64, [vp]),
        "fr_export": (C.c_int64, [vp, _i64p, _i64p, _i32p, _i32p]),
        "fr_shortest_distance": (C.c_int, [vp, C.c_int64, C.c_int, C.c_int, C.c_int, C.c_int, _i64p, P(C.c_int)]),
        "fr_pagerank": (C.c_int, [vp, C.c_double, C.c_int64, C.c_int, C.c_int, C.POINTER(C.c_double), P(C.c_int)]),
        "fr_degree_counter": (C.c_int, [vp, C.c_int, C.c_int, _i32p, P(C.c_int)]),
        "fr_gather": (C.c_int, [vp, C.c_int, C.c_int, C.c_int, C.c_int, vp, _u8p, vp, _u8p]),
        "fr_set_edge_program": (C.c_int, [_i32p, C.c_int, _i64p, C.POINTER(C.c_double), C.c_int]),
        "fr_gather_lists": (C.c_int, [vp, C.c_int, C.c_int, C.c_int, vp, _u8p, _i64p, vp]),
        "fr_combine_global": (C.c_int, [C.c_int64, C.c_int, C.c_int, C.c_int64, _i64p, vp, vp, _u8p]),
    }
    for name, (res, args) in sig.items():
        f = getattr(lib, name)
        f.restype = res
        f.argtypes = args
    _lib = lib
    return lib


def _p(arr, t):
    return None if arr is None else arr.ctypes.data_as(C.POINTER(t))


# ----------------------------------------------------------------------------- codec helpers
def buf_bytes(fn, *args) -> bytes:
    lib = load()
    b = FrBuf()
    getattr(lib, fn)(C.byref(b), *args)
    out = C.string_at(b.p, b.len) if b.len else b""
    lib.fr_buf_free(C.byref(b))
    return out


class OracleSchema:
    """Holds ctypes arrays alive for an FrSchema built from a python schema description."""

    def __init__(self, edge_types, property_keys):
        # edge_types: list of dicts {type_id, multiplicity, sort_key:[ids], signature:[ids],
        # order: "ASC" | "DESC"}
        self._keep = []
        et = (FrEdgeType * max(1, len(edge_types)))()
        for i, t in enumerate(edge_types):
            sk = np.asarray(t.get("sort_key", []), dtype=np.int64)
            sg = np.asarray(t.get("signature", []), dtype=np.int64)
            self._keep += [sk, sg]
            et[i] = FrEdgeType(t["type_id"], t["multiplicity"], len(sk), _p(sk, C.c_int64), len(sg),
                               1 if t.get("order", "ASC") == "DESC" else 0, _p(sg, C.c_int64))
        pk = (FrPropertyKey * max(1, len(property_keys)))()
        for i, (kid, dt) in enumerate(property_keys):
            pk[i] = FrPropertyKey(kid, dt)
        self._keep += [et, pk]
        self.s = FrSchema(len(edge_types), et, len(property_keys), pk)


def encode_edge(schema: OracleSchema, type_id, direction, other, relation_id, props=()):
    lib = load()
    b = FrBuf()
    vp = C.c_int32(0)
    arr = (FrProp * max(1, len(props)))(*[FrProp(k, v) for k, v in props])
    rc = lib.fr_encode_edge(C.byref(b), C.byref(vp), C.byref(schema.s), type_id, direction, other,
                            relation_id, arr, len(props))
    if rc:
        raise ValueError(f"fr_encode_edge rc={rc}")
    out = C.string_at(b.p, b.len)
    lib.fr_buf_free(C.byref(b))
    return out, vp.value


def encode_property(key_id, datatype, value, relation_id):
    lib = load()
    b = FrBuf()
    vp = C.c_int32(0)
    rc = lib.fr_encode_property(C.byref(b), C.byref(vp), key_id, datatype, value, relation_id)
    if rc:
        raise ValueError(f"fr_encode_property rc={rc}")
    out = C.string_at(b.p, b.len)
    lib.fr_buf_free(C.byref(b))
    return out, vp.value


def encode_property_generic(key_id, value_dt, value, relation_id):
    """A generic (Object) key's entry; value_dt = the value's class (DT_INTEGER / LONG / DOUBLE)."""
    import struct
    lib = load()
    b = FrBuf()
    vp = C.c_int32(0)
    if value_dt == 6:
        value = struct.unpack("<q", struct.pack("<d", float(value)))[0]
    rc = lib.fr_encode_property_generic(C.byref(b), C.byref(vp), key_id, value_dt, int(value), relation_id)
    if rc:
        raise ValueError(f"fr_encode_property_generic rc={rc}")
    out = C.string_at(b.p, b.len)
    lib.fr_buf_free(C.byref(b))
    return out, vp.value


def encode_property_f64(key_id, value, relation_id):
    lib = load()
    b = FrBuf()
    vp = C.c_int32(0)
    lib.fr_encode_property_f64(C.byref(b), C.byref(vp), key_id, float(value), relation_id)
    out = C.string_at(b.p, b.len)
    lib.fr_buf_free(C.byref(b))
    return out, vp.value


def encode_vertex_exists(relation_id):
    lib = load()
    b = FrBuf()
    vp = C.c_int32(0)
    lib.fr_encode_vertex_exists(C.byref(b), C.byref(vp), relation_id)
    out = C.string_at(b.p, b.len)
    lib.fr_buf_free(C.byref(b))
    return out, vp.value


def set_edge_program(ops, iconsts=None, fconsts=None):
    """fr_set_edge_program: the postfix edge-function program edge_fn 8 evaluates."""
    o = np.ascontiguousarray(ops, np.int32)
    nc = len(iconsts if iconsts is not None else (fconsts if fconsts is not None else []))
    ic = None if iconsts is None else np.ascontiguousarray(iconsts, np.int64)
    fc = None if fconsts is None else np.ascontiguousarray(fconsts, np.float64)
    rc = load().fr_set_edge_program(_p(o, C.c_int32), len(o), _p(ic, C.c_int64), _p(fc, C.c_double), nc)
    if rc:
        raise RuntimeError(f"fr_set_edge_program rc={rc}")


def combine_global(n, value_type, combiner, targets, values):
    """Global-scope messages folded per target in send order (fr_combine_global)."""
    dt = np.int64 if value_type == 0 else np.float64
    t = np.ascontiguousarray(targets, np.int64)
    v = np.ascontiguousarray(values, dt)
    out = np.zeros(n, dt)
    oh = np.zeros(n, np.uint8)
    load().fr_combine_global(n, value_type, combiner, len(t), _p(t, C.c_int64), v.ctypes.data_as(C.c_void_p),
                             out.ctypes.data_as(C.c_void_p), _p(oh, C.c_uint8))
    return out, oh.astype(bool)


# ----------------------------------------------------------------------------- graph
class OracleGraph:
    def __init__(self, handle, stats=None):
        self.h = handle
        self.stats = stats

    @classmethod
    def from_rows(cls, rows, schema: OracleSchema, scope, apply_cap=1, hard_limit=100000,
                  labels=(), weight_key=0, partition_bits=5):
        lib = load()
        lab = np.asarray(labels, dtype=np.int64)
        fr = FrRows(rows.nrows, _p(rows.keys, C.c_int64), _p(rows.entry_begin, C.c_int64),
                    _p(rows.byte_begin, C.c_int64), _p(rows.data, C.c_uint8), _p(rows.limit_valpos, C.c_int64))
        opts = FrLoadOpts(scope, apply_cap, hard_limit, len(lab), _p(lab, C.c_int64) if len(lab) else None,
                          weight_key, partition_bits)
        h = C.c_void_p()
        st = FrLoadStats()
        rc = lib.fr_load_rows(C.byref(fr), C.byref(schema.s), C.byref(opts), C.byref(h), C.byref(st))
        if rc:
            raise RuntimeError(f"fr_load_rows rc={rc}")
        return cls(h, st)

    @classmethod
    def from_adjacency(cls, titan_ids, off, mid, adj, w=None):
        lib = load()
        h = C.c_void_p()
        rc = lib.fr_load_adjacency(len(titan_ids), _p(titan_ids, C.c_int64), _p(off, C.c_int64), _p(mid, C.c_int64),
                                   _p(adj, C.c_int32), _p(w, C.c_int32), C.byref(h))
        if rc:
            raise RuntimeError(f"fr_load_adjacency rc={rc}")
        return cls(h)

    @classmethod
    def from_edges(cls, n, src, dst, w=None, titan_ids=None, hard_limit=0):
        """Rows of a directed edge list (one MULTI label).  hard_limit > 0 applies the preload
        cap of an untyped inE/outE scope; stats.truncated_results counts the cut rows."""
        lib = load()
        src = np.ascontiguousarray(src, np.int32)
        dst = np.ascontiguousarray(dst, np.int32)
        w = None if w is None else np.ascontiguousarray(w, np.int32)
        ids = (np.arange(n, dtype=np.int64) + 1) << 3 if titan_ids is None else np.ascontiguousarray(titan_ids, np.int64)
        h = C.c_void_p()
        cut = C.c_int64(0)
        rc = lib.fr_load_edges_capped(n, len(src), _p(src, C.c_int32), _p(dst, C.c_int32), _p(w, C.c_int32),
                                      _p(ids, C.c_int64), int(hard_limit), C.byref(cut), C.byref(h))
        if rc:
            raise RuntimeError(f"fr_load_edges rc={rc}")
        st = FrLoadStats()
        st.truncated_results = cut.value
        return cls(h, st)

    def resolve(self, threads=16):
        """Memoise the per-entry hash lookups (faster supersteps, identical results)."""
        rc = load().fr_resolve(self.h, int(threads))
        if rc:
            raise RuntimeError(f"fr_resolve rc={rc}")
        return self

    def __del__(self):
        if getattr(self, "h", None) and _lib is not None:
            _lib.fr_free(self.h)
            self.h = None

    @property
    def n(self):
        return load().fr_num_vertices(self.h)

    def vertex_ids(self):
        out = np.zeros(self.n, dtype=np.int64)
        load().fr_vertex_ids(self.h, _p(out, C.c_int64))
        return out

    def export(self, weighted=False):
        lib = load()
        n = self.n
        E = lib.fr_num_entries(self.h)
        off = np.zeros(n + 1, np.int64)
        mid = np.zeros(max(n, 1), np.int64)
        adj = np.zeros(max(E, 1), np.int32)
        w = np.zeros(max(E, 1), np.int32) if weighted else None
        e = lib.fr_export(self.h, _p(off, C.c_int64), _p(mid, C.c_int64), _p(adj, C.c_int32), _p(w, C.c_int32))
        return off, mid[:n], adj[:e], (w[:e] if weighted else None)

    def shortest_distance(self, seed, max_depth, scope, weighted=False, threads=1):
        out = np.zeros(self.n, dtype=np.int64)
        it = C.c_int(0)
        rc = load().fr_shortest_distance(self.h, seed, max_depth, scope, 1 if weighted else 0, threads,
                                         _p(out, C.c_int64), C.byref(it))
        if rc:
            raise RuntimeError(f"fr_shortest_distance rc={rc}")
        return out, it.value

    def pagerank(self, alpha, vertex_count, max_iterations, threads=1):
        out = np.zeros(self.n, dtype=np.float64)
        it = C.c_int(0)
        rc = load().fr_pagerank(self.h, alpha, vertex_count, max_iterations, threads,
                                _p(out, C.c_double), C.byref(it))
        if rc:
            raise RuntimeError(f"fr_pagerank rc={rc}")
        return out, it.value

    def gather(self, scope, value_type, combiner, edge_fn, msg, has):
        """Local-scope receive folded with the combiner (fr_gather); vectors in vertex order."""
        dt = np.int64 if value_type == 0 else np.float64
        m = np.ascontiguousarray(msg, dt)
        h = np.ascontiguousarray(has, np.uint8)
        out = np.zeros(self.n, dt)
        oh = np.zeros(self.n, np.uint8)
        rc = load().fr_gather(self.h, scope, value_type, combiner, edge_fn, m.ctypes.data_as(C.c_void_p), _p(h, C.c_uint8),
                              out.ctypes.data_as(C.c_void_p), _p(oh, C.c_uint8))
        if rc:
            raise RuntimeError(f"fr_gather rc={rc}")
        return out, oh.astype(bool)

    def gather_lists(self, scope, value_type, edge_fn, msg, has):
        """Local-scope receive without a combiner (fr_gather_lists): (offsets n+1, values), every
        vertex's messages in its row's column order."""
        dt = np.int64 if value_type == 0 else np.float64
        m = np.ascontiguousarray(msg, dt)
        h = np.ascontiguousarray(has, np.uint8)
        off = np.zeros(self.n + 1, np.int64)
        lib = load()
        rc = lib.fr_gather_lists(self.h, scope, value_type, edge_fn, m.ctypes.data_as(C.c_void_p), _p(h, C.c_uint8),
                                 _p(off, C.c_int64), None)
        if rc:
            raise RuntimeError(f"fr_gather_lists rc={rc}")
        vals = np.zeros(max(int(off[-1]), 1), dt)
        rc = lib.fr_gather_lists(self.h, scope, value_type, edge_fn, m.ctypes.data_as(C.c_void_p), _p(h, C.c_uint8),
                                 _p(off, C.c_int64), vals.ctypes.data_as(C.c_void_p))
        if rc:
            raise RuntimeError(f"fr_gather_lists rc={rc}")
        return off, vals[:int(off[-1])]

    def degree_counter(self, length, threads=1):
        out = np.zeros(self.n, dtype=np.int32)
        it = C.c_int(0)
        rc = load().fr_degree_counter(self.h, length, threads, _p(out, C.c_int32), C.byref(it))
        if rc:
            raise RuntimeError(f"fr_degree_counter rc={rc}")
        return out, it.value

"""ctypes binding of the C-ABI in include/titan_gpu_olap.h (libtitan_gpu_olap.so).

The library is built in-tree (titan_amd/libtitan_gpu_olap.so, see titan_amd/csrc/Makefile)
and is the only compute path: there is no CPU fallback.  Loading fails loudly when the
shared object is missing.
"""
from __future__ import annotations

import ctypes as C
import os

_HERE = os.path.dirname(os.path.abspath(__file__))
# TGO_LIB_PATH: a probe build of the same sources (e.g. another tile size, scripts/gpu_ktile.sh)
LIB_PATH = os.environ.get("TGO_LIB_PATH") or os.path.join(_HERE, "libtitan_gpu_olap.so")

# status codes (tgo_status)
TGO_OK = 0
TGO_E_INVALID = -1
TGO_E_HIP = -2
TGO_E_OOM = -3
TGO_E_CODEC = -4
TGO_E_STATE = -5
TGO_E_PROGRAM = -6
TGO_E_UNSUPPORTED = -7
TGO_E_COMM = -8

SCOPE_OUT_E, SCOPE_IN_E, SCOPE_BOTH_E = 0, 1, 2
MULTI, SIMPLE, MANY2ONE, ONE2MANY, ONE2ONE = 0, 1, 2, 3, 4
DT_BYTE, DT_SHORT, DT_INTEGER, DT_LONG, DT_FLOAT, DT_DOUBLE, DT_BOOLEAN = 1, 2, 3, 4, 5, 6, 7
DT_OBJECT = 11      # generic key (DefaultSchemaMaker: dataType(Object.class)); result write-back only
DT_DATE, DT_CHARACTER, DT_STRING = 8, 9, 10
ORDER_ASC, ORDER_DESC = 0, 1
RESULT_DISTANCE, RESULT_PAGERANK, RESULT_DEGREE, RESULT_VALUES = 0, 1, 2, 3
SSSP_HOP_BOUNDED, SSSP_DELTA = 0, 1
FLAG_STATS = 1
TUNE_MS_SPLIT, TUNE_MS_GHOST, TUNE_DS_BINS, TUNE_DS_PILE_CAP, TUNE_DS_DONE, TUNE_MS_COLD, TUNE_DS_PULL = 1, 2, 3, 4, 5, 6, 7   # tgo_set_tuning keys
TUNE_DS_SMALL = 8
TRACE_JSON, TRACE_ROCTX = 1, 2   # tgo_trace_enable flags
DIST_ABSENT = -(1 << 63)
ABI_VERSION = 2
COMBINE_SUM, COMBINE_MIN, COMBINE_MAX = 0, 1, 2
VAL_INT64, VAL_FP64 = 0, 1
EDGE_IDENTITY, EDGE_ADD_ONE, EDGE_ADD_WEIGHT, EDGE_MUL_WEIGHT = 0, 1, 2, 3
EDGE_SUB_WEIGHT, EDGE_MIN_WEIGHT, EDGE_MAX_WEIGHT, EDGE_DIV_WEIGHT = 4, 5, 6, 7
EDGE_PROGRAM = 8
# tgo_edge_op (edge-function programs, titan_amd/generic.py EdgeExpr)
OP_MSG, OP_WEIGHT, OP_CONST, OP_ADD, OP_SUB, OP_MUL, OP_DIV, OP_REM, OP_MIN, OP_MAX, OP_NEG, OP_ABS = range(12)
EDGE_PROGRAM_MAX_OPS, EDGE_PROGRAM_MAX_CONSTS, EDGE_PROGRAM_MAX_STACK = 32, 16, 8

_i64p = C.POINTER(C.c_int64)
_i32p = C.POINTER(C.c_int32)
_u8p = C.POINTER(C.c_uint8)


class Options(C.Structure):
    _fields_ = [("abi_version", C.c_int32), ("device", C.c_int32), ("partition_bits", C.c_int32),
                ("host_threads", C.c_int32), ("hard_query_limit", C.c_int64), ("stream", C.c_void_p)]


class Rows(C.Structure):
    _fields_ = [("nrows", C.c_int64), ("row_keys", _i64p), ("row_entry_begin", _i64p),
                ("row_byte_begin", _i64p), ("entry_bytes", _u8p), ("entry_limit_valpos", _i64p)]


class EdgeType(C.Structure):
    _fields_ = [("type_id", C.c_int64), ("multiplicity", C.c_int32), ("n_sort_key", C.c_int32),
                ("sort_key_ids", _i64p), ("n_signature", C.c_int32), ("sort_order", C.c_int32),
                ("signature_ids", _i64p)]


class PropertyKey(C.Structure):
    _fields_ = [("key_id", C.c_int64), ("datatype", C.c_int32)]


class Schema(C.Structure):
    _fields_ = [("n_edge_types", C.c_int32), ("edge_types", C.POINTER(EdgeType)),
                ("n_property_keys", C.c_int32), ("property_keys", C.POINTER(PropertyKey))]


class LoadOpts(C.Structure):
    # flags sits in what was the padding after n_labels: same size and offsets as before
    _fields_ = [("scope", C.c_int32), ("apply_cap", C.c_int32), ("n_labels", C.c_int32), ("flags", C.c_int32),
                ("label_ids", _i64p), ("weight_key", C.c_int64)]


LOAD_COLUMN_ORDER = 1       # tgo_load_opts.flags: keep column positions (tgo_gather_lists order)


class EdgeEntry(C.Structure):
    _fields_ = [("type_id", C.c_int64), ("other_id", C.c_int64), ("dir", C.c_int32), ("selected", C.c_int32),
                ("has_weight", C.c_int32), ("weight", C.c_int32)]


class ResultArgs(C.Structure):
    _fields_ = [("kind", C.c_int32), ("reserved", C.c_int32), ("key_ids", C.c_int64 * 2), ("datatypes", C.c_int32 * 2),
                ("relation_id_base", C.c_int64)]


class ResultSize(C.Structure):
    _fields_ = [("nrows", C.c_int64), ("nentries", C.c_int64), ("nbytes", C.c_int64)]


class RowsBuf(C.Structure):
    _fields_ = [("row_keys", _i64p), ("row_entry_begin", _i64p), ("row_byte_begin", _i64p),
                ("entry_bytes", _u8p), ("entry_limit_valpos", _i64p)]


class Edges(C.Structure):
    _fields_ = [("n", C.c_int64), ("m", C.c_int64), ("src", _i32p), ("dst", _i32p),
                ("weight", _i32p), ("titan_ids", _i64p)]


class BfsArgs(C.Structure):
    _fields_ = [("seed", C.c_int64), ("seed_is_dense", C.c_int32), ("max_depth", C.c_int32),
                ("scope", C.c_int32), ("flags", C.c_int32)]


class SsspArgs(C.Structure):
    _fields_ = [("seed", C.c_int64), ("seed_is_dense", C.c_int32), ("max_depth", C.c_int32),
                ("scope", C.c_int32), ("mode", C.c_int32), ("delta", C.c_int64),
                ("flags", C.c_int32), ("reserved", C.c_int32)]


class PrArgs(C.Structure):
    _fields_ = [("alpha", C.c_double), ("vertex_count", C.c_int64), ("max_iterations", C.c_int32),
                ("reserved", C.c_int32)]


class GatherArgs(C.Structure):
    _fields_ = [("scope", C.c_int32), ("value_type", C.c_int32), ("combiner", C.c_int32), ("edge_fn", C.c_int32)]


class EdgeProgram(C.Structure):
    _fields_ = [("n_ops", C.c_int32), ("ops", C.POINTER(C.c_int32)), ("n_consts", C.c_int32),
                ("iconsts", C.POINTER(C.c_int64)), ("fconsts", C.POINTER(C.c_double))]


class Stats(C.Structure):
    _fields_ = [("num_vertices", C.c_int64), ("out_entries", C.c_int64), ("in_entries", C.c_int64), ("ghost_vertices", C.c_int64),
                ("truncated_results", C.c_int64), ("skipped_rows", C.c_int64), ("iterations", C.c_int32),
                ("levels", C.c_int32), ("reached", C.c_int64), ("reached_entries", C.c_int64),
                ("load_ms", C.c_double), ("last_kernel_ms", C.c_double), ("device_bytes", C.c_int64),
                ("relaxed_entries", C.c_int64), ("partitioned_vertices", C.c_int64),
                ("partition_rows", C.c_int64), ("ghost_partition_rows", C.c_int64), ("exact_reruns", C.c_int64)]


# Every symbol include/*.h declares (checked by tests/test_abi.py).
EXPORTS = [
    "tgo_default_options", "tgo_create", "tgo_destroy", "tgo_last_error", "tgo_load_rows",
    "tgo_finish_load", "tgo_load_edges", "tgo_load_csr", "tgo_num_vertices", "tgo_vertex_ids", "tgo_graph_csr", "tgo_graph_perm",
    "tgo_bfs",
    "tgo_sssp", "tgo_copy_distances", "tgo_pagerank", "tgo_walkcount", "tgo_stats_get", "tgo_sync",
    "tgo_bfs_multi", "tgo_copy_multi_distances", "tgo_multi_stats", "tgo_set_tuning",
    "tgo_trace_enable", "tgo_trace_flush", "tgo_trace_clear", "tgo_trace_range_push", "tgo_trace_range_pop",
    "tgo_gather", "tgo_combine_global", "tgo_dense_ids", "tgo_decode_edge_entry", "tgo_result_rows",
    "tgo_gather_lists", "tgo_result_rows_values", "tgo_set_edge_program",
    "tgo_rmat_edges", "tgo_rmat_edges_device", "tgo_rmat_partition_device", "tgo_pick_roots", "tgo_synth_rows",
    # titan_gpu_olap_part.h (1-D vertex-partitioned multi-GPU)
    "tgo_load_partition", "tgo_part_layout", "tgo_load_partition_layout", "tgo_part_bfs_begin", "tgo_part_bfs_td", "tgo_part_bfs_claim", "tgo_part_bfs_bu",
    "tgo_part_bfs_end", "tgo_part_pr_begin", "tgo_part_pr_step", "tgo_part_pr_end", "tgo_part_pr_exact_check", "tgo_part_pr_plain",
    "tgo_part_weight_min", "tgo_load_partition_rows", "tgo_finish_partition_rows",
    "tgo_rmat_partition",
    "tgo_part_active_rows", "tgo_part_pr_blocked", "tgo_part_device_counts", "tgo_part_set_local_qlen", "tgo_part_ms_pack_dev", "tgo_part_pr_step_cold", "tgo_part_pr_step_hot",
    "tgo_part_ms_begin", "tgo_part_ms_pull", "tgo_part_ms_push", "tgo_part_ms_settle", "tgo_part_ms_end",
    "tgo_part_ms_pack", "tgo_part_ms_settle_pairs", "tgo_part_ms_pack_fixed", "tgo_part_ms_settle_fixed",
    "tgo_part_ms_source_counts", "tgo_part_ms_source_entries", "tgo_part_ms_push_masked", "tgo_part_ms_or_fixed",
    "tgo_part_ms_or_pairs", "tgo_part_ms_pull_split",
    "tgo_part_ms_levels", "tgo_part_sssp_begin", "tgo_part_sssp_relax", "tgo_part_sssp_apply",
    "tgo_part_sssp_pending_min", "tgo_part_sssp_extract", "tgo_part_sssp_end",
    "tgo_exchange_rccl_id", "tgo_exchange_rccl_create", "tgo_exchange_local_group", "tgo_exchange_destroy",
    "tgo_exchange_last_error", "tgo_part_msbfs_run", "tgo_part_bfs_run", "tgo_part_sssp_run", "tgo_part_pagerank_run",
]

_lib = None


def load() -> C.CDLL:
    """Load libtitan_gpu_olap.so (raises when it has not been built)."""
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(LIB_PATH):
        raise RuntimeError(f"{LIB_PATH} is missing: build it with `make -C titan_amd/csrc` "
                           "(or __graft_entry__.build()); there is no CPU fallback")
    # If torch is present in this process its HIP runtime must be the one we bind to:
    # import it first so the loader resolves libamdhip64.so.7 to the same copy.
    try:
        import torch  # noqa: F401
    except Exception:  # pragma: no cover - torch is optional for the library itself
        pass
    lib = C.CDLL(LIB_PATH, mode=C.RTLD_GLOBAL)
    P = C.POINTER
    vp = C.c_void_p
    sig = {
        "tgo_default_options": (None, [P(Options)]),
        "tgo_create": (C.c_int, [P(Options), P(vp)]),
        "tgo_destroy": (None, [vp]),
        "tgo_last_error": (C.c_char_p, [vp]),
        "tgo_load_rows": (C.c_int, [vp, P(Rows), P(Schema), P(LoadOpts)]),
        "tgo_finish_load": (C.c_int, [vp]),
        "tgo_result_rows": (C.c_int, [vp, P(ResultArgs), P(ResultSize), P(RowsBuf)]),
        "tgo_decode_edge_entry": (C.c_int, [P(Schema), P(LoadOpts), _u8p, C.c_int64, C.c_int64, P(EdgeEntry)]),
        "tgo_load_edges": (C.c_int, [vp, P(Edges), P(LoadOpts)]),
        "tgo_load_csr": (C.c_int, [vp, C.c_int64, P(C.c_int64), P(C.c_int64), P(C.c_int32), P(C.c_int32),
                                   P(C.c_int64), P(C.c_int32), P(C.c_int32), P(LoadOpts)]),
        "tgo_num_vertices": (C.c_int64, [vp]),
        "tgo_vertex_ids": (C.c_int, [vp, _i64p]),
        "tgo_graph_csr": (C.c_int, [vp, C.c_int32, _i64p, _i64p, P(C.c_int32), P(C.c_int32), P(C.c_uint32)]),
        "tgo_graph_perm": (C.c_int, [vp, P(C.c_int32)]),
        "tgo_bfs": (C.c_int, [vp, P(BfsArgs), _i64p]),
        "tgo_sssp": (C.c_int, [vp, P(SsspArgs), _i64p]),
        "tgo_copy_distances": (C.c_int, [vp, _i64p]),
        "tgo_pagerank": (C.c_int, [vp, P(PrArgs), C.POINTER(C.c_double)]),
        "tgo_walkcount": (C.c_int, [vp, C.c_int32, _i32p]),
        "tgo_stats_get": (C.c_int, [vp, P(Stats)]),
        "tgo_sync": (C.c_int, [vp]),
        "tgo_bfs_multi": (C.c_int, [vp, _i64p, C.c_int32, P(BfsArgs), _i64p]),
        "tgo_copy_multi_distances": (C.c_int, [vp, C.c_int32, _i64p]),
        "tgo_multi_stats": (C.c_int, [vp, _i64p, _i64p]),
        "tgo_set_tuning": (C.c_int, [vp, C.c_int32, C.c_double]),
        "tgo_trace_enable": (C.c_int, [C.c_char_p, C.c_int32]),
        "tgo_trace_flush": (C.c_int, [C.c_char_p]),
        "tgo_trace_clear": (C.c_int, []),
        "tgo_trace_range_push": (C.c_int, [C.c_char_p]),
        "tgo_trace_range_pop": (C.c_int, []),
        "tgo_gather": (C.c_int, [vp, P(GatherArgs), vp, P(C.c_uint8), vp, P(C.c_uint8)]),
        "tgo_gather_lists": (C.c_int, [vp, P(GatherArgs), vp, P(C.c_uint8), _i64p, vp]),
        "tgo_set_edge_program": (C.c_int, [vp, P(EdgeProgram)]),
        "tgo_result_rows_values": (C.c_int, [vp, P(ResultArgs), vp, P(C.c_uint8), P(ResultSize), P(RowsBuf)]),
        "tgo_combine_global": (C.c_int, [vp, C.c_int32, C.c_int32, C.c_int64, _i64p, vp, vp, P(C.c_uint8)]),
        "tgo_dense_ids": (C.c_int, [vp, _i64p, C.c_int64, _i64p]),
        "tgo_rmat_edges": (C.c_int, [C.c_int32, C.c_int32, C.c_uint64, C.c_int64, C.c_int64,
                                     _i32p, _i32p, _i32p, C.c_int32]),
        "tgo_rmat_edges_device": (C.c_int, [C.c_int32, C.c_int32, C.c_uint64, C.c_int64, C.c_int64,
                                            _i32p, _i32p, _i32p, C.c_int32]),
        "tgo_rmat_partition_device": (C.c_int, [C.c_int32, C.c_int32, C.c_uint64, C.c_int64, C.c_int64, _i32p, _i32p,
                                                _i32p, C.c_int64, _i64p, C.c_int32]),
        "tgo_pick_roots": (C.c_int, [C.c_int64, C.c_int64, _i32p, _i32p, C.c_uint64, C.c_int32, _i64p]),
        "tgo_synth_rows": (C.c_int, [C.c_int64, C.c_int64, _i32p, _i32p, _i32p, C.c_int64, C.c_int32, C.c_int32,
                                     _i64p, _i64p, _i64p, _i64p, P(C.c_uint8), _i64p]),
        "tgo_load_partition": (C.c_int, [vp, C.c_int64, C.c_int64, C.c_int64, P(Edges), P(LoadOpts)]),
        "tgo_part_layout": (C.c_int, [P(Edges), C.c_int64, C.c_int64, C.c_int64, C.c_int32, _i32p]),
        "tgo_load_partition_layout": (C.c_int, [vp, C.c_int64, C.c_int64, C.c_int64, P(Edges), P(LoadOpts), _i32p]),
        "tgo_part_bfs_begin": (C.c_int, [vp, C.c_int64, vp, _i64p]),
        "tgo_part_bfs_td": (C.c_int, [vp, C.c_int32, vp]),
        "tgo_part_bfs_claim": (C.c_int, [vp, C.c_int32, vp, C.c_int32, vp, _i64p]),
        "tgo_part_bfs_bu": (C.c_int, [vp, C.c_int32, vp, vp, _i64p]),
        "tgo_part_bfs_end": (C.c_int, [vp, _i64p, _i64p]),
        "tgo_part_ms_begin": (C.c_int, [vp, _i64p, C.c_int32, vp, _i64p]),
        "tgo_part_ms_pull": (C.c_int, [vp, C.c_int32, vp, vp, _i64p]),
        "tgo_part_ms_push": (C.c_int, [vp, C.c_int32, vp, vp]),
        "tgo_part_ms_settle": (C.c_int, [vp, C.c_int32, vp, C.c_int32, vp, _i64p]),
        "tgo_part_ms_pack": (C.c_int, [vp, vp, C.c_int32, vp, _i64p]),
        "tgo_part_ms_settle_pairs": (C.c_int, [vp, C.c_int32, vp, _i64p, C.c_int32, vp, _i64p]),
        "tgo_part_ms_end": (C.c_int, [vp, _i64p, _i64p]),
        "tgo_part_ms_levels": (C.c_int, [vp, C.c_int32, _i64p]),
        "tgo_part_sssp_begin": (C.c_int, [vp, C.c_int64, C.c_int64, _i64p]),
        "tgo_part_sssp_relax": (C.c_int, [vp, C.c_int64, C.c_int32, vp, _i64p]),
        "tgo_part_sssp_apply": (C.c_int, [vp, C.c_int64, vp, C.c_int64, _i64p]),
        "tgo_part_sssp_pending_min": (C.c_int, [vp, _i64p]),
        "tgo_part_sssp_extract": (C.c_int, [vp, C.c_int64, _i64p]),
        "tgo_part_sssp_end": (C.c_int, [vp, _i64p, _i64p]),
        "tgo_part_pr_begin": (C.c_int, [vp, P(PrArgs), vp]),
        "tgo_part_pr_step": (C.c_int, [vp, vp, vp]),
        "tgo_part_pr_end": (C.c_int, [vp, C.POINTER(C.c_double)]),
        "tgo_part_pr_exact_check": (C.c_int, [vp, C.POINTER(C.c_int32)]),
        "tgo_part_pr_plain": (C.c_int, [vp, C.c_int32]),
        "tgo_part_weight_min": (C.c_int, [vp, _i64p]),
        "tgo_load_partition_rows": (C.c_int, [vp, vp, P(Rows), P(Schema), P(LoadOpts), C.c_int32, _i64p]),
        "tgo_finish_partition_rows": (C.c_int, [vp, vp, C.c_int32, _i64p]),
        "tgo_part_active_rows": (C.c_int, [vp, _i64p]),
        "tgo_part_device_counts": (C.c_int, [vp, vp]),
        "tgo_part_set_local_qlen": (C.c_int, [vp, C.c_int64]),
        "tgo_part_ms_pack_dev": (C.c_int, [vp, vp, C.c_int32, vp, vp]),
        "tgo_part_ms_pack_fixed": (C.c_int, [vp, vp, C.c_int32, C.c_int64, vp]),
        "tgo_part_ms_settle_fixed": (C.c_int, [vp, C.c_int32, vp, C.c_int32, C.c_int64, vp, _i64p]),
        "tgo_part_ms_source_counts": (C.c_int, [vp, vp, vp]),
        "tgo_part_ms_source_entries": (C.c_int, [vp, vp, C.c_uint64, vp]),
        "tgo_part_ms_push_masked": (C.c_int, [vp, vp, vp, C.c_uint64]),
        "tgo_part_ms_or_fixed": (C.c_int, [vp, vp, C.c_int32, C.c_int64, vp]),
        "tgo_part_ms_or_pairs": (C.c_int, [vp, vp, _i64p, C.c_int32, vp]),
        "tgo_part_ms_pull_split": (C.c_int, [vp, C.c_int32, vp, vp, C.c_uint64, C.c_int32, _i64p]),
        "tgo_part_pr_blocked": (C.c_int, [vp, C.c_int32, C.c_int64, _i64p]),
        "tgo_part_pr_step_cold": (C.c_int, [vp, vp]),
        "tgo_part_pr_step_hot": (C.c_int, [vp, vp, vp]),
        "tgo_rmat_partition": (C.c_int, [C.c_int32, C.c_int32, C.c_uint64, C.c_int64, C.c_int64, _i32p, _i32p,
                                         _i32p, C.c_int64, _i64p, C.c_int32]),
        "tgo_exchange_rccl_id": (C.c_int, [_u8p]),
        "tgo_exchange_rccl_create": (C.c_int, [C.c_int32, C.c_int32, _u8p, C.c_int32, P(vp)]),
        "tgo_exchange_local_group": (C.c_int, [C.c_int32, P(vp)]),
        "tgo_exchange_destroy": (None, [vp]),
        "tgo_exchange_last_error": (C.c_char_p, [vp]),
        "tgo_part_msbfs_run": (C.c_int, [vp, vp, _i64p, C.c_int32, C.c_int32, C.c_double, C.c_int64, _i64p, _i64p,
                                         P(C.c_int32)]),
        "tgo_part_bfs_run": (C.c_int, [vp, vp, C.c_int64, C.c_int32, C.c_double, C.c_double, _i64p, _i64p,
                                       P(C.c_int32)]),
        "tgo_part_sssp_run": (C.c_int, [vp, vp, C.c_int64, C.c_int64, _i64p, _i64p, P(C.c_int32)]),
        "tgo_part_pagerank_run": (C.c_int, [vp, vp, P(PrArgs), C.c_int32, C.POINTER(C.c_double), _i64p]),
    }
    for name, (res, args) in sig.items():
        f = getattr(lib, name)
        f.restype = res
        f.argtypes = args
    _lib = lib
    return lib


def ptr(arr, ctype):
    """ctypes pointer to a contiguous numpy array (None -> NULL)."""
    if arr is None:
        return None
    return arr.ctypes.data_as(C.POINTER(ctype))

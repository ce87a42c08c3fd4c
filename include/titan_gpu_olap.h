/*
 * titan_gpu_olap.h — C-ABI of the MI355X-native OLAP traversal engine for Titan.
 *
 * This is the drop-in boundary for Titan's in-JVM OLAP executor ("Fulgora"):
 *
 *   graph.compute()                          TitanBlueprintsGraph.java:133-146
 *     .program(VertexProgram)                FulgoraGraphComputer.java:103-107
 *     .workers(n)                            FulgoraGraphComputer.java:96-100
 *     .submit().get()                        FulgoraGraphComputer.java:117-311
 *
 * The Java side keeps TitanGraphComputer (titan-core/.../core/TitanGraphComputer.java:8-43)
 * and the edgestore scan (Backend.buildEdgeScanJob(), Backend.java:336-355 →
 * StandardScanner.Builder, StandardScanner.java:100-209).  A CSR-collecting
 * VertexScanJob hands every scanned row to tgo_load_rows() in the reference's own
 * StaticArrayEntryList layout (StaticArrayEntryList.java:15-50); the superstep loop
 * of FulgoraGraphComputer.submit (:151-189) and the per-vertex gather of
 * VertexMemoryHandler.receiveMessages (VertexMemoryHandler.java:77-103) are replaced
 * by one call per vertex program (tgo_bfs / tgo_sssp / tgo_pagerank / tgo_walkcount)
 * executed by hand-written HIP kernels for gfx950 over a device-resident adjacency.
 *
 * ABI conventions
 *  - Plain C types only; no C++ exceptions cross this boundary.
 *  - Every call returns a tgo_status (0 = ok, < 0 = error class);
 *    tgo_last_error() returns a message for the last failing call on that ctx.
 *    This mirrors the reference's error behaviour: TitanException /
 *    IllegalArgumentException thrown from submit().get() (OLAPTest.java:222-239,
 *    FulgoraGraphComputer.java:165-174).
 *  - The caller owns every host buffer; buffers are read during the call and never
 *    retained.  Output buffers are caller-allocated (n = tgo_num_vertices()).
 *  - Device memory is owned by the ctx and freed by tgo_destroy().
 *  - A ctx is used by one host thread at a time; several ctxs may coexist.
 *  - The library owns one HIP stream per ctx unless tgo_options.stream is given.
 *  - There is NO CPU fallback: when no gfx950 device is usable, tgo_create() fails
 *    with TGO_E_HIP.
 */
#ifndef TITAN_GPU_OLAP_H
#define TITAN_GPU_OLAP_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define TGO_ABI_VERSION 2

typedef struct tgo_ctx tgo_ctx;

typedef enum {
    TGO_OK = 0,
    TGO_E_INVALID = -1,     /* bad argument (Preconditions.checkArgument)               */
    TGO_E_HIP = -2,         /* HIP runtime error / no usable device                      */
    TGO_E_OOM = -3,         /* device or host allocation failed                          */
    TGO_E_CODEC = -4,       /* malformed edgestore entry (EdgeSerializer.parseRelation)  */
    TGO_E_STATE = -5,       /* call order violated (e.g. program before load)            */
    TGO_E_PROGRAM = -6,     /* vertex program failure: the reference throws in execute() */
    TGO_E_UNSUPPORTED = -7, /* feature outside the implemented scope (e.g. Float weights)  */
    TGO_E_COMM = -8         /* multi-GPU exchange failure                                */
} tgo_status;

/* Incident direction of a MessageScope.Local(__::outE / __::inE / __::bothE).
 * Messages flow AGAINST the declared direction: a receiver gathers over the
 * reversed incident step (FulgoraUtil.java:49-62, reversal at :57). */
typedef enum { TGO_SCOPE_OUT_E = 0, TGO_SCOPE_IN_E = 1, TGO_SCOPE_BOTH_E = 2 } tgo_scope;

/* tgo_load_opts.flags: TGO_LOAD_COLUMN_ORDER keeps every entry's position in its Titan row
 * (4 more bytes per entry) so tgo_gather_lists can hand a vertex its messages in the order
 * the reference's receive stream yields them. */
enum { TGO_LOAD_COLUMN_ORDER = 1 };

/* Multiplicity of an edge label (core/Multiplicity.java:21-75). Decides where the
 * other vertex id sits inside an edge entry (EdgeSerializer.java:90-110). */
typedef enum {
    TGO_MULTI = 0, TGO_SIMPLE = 1, TGO_MANY2ONE = 2, TGO_ONE2MANY = 3, TGO_ONE2ONE = 4
} tgo_multiplicity;

/* Datatypes of inline edge properties the decoder can read or skip
 * (graphdb/database/serialize/attribute/ IntegerSerializer.java, LongSerializer.java, ...). */
typedef enum {
    TGO_DT_BYTE = 1, TGO_DT_SHORT = 2, TGO_DT_INTEGER = 3, TGO_DT_LONG = 4,
    TGO_DT_FLOAT = 5, TGO_DT_DOUBLE = 6, TGO_DT_BOOLEAN = 7,
    TGO_DT_DATE = 8,       /* DateSerializer: the Long form of getTime()                    */
    TGO_DT_CHARACTER = 9,  /* CharacterSerializer: 2 bytes                                  */
    TGO_DT_STRING = 10,    /* StringSerializer: ASCII / full UTF / compressed (skipped only) */
    TGO_DT_OBJECT = 11     /* generic key (DefaultSchemaMaker: dataType(Object.class)): the value
                            * class's registration number, then its serializer without a null flag
                            * (StandardSerializer.writeClassAndObject :316-322) — result write-back only */
} tgo_datatype;

/* RelationType sort order (EdgeSerializer.java:137,311-313): DESC inverts the sort-key bytes. */
typedef enum { TGO_ORDER_ASC = 0, TGO_ORDER_DESC = 1 } tgo_sort_order;

typedef struct {
    int32_t abi_version;       /* must be TGO_ABI_VERSION                                  */
    int32_t device;            /* HIP device ordinal                                       */
    int32_t partition_bits;    /* log2(cluster.max-partitions); reference default 5
                                  (GraphDatabaseConfiguration.java:665; VertexIDAssigner.java:73-74) */
    int32_t host_threads;      /* CSR-assembly threads (0 = hardware concurrency)          */
    int64_t hard_query_limit;  /* QueryContainer.DEFAULT_HARD_QUERY_LIMIT = 100000 (QueryContainer.java:28) */
    void*   stream;            /* optional external hipStream_t; NULL = ctx-owned stream   */
} tgo_options;

/* ---- Edgestore input (tgo_load_rows) ------------------------------------------------
 * Rows are passed exactly as the scan hands them to VertexJobConverter.process
 * (VertexJobConverter.java:109-129): per row, the 8-byte key and the row's entry list
 * in StaticArrayEntryList form (StaticArrayEntryList.java:15-50), concatenated over rows:
 *   row_keys[r]                 key as StaticBuffer.getLong(0) (big-endian long)
 *   row_entry_begin[r..r+1)     entry index range of row r                (nrows+1)
 *   row_byte_begin[r]           byte offset of row r's data in entry_bytes (nrows+1)
 *   entry_limit_valpos[e]       (limit << 32) | valuePos, limit = end offset of entry e
 *                               relative to row_byte_begin[r] (StaticArrayEntryList:46-56)
 * Entries of a row are in column byte order, as every backend returns them. */
typedef struct {
    int64_t nrows;
    const int64_t* row_keys;
    const int64_t* row_entry_begin;
    const int64_t* row_byte_begin;
    const uint8_t* entry_bytes;
    const int64_t* entry_limit_valpos;
} tgo_rows;

typedef struct {
    int64_t type_id;              /* UserEdgeLabel schema id (IDManager.getSchemaId)          */
    int32_t multiplicity;         /* tgo_multiplicity                                        */
    int32_t n_sort_key;           /* sort-key property keys (only for MULTI; KEY inline)       */
    const int64_t* sort_key_ids;
    int32_t n_signature;          /* signature property keys, in definition order             */
    int32_t sort_order;           /* tgo_sort_order of the label's sort key (0 = ASC)         */
    const int64_t* signature_ids;
} tgo_edge_type;

typedef struct {
    int64_t key_id;               /* PropertyKey schema id                                    */
    int32_t datatype;             /* tgo_datatype                                             */
} tgo_property_key;

typedef struct {
    int32_t n_edge_types;  const tgo_edge_type* edge_types;
    int32_t n_property_keys; const tgo_property_key* property_keys;
} tgo_schema;

typedef struct {
    int32_t scope;                /* tgo_scope the programs will use; decides the per-row
                                     preload cap: untyped single-direction scopes are cut at
                                     hard_query_limit entries of slice [0x60,0x80), BOTH is
                                     fitted and uncapped (BasicVertexCentricQueryBuilder.java:418-431,
                                     QueryContainer.java:110-134)                              */
    int32_t apply_cap;            /* 1 = reproduce the reference's cap (parity mode), 0 = not   */
    int32_t n_labels;             /* 0 = untyped scope (all user edge labels)                  */
    int32_t flags;                /* TGO_LOAD_* bits (0 = none); fills what was padding        */
    const int64_t* label_ids;     /* typed scope: __.inE("label")... — fitted, no cap          */
    int64_t weight_key;           /* edge property read as weight; 0 = none.  It may sit in a
                                     MULTI label's sort key (ASC or DESC), its signature or its
                                     remaining properties.  Byte, Short, Integer, Character and
                                     Boolean keys are read as integers, Float keys as their IEEE
                                     bits (-0.0 reads as +0.0), Long and Double keys into a
                                     64-bit value table (row loads; generic edge functions only);
                                     other datatypes fail with TGO_E_UNSUPPORTED.
                                     tgo_sssp / tgo_bfs need an Integer key
                                     (ShortestDistanceVertexProgram.java:53 casts edge.<Integer>
                                     value; another datatype is a ClassCastException there);
                                     generic edge functions take any of them.  TTL / timestamp metadata is not
                                     part of the entry bytes (EdgeSerializer.java:154-161 only
                                     copies it into the relation); expired cells never reach the
                                     scan.                                                     */
} tgo_load_opts;

/* Decoded adjacency given directly (bench / already-decoded callers).  Dense vertex ids
 * 0..n-1 in row order; titan_ids may be NULL (ids are then synthesised monotonically).
 * Each directed edge u->v yields an OUT entry at u and an IN entry at v, as the
 * reference's commit path writes two entries per edge (StandardTitanGraph.java:564-591). */
typedef struct {
    int64_t n;                    /* vertices                                                 */
    int64_t m;                    /* directed edges                                           */
    const int32_t* src;           /* m                                                        */
    const int32_t* dst;           /* m                                                        */
    const int32_t* weight;        /* m or NULL                                                */
    const int64_t* titan_ids;     /* n or NULL                                                */
} tgo_edges;

/* ---- Programs ----------------------------------------------------------------------- */

/* ShortestDistanceVertexProgram (titan-test/.../olap/ShortestDistanceVertexProgram.java:49-130)
 * with the edge function (m,e) -> m + 1 (BFS / k-hop) or m + e.value(weight) (SSSP).
 * Iterations 0..max_depth are executed; a vertex's distance is the minimum over walks of
 * at most max_depth hops (Jacobi Bellman-Ford, :96-130).  dist_out[v] = TGO_DIST_ABSENT
 * when no distance property was set (ShortestDistanceMapReduce emits nothing, :45-50). */
typedef struct {
    int64_t seed;                 /* Titan vertex id (ShortestDistanceVertexProgram.seed)     */
    int32_t seed_is_dense;        /* 1: seed is a dense index instead of a Titan id            */
    int32_t max_depth;            /* terminate when iteration >= max_depth (:128-130)          */
    int32_t scope;                /* tgo_scope; must match the loaded scope                    */
    int32_t flags;                /* TGO_FLAG_STATS: fill tgo_stats.reached / reached_entries  */
} tgo_bfs_args;

#define TGO_FLAG_STATS 1
/* Distance value for "no DISTANCE property" (the vertex was not reached). */
#define TGO_DIST_ABSENT INT64_MIN

typedef enum { TGO_SSSP_HOP_BOUNDED = 0, TGO_SSSP_DELTA = 1 } tgo_sssp_mode;

typedef struct {
    int64_t seed;
    int32_t seed_is_dense;
    int32_t max_depth;
    int32_t scope;
    int32_t mode;                 /* tgo_sssp_mode: HOP_BOUNDED = exact reference semantics;
                                     DELTA = converged distances (== reference iff every
                                     shortest path has <= max_depth hops)                     */
    int64_t delta;                /* bucket width for DELTA (0 = auto)                         */
    int32_t flags;                /* TGO_FLAG_STATS                                            */
    int32_t reserved;
} tgo_sssp_args;

/* PageRankVertexProgram (titan-test/.../olap/PageRankVertexProgram.java:45-100):
 * it0 send 1 on inE; it1 edgeCount = sum, PR = 1/N; it>=2 PR = a*sum + (1-a)/N;
 * terminate when iteration >= max_iterations, i.e. max_iterations-1 rank updates. */
typedef struct {
    double  alpha;                /* dampingFactor, default 0.85 (:52)                         */
    int64_t vertex_count;         /* N = configured vertexCount (:54)                          */
    int32_t max_iterations;       /* iterations(k), default 10 (:53)                           */
    int32_t reserved;
} tgo_pr_args;

typedef struct {
    int64_t num_vertices;         /* executed (non-ghost, visible) vertices                   */
    int64_t out_entries;          /* OUT-list entries kept (out-CSR)                           */
    int64_t in_entries;           /* IN-list entries kept (in-CSR)                             */
    int64_t ghost_vertices;       /* VertexJobConverter GHOST_VERTEX_COUNT ("ghost-vertices")  */
    int64_t truncated_results;    /* VertexJobConverter TRUNCATED_ENTRY_LISTS ("truncated-results") */
    int64_t skipped_rows;         /* rows rejected by the key filter (Invisible ids)           */
    int32_t iterations;           /* memory.getIteration() of the last program (FulgoraMemory.java:73-76) */
    int32_t levels;               /* BFS/SSSP frontier levels executed on device               */
    int64_t reached;              /* vertices with a distance after the last BFS/SSSP          */
    int64_t reached_entries;      /* adjacency entries of reached vertices (m_R)               */
    double  load_ms;              /* CSR assembly + upload                                     */
    double  last_kernel_ms;       /* device time of the last program (HIP events)              */
    int64_t device_bytes;         /* device memory held by the ctx                             */
    int64_t relaxed_entries;      /* push entries relaxed by the last SSSP (work done; equals
                                     reached_entries when every vertex is relaxed once)         */
    /* vertex cuts (IDManager PartitionedVertex ids; VertexProgramScanJob.java:76-92) */
    int64_t partitioned_vertices; /* canonical partitioned vertices executed                  */
    int64_t partition_rows;       /* non-canonical representative rows folded into them       */
    int64_t ghost_partition_rows; /* representative rows whose canonical row is absent or a
                                     ghost (PartitionedVertexProgramExecutor "partition-ghost") */
    int64_t exact_reruns;         /* PageRank: 1 when the last program re-ran on the plain fp64
                                     gather because a message left the fixed-point passes' exact
                                     range (+inf from edgeCount 0 after a row cut, NaN, or a
                                     magnitude outside [2^-53, 2^47 / longest row)); 0 otherwise */
} tgo_stats;

/* ---- Entry points ------------------------------------------------------------------- */

void tgo_default_options(tgo_options* opts);
int  tgo_create(const tgo_options* opts, tgo_ctx** out);
void tgo_destroy(tgo_ctx* ctx);
const char* tgo_last_error(const tgo_ctx* ctx);

/* Append one batch of scanned rows (the scan delivers rows in work blocks:
 * StandardScannerExecutor.java:235-288); tgo_finish_load() decodes, assembles and
 * uploads the adjacency.  Replaces the per-superstep rescan + decode. */
int  tgo_load_rows(tgo_ctx* ctx, const tgo_rows* rows, const tgo_schema* schema,
                   const tgo_load_opts* opts);
int  tgo_finish_load(tgo_ctx* ctx);
/* Load an already-decoded edge list (finishes the load). */
int  tgo_load_edges(tgo_ctx* ctx, const tgo_edges* edges, const tgo_load_opts* opts);
/* Load a caller-assembled adjacency (SURVEY §8(b) tgo_load_csr; finishes the load): the
 * rows as a CSR-collecting scan job holds them after VertexJobConverter
 * (VertexJobConverter.java:109-129) — row v (dense index 0..n-1 in row order, Titan id
 * titan_ids[v], strictly increasing; NULL = synthesised) has the OUT entries
 * [out_off[v], out_off[v+1]) and the IN entries [in_off[v], in_off[v+1]) of out_idx / in_idx
 * (dense neighbour indices), weights out_w / in_w (NULL when opts->weight_key == 0).
 * The rows are taken as preloaded: a cut the scan applied stays (opts->apply_cap is not
 * applied again) and the OUT and IN lists need not be transposes of each other (the push view
 * is then an explicit transpose).  A row's OUT entries and then its IN entries, in the given
 * order, are its column order (TGO_LOAD_COLUMN_ORDER positions).  opts->scope picks the
 * views as for every load; label_ids must be empty.
 * Returns TGO_E_INVALID for decreasing offsets, an index outside [0, n), non-increasing
 * titan_ids or a missing weight array; TGO_E_STATE while a tgo_load_rows scan is in progress
 * (its staged rows are kept: tgo_finish_load still completes it). */
int  tgo_load_csr(tgo_ctx* ctx, int64_t n, const int64_t* titan_ids, const int64_t* out_off,
                  const int32_t* out_idx, const int32_t* out_w, const int64_t* in_off,
                  const int32_t* in_idx, const int32_t* in_w, const tgo_load_opts* opts);

/* One edge entry through the product decoder (EdgeSerializer.parseRelation, :73-166, restricted
 * to what the traversal reads), on the host, without a ctx or a device: the per-entry half of
 * tgo_load_rows, for callers that decode single entries and for codec tests.
 * Returns TGO_OK, TGO_E_CODEC (malformed), TGO_E_UNSUPPORTED (an inline property of a key
 * missing from the schema; a non-Integer weight key).  selected = 0: the label is outside the
 * typed scope (the entry is not preloaded). */
typedef struct {
    int64_t type_id;
    int64_t other_id;             /* other vertex Titan id                                    */
    int32_t dir;                  /* 0 OUT, 1 IN                                              */
    int32_t selected;
    int32_t has_weight;
    int32_t weight;
} tgo_edge_entry;
/* (A Long / Double weight key fails here with TGO_E_UNSUPPORTED: the weight field is 32 bits.) */
int  tgo_decode_edge_entry(const tgo_schema* schema, const tgo_load_opts* opts, const uint8_t* entry,
                           int64_t len, int64_t value_pos, tgo_edge_entry* out);

int64_t tgo_num_vertices(const tgo_ctx* ctx);
/* Titan vertex id of every dense index, in row order (n entries). */
int  tgo_vertex_ids(tgo_ctx* ctx, int64_t* titan_ids_out);

/* Inspection of the assembled device graph (tests: device vs host assembly, array for
 * array).  which: 0 = OUT lists, 1 = IN lists, 2 = the push transpose (absent: *nnz = -1).
 * Internal (degree-grouped) ids.  *nnz = entries; off (n+1), adj, w, col (nnz each) are
 * filled when non-NULL (w / col only if the load kept them).  tgo_graph_perm: row-order
 * dense id -> internal id (n).  A load assembles on the device unless TGO_HOST_ASSEMBLY=1
 * (edge lists; rows keep the host assembly), latched per load. */
int  tgo_graph_csr(tgo_ctx* ctx, int32_t which, int64_t* nnz, int64_t* off, int32_t* adj, int32_t* w, uint32_t* col);
int  tgo_graph_perm(tgo_ctx* ctx, int32_t* perm);

/* BFS / k-hop: ShortestDistance with unit edge function.  dist_out may be NULL: the
 * result then stays on the device (tgo_copy_distances fetches it). */
int  tgo_bfs(tgo_ctx* ctx, const tgo_bfs_args* args, int64_t* dist_out);
int  tgo_sssp(tgo_ctx* ctx, const tgo_sssp_args* args, int64_t* dist_out);

/* Multi-source BFS: up to TGO_MAX_SOURCES ShortestDistance programs with unit weights (one
 * per seed; args->seed is ignored) run together with bit-parallel frontiers, one pass over
 * the adjacency per level for all of them.  Each seed's distances equal its own tgo_bfs.
 * dist_out: NULL (results stay on the device) or nseeds * n values, seed-major. */
#define TGO_MAX_SOURCES 64
int  tgo_bfs_multi(tgo_ctx* ctx, const int64_t* seeds, int32_t nseeds, const tgo_bfs_args* args,
                   int64_t* dist_out);
int  tgo_copy_multi_distances(tgo_ctx* ctx, int32_t source, int64_t* dist_out);
/* Per-ctx tuning of a traversal policy (never of a result: every value gives the same
 * distances / ranks).  TGO_TUNE_MS_SPLIT: push budget of the sparse sources at the first pull
 * level of a multi-source sweep (tgo_bfs_multi, tgo_part_msbfs_run), a fraction of the list
 * entries; 0 = every source pulled; < 0 = the default (TGO_MS_SPLIT or 0.005). */
/* TGO_TUNE_MS_GHOST (partitioned tgo_part_msbfs_run): 1 (default) = a dense level refreshes
 * only the frontier masks this rank's lists read (ghost exchange: all-to-allv of precomputed
 * lists), 0 = all-gather of every rank's masks. */
/* TGO_TUNE_DS_BINS (one-GPU delta SSSP, tgo_sssp DELTA on a weighted load): 1 (default, or
 * TGO_DS_BINS) = the next bucket is extracted from a pile of the vertices improved into it,
 * 0 = by a scan of the whole pending bitmap.  TGO_TUNE_DS_PILE_CAP: entries a pile holds per
 * bucket before that bucket falls back to the scan (0 = the vertex count; tests use small caps). */
/* TGO_TUNE_DS_DONE: 1 = the binned loop's relax skips the distance read of targets whose bucket
 * finished (0, default: reads every target).  TGO_TUNE_MS_COLD (tgo_bfs_multi): 1 = the first
 * pull level of a run walks only the hot neighbours and a blocked pass over the cold entries
 * completes the open rows; 0 (default, or TGO_MS_COLD) = the plain walk; a value > 1 = on, with
 * that many hot neighbours and cold segments of that size (tests). */
/* TGO_TUNE_DS_PULL (binned delta SSSP): a fraction f in (0, 1] = a finished bucket with at least
 * f * n members has its heavy entries pulled by the vertices that can still improve instead of
 * pushed; 0 = always pushed; -1 = TGO_DS_PULL (default 0).  Same distances either way. */
/* TGO_TUNE_DS_SMALL (binned delta SSSP without the done filter and pulls): 1 = the tiny steps
 * run in one block inside one launch (ds_small_steps), 0 = four grid launches per step;
 * -1 = TGO_DS_SMALL (default 0: measured slower).  Same distances either way. */
enum { TGO_TUNE_MS_SPLIT = 1, TGO_TUNE_MS_GHOST = 2, TGO_TUNE_DS_BINS = 3, TGO_TUNE_DS_PILE_CAP = 4,
       TGO_TUNE_DS_DONE = 5, TGO_TUNE_MS_COLD = 6, TGO_TUNE_DS_PULL = 7, TGO_TUNE_DS_SMALL = 8 };
int  tgo_set_tuning(tgo_ctx* ctx, int32_t key, double value);

/* ---- Tracing (the reference's only hook is FulgoraGraphComputer.java:143,307
 * memory.setRuntime).  Every program marks its supersteps / levels / phases as spans:
 * TGO_TRACE_ROCTX: roctx ranges (rocprofv3 --marker-trace shows them beside the kernels);
 * TGO_TRACE_JSON: Chrome-trace events ("traceEvents", ph "X"; cat "device" spans carry GPU
 * times from HIP events on the engine stream, cat "host" spans host times; args = the level,
 * iteration, frontier size ...), written by tgo_trace_flush (json_path NULL = the path given
 * to tgo_trace_enable or TGO_TRACE_JSON; TGO_TRACE_JSON also flushes at exit).  Process-wide.
 * tgo_trace_range_push / _pop: the caller's own ranges (per thread, nested). */
enum { TGO_TRACE_JSON = 1, TGO_TRACE_ROCTX = 2 };
int  tgo_trace_enable(const char* json_path, int32_t flags);   /* flags 0 = off */
int  tgo_trace_flush(const char* json_path);
int  tgo_trace_clear(void);
int  tgo_trace_range_push(const char* name);
int  tgo_trace_range_pop(void);
/* After tgo_bfs_multi with TGO_FLAG_STATS: per seed, reached vertices and their entries. */
int  tgo_multi_stats(tgo_ctx* ctx, int64_t* reached, int64_t* reached_entries);
int  tgo_copy_distances(tgo_ctx* ctx, int64_t* dist_out);
int  tgo_pagerank(tgo_ctx* ctx, const tgo_pr_args* args, double* pr_out);
/* OLAPTest.DegreeCounter(k) (OLAPTest.java:334-416): k-walk counts, Java int wrap. */
int  tgo_walkcount(tgo_ctx* ctx, int32_t k, int32_t* out);

/* ---- Generic vertex programs ----------------------------------------
 * A vertex program the engine does not implement natively runs its execute() on the host
 * over whole per-vertex vectors (titan_amd/computer.py GenericVertexProgram; the Java host
 * would do the same) while the device combines its messages, superstep by superstep:
 *   tgo_gather          MessageScope.Local(incident, edgeFct): for every vertex, the combiner
 *                       over edgeFct(msg[u], e) for the entries of its reversed incident
 *                       traversal whose sender u holds a message (VertexMemoryHandler.java:
 *                       77-93, FulgoraUtil.java:57).  The scope must be the loaded scope, or
 *                       any direction of a bothE load (whose lists are uncapped).
 *   tgo_combine_global  MessageScope.Global: the messages sent to each target combined in the
 *                       order they were sent (VertexState.addMessage, VertexState.java:63-78).
 * Vectors are host arrays in the API's row order (n = tgo_num_vertices); has[] = 1 where a
 * message is present (NULL in: every vertex holds one).  MIN/MAX and int64 SUM are exact;
 * fp64 SUM folds in a fixed order (list order / message order): bitwise reproducible.
 * int64 arithmetic wraps like Java long.  A weight edge function over an edge without the
 * weight property fails with TGO_E_PROGRAM (edge.value() throws in the reference). */
typedef enum { TGO_COMBINE_SUM = 0, TGO_COMBINE_MIN = 1, TGO_COMBINE_MAX = 2 } tgo_combiner;
typedef enum { TGO_VAL_INT64 = 0, TGO_VAL_FP64 = 1 } tgo_value_type;
/* Edge functions: (message, edge) -> message, the BiFunction of MessageScope.Local
 * (VertexMemoryHandler.java:85,90) as "message op w", w = e.value(weight) of the load's
 * weight key (an integral key, Float, Long or Double).  int64 arithmetic wraps like Java
 * long; int64 / 0 fails with TGO_E_PROGRAM; a Float or Double weight with int64 messages
 * with TGO_E_INVALID (long op double is a double in Java). */
typedef enum {
    TGO_EDGE_IDENTITY = 0,    /* (m, e) -> m                    */
    TGO_EDGE_ADD_ONE = 1,     /* (m, e) -> m + 1                */
    TGO_EDGE_ADD_WEIGHT = 2,  /* (m, e) -> m + w                */
    TGO_EDGE_MUL_WEIGHT = 3,  /* (m, e) -> m * w                */
    TGO_EDGE_SUB_WEIGHT = 4,  /* (m, e) -> m - w                */
    TGO_EDGE_MIN_WEIGHT = 5,  /* (m, e) -> min(m, w)            */
    TGO_EDGE_MAX_WEIGHT = 6,  /* (m, e) -> max(m, w)            */
    TGO_EDGE_DIV_WEIGHT = 7,  /* (m, e) -> m / w (Java / : int64 truncates, / 0 throws) */
    TGO_EDGE_PROGRAM = 8      /* (m, e) -> the ctx's edge-function program (below)       */
} tgo_edge_fn;
/* Edge-function programs: any composition of Java arithmetic over the message m, the weight
 * w = e.value(weight) and constants — the BiFunction<M, Edge, M> of MessageScope.Local
 * (VertexMemoryHandler.java:85,90) beyond the fixed menu, as a postfix program interpreted per
 * entry on the device.  ops[i] = tgo_edge_op | (constant index << 8); a binary op pops b, then
 * a, and pushes a op b.  Arithmetic is the message type's (Java long: + - * and negation wrap,
 * / and % truncate, / 0 and % 0 throw -> TGO_E_PROGRAM, MIN_VALUE / -1 = MIN_VALUE; Java double:
 * IEEE, % = fmod, min / max / abs as Math.min / max / abs).  The constants come in both types
 * (iconsts for long messages, fconsts for double ones; NULL: the program cannot run on that
 * type).  At most TGO_EDGE_PROGRAM_MAX_OPS ops, TGO_EDGE_PROGRAM_MAX_CONSTS constants and a
 * stack of TGO_EDGE_PROGRAM_MAX_STACK; the program must leave exactly one value.  A program
 * that pushes w fails on an edge without the weight property like the menu's weight functions,
 * and with long messages needs an integral weight key. */
typedef enum {
    TGO_OP_MSG = 0, TGO_OP_WEIGHT = 1, TGO_OP_CONST = 2,
    TGO_OP_ADD = 3, TGO_OP_SUB = 4, TGO_OP_MUL = 5, TGO_OP_DIV = 6, TGO_OP_REM = 7,
    TGO_OP_MIN = 8, TGO_OP_MAX = 9, TGO_OP_NEG = 10, TGO_OP_ABS = 11
} tgo_edge_op;
#define TGO_EDGE_PROGRAM_MAX_OPS 32
#define TGO_EDGE_PROGRAM_MAX_CONSTS 16
#define TGO_EDGE_PROGRAM_MAX_STACK 8
typedef struct {
    int32_t n_ops;
    const int32_t* ops;
    int32_t n_consts;
    const int64_t* iconsts;   /* n_consts long constants, or NULL                          */
    const double* fconsts;    /* n_consts double constants, or NULL                        */
} tgo_edge_program;
/* Validates and stores the program on the ctx (NULL clears it); TGO_E_INVALID names the first
 * bad op.  Host-only: no device work. */
int  tgo_set_edge_program(tgo_ctx* ctx, const tgo_edge_program* prog);
typedef struct {
    int32_t scope;            /* tgo_scope of the Local message scope                     */
    int32_t value_type;       /* tgo_value_type                                          */
    int32_t combiner;         /* tgo_combiner (the program's MessageCombiner)            */
    int32_t edge_fn;          /* tgo_edge_fn                                             */
} tgo_gather_args;
int  tgo_gather(tgo_ctx* ctx, const tgo_gather_args* args, const void* msg, const uint8_t* has,
                void* out, uint8_t* out_has);
/* The same receive WITHOUT a combiner: every vertex's message stream materialised —
 * edgeFct(msg[u], e) for each entry of its reversed incident traversal whose sender holds a
 * message, in the row's column order (the order the reference's stream yields them,
 * VertexMemoryHandler.java:83-92) when the graph was loaded with TGO_LOAD_COLUMN_ORDER, else
 * in (direction, neighbour) order.  row_offsets: n+1 (row order); values: NULL for a sizing
 * call, else row_offsets[n] values.  args->combiner is ignored.  A vertex cut receiving 2 or
 * more messages fails with TGO_E_PROGRAM (FulgoraUtil's ThrowingCombiner, :80-91). */
int  tgo_gather_lists(tgo_ctx* ctx, const tgo_gather_args* args, const void* msg, const uint8_t* has,
                      int64_t* row_offsets, void* values);
/* targets: dense row ids (tgo_dense_ids); values: nmsgs int64 or fp64. */
int  tgo_combine_global(tgo_ctx* ctx, int32_t value_type, int32_t combiner, int64_t nmsgs,
                        const int64_t* targets, const void* values, void* out, uint8_t* out_has);
/* Titan vertex ids -> dense row ids (canonical id of a vertex cut, VertexMemoryHandler.java:
 * 111-115); -1 for an id that is not an executed vertex (its messages are never read). */
int  tgo_dense_ids(tgo_ctx* ctx, const int64_t* titan_ids, int64_t count, int64_t* dense_out);

/* ---- Result write-back ----------------------------------------------
 * ResultMode PERSIST / LOCALTX: FulgoraGraphComputer writes every vertex's compute-key
 * properties back with v.property(Cardinality.single, key, value) in batched transactions
 * (FulgoraGraphComputer.java:248-305, VertexPropertyWriter :314-342).  tgo_result_rows encodes,
 * on the device, the edgestore entries those writes produce for the LAST finished program of
 * `kind` — one row per vertex holding the property, in the API's row order, each entry a
 * SINGLE-cardinality property entry (EdgeSerializer.writeRelation :261-283): column = the key's
 * relation-type header, value = null flag + serialized value + relation id.  The caller hands
 * the rows to the store as mutations (column overwrite = the single-cardinality replace).
 *   DISTANCE  ShortestDistance DISTANCE (Long) on reached vertices (tgo_bfs / tgo_sssp)
 *   PAGERANK  PAGE_RANK and OUTGOING_EDGE_COUNT (Double) on every executed vertex once
 *             iterations >= 1 (PageRankVertexProgram.java:79-88)
 *   DEGREE    OLAPTest.DegreeCounter DEGREE (Integer) on every executed vertex
 * Compute keys are typed property keys of those datatypes, or generic keys (TGO_DT_OBJECT: what
 * getOrCreatePropertyKey makes for a key the program sets without a schema, DefaultSchemaMaker
 * .java:46-48), whose values carry their class (Long 13, Double 20, Integer 12).  Relation ids are
 * relation_id_base + the entry's running index (a block the caller reserved).
 * out == NULL: only *size is filled; otherwise out's buffers (sized from a first call) get
 * nrows keys, nrows+1 entry / byte offsets, nbytes bytes and nentries limit|valuePos words
 * (the tgo_rows layout, so the rows can be scanned again). */
typedef enum { TGO_RESULT_DISTANCE = 0, TGO_RESULT_PAGERANK = 1, TGO_RESULT_DEGREE = 2,
               TGO_RESULT_VALUES = 3 } tgo_result_kind;
typedef struct {
    int32_t kind;                 /* tgo_result_kind                                          */
    int32_t reserved;             /* TGO_RESULT_VALUES: tgo_value_type of the values           */
    int64_t key_ids[2];           /* [0] DISTANCE / PAGE_RANK / DEGREE key; [1] OUTGOING_EDGE_COUNT */
    int32_t datatypes[2];         /* tgo_datatype of each key                                  */
    int64_t relation_id_base;
} tgo_result_args;
typedef struct { int64_t nrows, nentries, nbytes; } tgo_result_size;
typedef struct {
    int64_t* row_keys;
    int64_t* row_entry_begin;
    int64_t* row_byte_begin;
    uint8_t* entry_bytes;
    int64_t* entry_limit_valpos;
} tgo_rows_buf;
int  tgo_result_rows(tgo_ctx* ctx, const tgo_result_args* args, tgo_result_size* size, const tgo_rows_buf* out);
/* A generic program's compute key (kind TGO_RESULT_VALUES, key_ids[0], datatypes[0], value
 * type in args->reserved): values / present in the API's row order, the host vectors the
 * program's execute() left (int64: a Long, Integer or generic key — an Integer key needs
 * every present value in int range, else TGO_E_INVALID; fp64: a Double or generic key).
 * Entries exactly as for the native programs (one SINGLE-cardinality property entry per
 * present vertex, FulgoraGraphComputer.java:248-305). */
int  tgo_result_rows_values(tgo_ctx* ctx, const tgo_result_args* args, const void* values, const uint8_t* present,
                            tgo_result_size* size, const tgo_rows_buf* out);

int  tgo_stats_get(tgo_ctx* ctx, tgo_stats* out);
/* Block until all work queued on the ctx stream has finished. */
int  tgo_sync(tgo_ctx* ctx);

#ifdef __cplusplus
}
#endif
#endif /* TITAN_GPU_OLAP_H */

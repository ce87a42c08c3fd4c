/*
 * fulgora_ref.h — CPU ORACLE (test infrastructure only; never shipped, never measured
 * as the product).  Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline
 * leg may load it.
 *
 * A plain-C restatement of the reference's OLAP path so the HIP engine can be checked
 * against it on identical inputs:
 *   - edgestore codec: VariableLong, IDManager, IDHandler, EdgeSerializer (decode and
 *     encode), StandardSerializer null flag + Integer/Long zig-zag/offset encodings;
 *   - row -> PreloadedVertex restatement: key filter, ghost check, user-edge slice
 *     [0x60,0x80) with the QueryContainer hard limit (VertexJobConverter.java:109-171,
 *     QueryContainer.java:28,110-134, BasicVertexCentricQueryBuilder.java:418-431);
 *   - the Fulgora BSP executor: every vertex executes every superstep, pulls messages
 *     over its own preloaded reversed-scope entries, neighbour messages looked up by
 *     Titan id in a hash map (FulgoraVertexMemory.java:49-96), double-buffered messages
 *     (VertexState.java:55-89), iteration numbering/termination
 *     (FulgoraGraphComputer.java:151-189, FulgoraMemory.java:73-76);
 *   - the programs: ShortestDistanceVertexProgram (unit or weighted), PageRankVertexProgram,
 *     OLAPTest.DegreeCounter.
 *
 * Parity pinning (see DESIGN.md "Oracle"): the Java reference cannot be built or run here
 * (no JDK, no jars), so this restatement is pinned by the reference's own known answers:
 * OLAPTest closed forms (PageRank tree, ShortestDistance tree, DegreeCounter uid/degree-2),
 * the GraphOfTheGods anchors in SURVEY.md §8c, and hand-derived codec vectors.
 */
#ifndef FULGORA_REF_H
#define FULGORA_REF_H
#include <stdint.h>
#include <stddef.h>
#ifdef __cplusplus
extern "C" {
#endif

enum { FR_OK = 0, FR_E_INVALID = -1, FR_E_CODEC = -4, FR_E_PROGRAM = -6, FR_E_UNSUPPORTED = -7 };
enum { FR_SCOPE_OUT_E = 0, FR_SCOPE_IN_E = 1, FR_SCOPE_BOTH_E = 2 };
enum { FR_MULTI = 0, FR_SIMPLE = 1, FR_MANY2ONE = 2, FR_ONE2MANY = 3, FR_ONE2ONE = 4 };
enum { FR_DT_BYTE = 1, FR_DT_SHORT = 2, FR_DT_INTEGER = 3, FR_DT_LONG = 4,
       FR_DT_FLOAT = 5, FR_DT_DOUBLE = 6, FR_DT_BOOLEAN = 7,
       FR_DT_DATE = 8, FR_DT_CHARACTER = 9, FR_DT_STRING = 10 };
enum { FR_ASC = 0, FR_DESC = 1 };   /* RelationType sort order (EdgeSerializer.java:137,311-313) */

#define FR_ABSENT INT64_MIN   /* "no distance property" */

/* ---- codec (VariableLong.java / IDManager.java / IDHandler.java) ---- */
typedef struct { uint8_t* p; size_t len, cap; } fr_buf;
void    fr_buf_free(fr_buf* b);
void    fr_vl_write_positive(fr_buf* b, int64_t v);                 /* VariableLong.java:84-87 */
int64_t fr_vl_read_positive(const uint8_t* d, size_t* pos);         /* :78-82 + :30-38 */
void    fr_vl_write(fr_buf* b, int64_t v);                          /* :125-127 zig-zag */
int64_t fr_vl_read(const uint8_t* d, size_t* pos);                  /* :129-131 */
void    fr_vl_write_positive_with_prefix(fr_buf* b, int64_t v, int64_t prefix, int prefix_len); /* :139-164 */
void    fr_vl_read_positive_with_prefix(const uint8_t* d, size_t* pos, int prefix_len,
                                        int64_t* value, int64_t* prefix); /* :171-186 */
void    fr_vl_write_positive_backward(fr_buf* b, int64_t v);        /* :193-196 + :234-245 */
int64_t fr_vl_read_positive_backward(const uint8_t* d, size_t* pos);/* :202-204 + :254-272; pos = end, moved to start */
int     fr_vl_positive_length(int64_t v);
int     fr_vl_backward_length(int64_t v);

int64_t fr_schema_id(int type /*0=UserPropertyKey,1=SystemPropertyKey,2=UserEdgeLabel,3=SystemEdgeLabel*/, int64_t count);
int64_t fr_vertex_id(int64_t count, int64_t partition, int partition_bits);     /* IDManager.constructId, NormalVertex */
int64_t fr_key_of(int64_t vertex_id, int partition_bits);                       /* IDManager.getKey :461-473 */
int64_t fr_key_id(int64_t key, int partition_bits);                             /* IDManager.getKeyID :476-486 */
int64_t fr_partitioned_vertex_id(int64_t count, int64_t partition, int partition_bits); /* constructId, PartitionedVertex */
int     fr_is_partitioned(int64_t vid, int partition_bits);                     /* isPartitionedVertex :557-559 */
int64_t fr_canonical_vertex_id(int64_t vid, int partition_bits);                /* getCanonicalVertexId :530-534 */
int     fr_is_invisible(int64_t vertex_id);

/* Relation-type column prefix (IDHandler.writeRelationType, :88-94). dir: 0 OUT/property, 1 IN. */
void    fr_write_relation_type(fr_buf* b, int64_t type_id, int is_edge, int dir, int invisible);
int     fr_read_relation_type(const uint8_t* d, size_t* pos, int64_t* type_id, int* is_edge, int* dir);

/* ---- rows / schema (same layout as tgo_rows) ---- */
typedef struct {
    int64_t nrows;
    const int64_t* row_keys;
    const int64_t* row_entry_begin;
    const int64_t* row_byte_begin;
    const uint8_t* entry_bytes;
    const int64_t* entry_limit_valpos;
} fr_rows;

typedef struct {
    int64_t type_id; int32_t multiplicity;
    int32_t n_sort_key; const int64_t* sort_key_ids;
    int32_t n_signature; int32_t sort_order;   /* FR_ASC / FR_DESC */
    const int64_t* signature_ids;
} fr_edge_type;
typedef struct { int64_t key_id; int32_t datatype; } fr_property_key;
typedef struct {
    int32_t n_edge_types; const fr_edge_type* edge_types;
    int32_t n_property_keys; const fr_property_key* property_keys;
} fr_schema;

/* ---- encoder: one edge entry (EdgeSerializer.writeRelation, :222-315) ---- */
/* Inline property value, carried as an int64 `value` whose meaning follows the key's
 * datatype: integral types and Date (ms) as is, Float/Double = (float)/(double)value,
 * Character = (uint16_t)value, String = fr_string_of(value) (decimal digits of |value|,
 * prefixed by U+00E9 U+2135 when value < 0 so both multi-byte UTF forms occur; "" for 0). */
typedef struct { int64_t key_id; int64_t value; } fr_prop;
/* UTF-16 code units of fr_prop's String for `value`; returns the length (<= 24). */
int fr_string_of(int64_t value, uint16_t* chars);
/* One value through StandardSerializer (byte_order: the sort-key form, writeByteOrder).
 * Exposed for the codec known-answer tests. */
int fr_write_value(fr_buf* out, int datatype, int present, int64_t value, int byte_order);
int fr_encode_edge(fr_buf* out, int32_t* value_pos, const fr_schema* schema, int64_t type_id,
                   int dir, int64_t other_vertex_id, int64_t relation_id,
                   const fr_prop* props, int nprops);
/* A SINGLE-cardinality user property entry (prefix 0x40-0x5F, outside the edge slice). */
int fr_encode_property(fr_buf* out, int32_t* value_pos, int64_t key_id, int datatype,
                       int64_t value, int64_t relation_id);
/* The same for a Double-valued key (DoubleSerializer.write: the raw IEEE bits, :33-36). */
int fr_encode_property_f64(fr_buf* out, int32_t* value_pos, int64_t key_id, double value, int64_t relation_id);
/* The same for a generic (Object-typed) key: writeClassAndObject — the value class's
 * registration number, then its serializer without a null flag (value_dt: INTEGER, LONG or
 * DOUBLE, a Double passed as its IEEE bits). */
int fr_encode_property_generic(fr_buf* out, int32_t* value_pos, int64_t key_id, int value_dt,
                               int64_t value, int64_t relation_id);
/* VertexExists system property entry (BaseKey.java:27-28), the first entry of every live row. */
int fr_encode_vertex_exists(fr_buf* out, int32_t* value_pos, int64_t relation_id);
/* Decode one edge entry.  weight_key==0: no weight.  Returns FR_OK / FR_E_CODEC. */
int fr_decode_edge(const uint8_t* d, size_t len, size_t value_pos, const fr_schema* schema,
                   int64_t weight_key, int64_t* type_id, int* dir, int64_t* other_id,
                   int64_t* relation_id, int* has_weight, int64_t* weight);

/* ---- preloaded graph ---- */
typedef struct fr_graph fr_graph;
typedef struct {
    int32_t scope; int32_t apply_cap; int64_t hard_query_limit;
    int32_t n_labels; const int64_t* label_ids; int64_t weight_key; int32_t partition_bits;
} fr_load_opts;
typedef struct {
    int64_t ghost_vertices, truncated_results, skipped_rows, num_entries;
    int64_t partitioned_vertices;      /* canonical vertex-cut vertices executed              */
    int64_t partition_rows;            /* non-canonical representative rows folded into them  */
    int64_t ghost_partition_rows;      /* representative rows whose canonical row is absent or a ghost
                                          (PartitionedVertexProgramExecutor GHOTST_PARTITION_VERTEX) */
} fr_load_stats;

int  fr_load_rows(const fr_rows* rows, const fr_schema* schema, const fr_load_opts* opts,
                  fr_graph** out, fr_load_stats* stats);
/* Decoded adjacency (dense ids; per vertex OUT entries [off[v],mid[v]), IN [mid[v],off[v+1])),
 * copied into the oracle's Titan-id keyed form. w may be NULL. */
int  fr_load_adjacency(int64_t n, const int64_t* titan_ids, const int64_t* off, const int64_t* mid,
                       const int32_t* adj, const int32_t* w, fr_graph** out);
/* Rows from a directed edge list (both entries per edge, column order). w may be NULL. */
int  fr_load_edges(int64_t n, int64_t m, const int32_t* src, const int32_t* dst, const int32_t* w,
                   const int64_t* titan_ids, fr_graph** out);
/* fr_load_edges with the preload cap of an untyped single-direction scope (hard_limit > 0;
 * QueryContainer.java:28,122): *truncated = rows with >= hard_limit entries. */
int  fr_load_edges_capped(int64_t n, int64_t m, const int32_t* src, const int32_t* dst, const int32_t* w,
                          const int64_t* titan_ids, int64_t hard_limit, int64_t* truncated, fr_graph** out);
/* Memoise every entry's hash-map lookup (speed only; results are unchanged). */
int  fr_resolve(fr_graph* g, int threads);
void fr_free(fr_graph* g);
int64_t fr_num_vertices(const fr_graph* g);
void fr_vertex_ids(const fr_graph* g, int64_t* out);
/* Export the oracle's decoded adjacency in dense form (for tests). */
int64_t fr_num_entries(const fr_graph* g);
int64_t fr_export(const fr_graph* g, int64_t* off, int64_t* mid, int32_t* adj, int32_t* w);

/* ---- programs (threads = FulgoraGraphComputer.workers) ---- */
int fr_shortest_distance(const fr_graph* g, int64_t seed_titan_id, int max_depth, int scope,
                         int weighted, int threads, int64_t* dist_out, int* iterations_out);
int fr_pagerank(const fr_graph* g, double alpha, int64_t vertex_count, int max_iterations,
                int threads, double* pr_out, int* iterations_out);
/* Generic message passing (value_type 0 = int64, 1 = fp64; combiner 0 SUM, 1 MIN, 2 MAX;
 * edge_fn 0 identity, 1 +1, 2 +weight, 3 *weight).  Vectors in oracle vertex order. */
int fr_weight_datatype_ok(int datatype);
int fr_gather_lists(const fr_graph* g, int scope, int value_type, int edge_fn, const void* msg, const uint8_t* has,
                    int64_t* off, void* vals);
/* edge_fn 8: the postfix program set here (op codes of tgo_edge_op; fulgora_ref.c prog_eval_*) */
int fr_set_edge_program(const int32_t* ops, int n, const int64_t* iconsts, const double* fconsts, int nconsts);
int fr_gather(const fr_graph* g, int scope, int value_type, int combiner, int edge_fn, const void* msg,
              const uint8_t* has, void* out, uint8_t* out_has);
int fr_combine_global(int64_t n, int value_type, int combiner, int64_t nmsgs, const int64_t* targets,
                      const void* values, void* out, uint8_t* out_has);
int fr_degree_counter(const fr_graph* g, int length, int threads, int32_t* out, int* iterations_out);

#ifdef __cplusplus
}
#endif
#endif

/*
 * tgo_synth.h — synthetic inputs for the bench and the parity tests (not part of the
 * reference boundary; the reference reads real edgestore rows).
 *
 * RMAT / Graph500 Kronecker generator (A,B,C,D = 0.57,0.19,0.19,0.05), counter-based
 * splitmix64 so any edge range can be generated independently and in parallel, followed
 * by a seeded vertex relabel.  Duplicates and self-loops are kept (a Titan MULTI label
 * stores them).  Weights: w = 1 + (splitmix64(seed ^ edge_index) mod 255).
 */
#ifndef TGO_SYNTH_H
#define TGO_SYNTH_H
#include <stdint.h>
#ifdef __cplusplus
extern "C" {
#endif

/* Fill src/dst (m entries each, m = edge_factor << scale) and optionally weight.
 * Edges [edge_begin, edge_begin + count) of the stream are produced. */
int tgo_rmat_edges(int32_t scale, int32_t edge_factor, uint64_t seed, int64_t edge_begin,
                   int64_t count, int32_t* src, int32_t* dst, int32_t* weight, int32_t threads);

/* tgo_rmat_edges computed on GPU `device` (the same stream, bit for bit): the edges are
 * generated there chunk by chunk and copied into the host arrays.  TGO_E_HIP without a usable
 * device. */
int tgo_rmat_edges_device(int32_t scale, int32_t edge_factor, uint64_t seed, int64_t edge_begin,
                          int64_t count, int32_t* src, int32_t* dst, int32_t* weight, int32_t device);

/* The edges of the stream with an endpoint in [lo, hi), in stream order, generated and
 * selected on GPU `device` (the same edges as tgo_rmat_partition, titan_gpu_olap_part.h);
 * capacity / *count / TGO_E_INVALID as there. */
int tgo_rmat_partition_device(int32_t scale, int32_t edge_factor, uint64_t seed, int64_t lo, int64_t hi,
                              int32_t* src, int32_t* dst, int32_t* weight, int64_t capacity, int64_t* count,
                              int32_t device);

/* Undirected degree (out + in) histogram helper and seeded root selection among vertices
 * of degree > 0 (Graph500 style): writes `nroots` distinct dense ids. */
int tgo_pick_roots(int64_t n, int64_t m, const int32_t* src, const int32_t* dst, uint64_t seed,
                   int32_t nroots, int64_t* roots_out);

/* Synthetic edgestore rows (the rows an ordered scan of Titan's `edgestore` returns to
 * VertexJobConverter.process, VertexJobConverter.java:109-129) for the directed edge list
 * (src, dst) of ONE MULTI edge label `label_id` (a UserEdgeLabel schema id), with the
 * Integer weight as the label's only signature property when `weight` is non-NULL.
 * Vertex i has id IDManager.constructId(i / 2^pb + 1, i % 2^pb) (round-robin partitions);
 * every row starts with VertexExists; OUT then IN entries, each sorted by (other id,
 * relation id); relation ids 1001 + i (VertexExists of i) and 1001 + n + k (edge k).
 * Output in the tgo_rows layout (titan_gpu_olap.h).  sizes_out = {nrows, nentries,
 * nbytes}; when any output array is NULL only the sizes are computed. */
int tgo_synth_rows(int64_t n, int64_t m, const int32_t* src, const int32_t* dst, const int32_t* weight,
                   int64_t label_id, int32_t partition_bits, int32_t threads, int64_t* sizes_out,
                   int64_t* row_keys, int64_t* row_entry_begin, int64_t* row_byte_begin,
                   uint8_t* entry_bytes, int64_t* entry_limit_valpos);

#ifdef __cplusplus
}
#endif
#endif

/*
 * titan_gpu_olap_part.h — multi-GPU (1-D vertex-partitioned) extension of the C-ABI.
 *
 * The reference has no multi-process OLAP executor (Fulgora is single-JVM,
 * FulgoraGraphComputer.java:117-311; cross-machine OLAP exists only as Hadoop scans,
 * hadoop/scan/HadoopScanRunner.java:63-137).  Graphs that outgrow one GPU are split over
 * the node's GPUs, one process per GPU: rank r owns global vertices [lo, hi) and holds
 * their Titan rows (OUT + IN entries, global neighbour ids).  Each superstep is a
 * local kernel plus one exchange, run by the caller with RCCL (torch.distributed, backend
 * "nccl") on the ctx stream — so the exchange buffers are caller-owned DEVICE pointers:
 *
 *   BFS bottom-up level : all-gather of the owned next-frontier bitmap slices
 *                         (nb_local, n_local/64 words each) into fb_global (n_global/64)
 *   BFS top-down level  : all-to-all of the "discovered" bitmap (disc, n_global/64 words,
 *                         slice r to rank r) into recv (nranks x n_local/64), then claim
 *   PageRank iteration  : all-gather of the owned contributions (n_local doubles), or
 *                         with tgo_part_pr_blocked two all-gathers into a hot-first layout
 *   every level         : all-reduce(SUM) of the two frontier counters
 * RCCL has no bitwise-OR reduction, hence slice exchanges instead of an all-reduce.
 *
 * Preconditions: n_local = hi - lo is a multiple of 64 (bitmap slices are whole words),
 * tgo_options.stream is the stream the caller's collectives run on.  A NULL stream makes
 * the ctx create its own stream, which the caller's collectives are NOT ordered with; the
 * entry points that leave kernels queued (bfs_td, ms_push, ms_pack, pr_begin, pr_step)
 * then finish them before returning, but inputs the caller wrote on another stream must
 * be complete before the call.  (torch's default stream has handle 0 = NULL: a torch
 * caller switches to a side stream first — titan_amd/distributed.exchange_stream.)
 */
#ifndef TITAN_GPU_OLAP_PART_H
#define TITAN_GPU_OLAP_PART_H
#include "titan_gpu_olap.h"
#ifdef __cplusplus
extern "C" {
#endif

/* Load the rows of global vertices [lo, hi) from an edge list (global ids) holding at
 * least every edge with an endpoint in [lo, hi). */
int tgo_load_partition(tgo_ctx* ctx, int64_t n_global, int64_t lo, int64_t hi,
                       const tgo_edges* edges, const tgo_load_opts* opts);

/* Device layout for the partitioned path (the multi-GPU form of the single-GPU
 * degree-grouped relabel): tgo_part_layout writes, for each owned vertex lo+v, its internal
 * global id layout_local[v] in [lo, hi) (owned vertices grouped by half-octave of degree,
 * hottest first).  The caller all-gathers the ranks' slices into layout_global (n_global
 * int32, host) and loads with tgo_load_partition_layout; every kernel then runs on internal
 * ids (hot vertices share cache lines in the gathered global vectors) while seeds and
 * outputs of the tgo_part_* calls stay in the caller's global ids / row order.  All ranks
 * must load with the same layout_global. */
int tgo_part_layout(const tgo_edges* edges, int64_t n_global, int64_t lo, int64_t hi, int32_t threads,
                    int32_t* layout_local);
int tgo_load_partition_layout(tgo_ctx* ctx, int64_t n_global, int64_t lo, int64_t hi,
                              const tgo_edges* edges, const tgo_load_opts* opts, const int32_t* layout_global);

/* counts[0] = vertices put in this rank's next frontier, counts[1] = their list entries */
int tgo_part_bfs_begin(tgo_ctx* ctx, int64_t seed_global, uint64_t* nb_local, int64_t* counts);
int tgo_part_bfs_td(tgo_ctx* ctx, int32_t level, uint64_t* disc_global);
int tgo_part_bfs_claim(tgo_ctx* ctx, int32_t level, const uint64_t* recv, int32_t nslices,
                       uint64_t* nb_local, int64_t* counts);
/* bfs_bu only counts the next frontier (nb_local); a following bfs_td queues it from
 * nb_local, which the caller must leave unchanged until then (the all-gather reads it). */
int tgo_part_bfs_bu(tgo_ctx* ctx, int32_t level, const uint64_t* fb_global, uint64_t* nb_local,
                    int64_t* counts);
/* Local distances (TGO_DIST_ABSENT = unreached) and reached[2] = {vertices, list entries}. */
int tgo_part_bfs_end(tgo_ctx* ctx, int64_t* dist_local, int64_t* reached);

/* Partitioned multi-source BFS (<= 64 seeds, global ids; bit r = seeds[r]).  Frontier
 * masks are per owned vertex (fr_local / fr_next: n_local uint64 each).  Dense level:
 * all-gather fr_local -> fr_global, then tgo_part_ms_pull.  Sparse level:
 * tgo_part_ms_push marks candidate masks of global neighbours in cand_global (n_global),
 * all-to-all of its slices into recv (nranks x n_local), then tgo_part_ms_settle. */
int tgo_part_ms_begin(tgo_ctx* ctx, const int64_t* seeds, int32_t nseeds, uint64_t* fr_local, int64_t* counts);
int tgo_part_ms_pull(tgo_ctx* ctx, int32_t level, const uint64_t* fr_global, uint64_t* fr_next, int64_t* counts);
int tgo_part_ms_push(tgo_ctx* ctx, int32_t level, const uint64_t* fr_local, uint64_t* cand_global);
int tgo_part_ms_settle(tgo_ctx* ctx, int32_t level, const uint64_t* recv, int32_t nslices, uint64_t* fr_next,
                       int64_t* counts);
/* Sparse form of the sparse-level exchange (what bench.py / distributed.py use): after
 * tgo_part_ms_push, tgo_part_ms_pack compacts the nonzero words of cand_global into
 * (owner-local id, mask) int64 pairs in `send` (device, capacity 2 * n_global int64),
 * rank-major and contiguous: send_counts[r] pairs for rank r (host), and zeroes the packed
 * words (cand_global is all-zero again afterwards).  The caller all-to-alls the counts, then
 * the pairs with split sizes (recv = the senders' pairs back to back, recv_counts[s] from
 * sender s), and tgo_part_ms_settle_pairs ORs them in.  Requires nranks * n_local ==
 * n_global.  Pair order within a rank's run is unspecified; results are not affected (the
 * masks are OR-ed). */
int tgo_part_ms_pack(tgo_ctx* ctx, uint64_t* cand_global, int32_t nranks, int64_t* send, int64_t* send_counts);
/* tgo_part_ms_pack without the host round trip: send_elems_dev (DEVICE int64[nranks])
 * receives the int64 element count per destination (2 per pair), stream-ordered, for a
 * device all-to-all of the split sizes. */
int tgo_part_ms_pack_dev(tgo_ctx* ctx, uint64_t* cand_global, int32_t nranks, int64_t* send, int64_t* send_elems_dev);
int tgo_part_ms_settle_pairs(tgo_ctx* ctx, int32_t level, const int64_t* recv, const int64_t* recv_counts,
                             int32_t nslices, uint64_t* fr_next, int64_t* counts);
/* Fixed-capacity form of the sparse exchange, for levels whose frontier is small: owner r's
 * slot of `send` is 2 * (cap + 1) int64 — a header pair (count, 0) then up to cap (owner-
 * local id, mask) pairs — so the caller's all-to-all has equal splits of 2 * (cap + 1)
 * elements known before the level (no all-to-all of split sizes, no host read of them).
 * cap must bound every owner's pair count: the level's global frontier entries (each pair
 * needs a pushed entry of this rank) capped at n_local.  A count over cap fails the sweep
 * at tgo_part_ms_end with TGO_E_STATE.  tgo_part_ms_settle_fixed ORs the received slots
 * (nslices of them, same cap) into fr_next and settles like tgo_part_ms_settle_pairs. */
int tgo_part_ms_pack_fixed(tgo_ctx* ctx, uint64_t* cand_global, int32_t nranks, int64_t cap, int64_t* send);
int tgo_part_ms_settle_fixed(tgo_ctx* ctx, int32_t level, const int64_t* recv, int32_t nslices, int64_t cap,
                             uint64_t* fr_next, int64_t* counts);
/* Source split of a dense level (tgo_bfs_multi's split, partitioned; tgo_part_msbfs_run does
 * it at the first dense level of a run of dense levels): a pull walk stops once every open
 * source is covered, and a source whose frontier barely reaches the vertex makes every walk
 * scan its whole list, so the sources with the smallest frontiers are pushed instead.
 *   tgo_part_ms_source_counts / _entries: this rank's per-source frontier sizes / exact push
 *     entries of the candidate sources `cand` into DEVICE int64[64] (the caller all-reduces);
 *   tgo_part_ms_push_masked: the `mask` sources' frontiers into cand_global (then the caller's
 *     pack + exchange, as at a sparse level, with cap = their global push entries);
 *   tgo_part_ms_or_fixed / _or_pairs: the received pairs OR-ed into fr_next (zeroed first),
 *     without settling;
 *   tgo_part_ms_pull_split: the pull for the sources outside `sparse`, OR-ing in the
 *     candidates already in fr_next when cand_in_next != 0.  Same traversal as the plain pull. */
int tgo_part_ms_source_counts(tgo_ctx* ctx, const uint64_t* fr_local, int64_t* counts_dev);
int tgo_part_ms_source_entries(tgo_ctx* ctx, const uint64_t* fr_local, uint64_t cand, int64_t* entries_dev);
int tgo_part_ms_push_masked(tgo_ctx* ctx, const uint64_t* fr_local, uint64_t* cand_global, uint64_t mask);
int tgo_part_ms_or_fixed(tgo_ctx* ctx, const int64_t* recv, int32_t nslices, int64_t cap, uint64_t* fr_next);
int tgo_part_ms_or_pairs(tgo_ctx* ctx, const int64_t* recv, const int64_t* recv_counts, int32_t nslices,
                         uint64_t* fr_next);
int tgo_part_ms_pull_split(tgo_ctx* ctx, int32_t level, const uint64_t* fr_global, uint64_t* fr_next, uint64_t sparse,
                           int32_t cand_in_next, int64_t* counts);
/* reached / entries: per seed, over this rank's vertices (NULL to skip). */
int tgo_part_ms_end(tgo_ctx* ctx, int64_t* reached, int64_t* entries);
/* Source `source`'s distances of the owned vertices (TGO_DIST_ABSENT = unreached). */
int tgo_part_ms_levels(tgo_ctx* ctx, int32_t source, int64_t* dist_local);

/* Partitioned delta-stepping SSSP (ShortestDistance converged distances over the loaded
 * scope; weights when the partition was loaded with them).  Per phase:
 *   tgo_part_sssp_relax  relaxes this rank's near queue; owned targets are updated in
 *                        place, remote ones are packed per owner into `send` (device,
 *                        capacity 2 * n_global int64: pairs {owner-local id, distance},
 *                        rank-major) with send_counts[r] pairs for rank r (host array);
 *   caller               all-to-all of the counts, then of the pairs (2 int64 each);
 *   tgo_part_sssp_apply  mins the received pairs in and builds the next near queue.
 * When every rank's near queue is empty: all-reduce(MIN) of tgo_part_sssp_pending_min's
 * out[0] (INT64_MAX = nothing pending = done), move thr to the end of that bucket, and
 * tgo_part_sssp_extract.  begin: out[0] = owned queue length, out[1] = the bucket width
 * (delta, or the default when delta <= 0; ranks should agree on the maximum).
 * counts = {next near-queue length, its push entries}.  Seeds are global ids. */
int tgo_part_sssp_begin(tgo_ctx* ctx, int64_t seed_global, int64_t delta, int64_t* out);
/* The smallest weight of this rank's load (0 without weights).  sssp_begin fails on a negative
 * weight: a driver all-reduces (MIN) this first so that every rank fails together (the native
 * tgo_part_sssp_run does). */
int tgo_part_weight_min(tgo_ctx* ctx, int64_t* min_weight);
int tgo_part_sssp_relax(tgo_ctx* ctx, int64_t thr, int32_t nranks, int64_t* send, int64_t* send_counts);
int tgo_part_sssp_apply(tgo_ctx* ctx, int64_t thr, const int64_t* recv, int64_t npairs, int64_t* counts);
int tgo_part_sssp_pending_min(tgo_ctx* ctx, int64_t* out);
int tgo_part_sssp_extract(tgo_ctx* ctx, int64_t thr, int64_t* counts);
/* Local distances (TGO_DIST_ABSENT = unreached) and reached[2] = {vertices, pull entries}. */
int tgo_part_sssp_end(tgo_ctx* ctx, int64_t* dist_local, int64_t* reached);

/* PageRankVertexProgram (PageRankVertexProgram.java:75-95) on the owned rows.
 * begin runs iteration 1 (contrib_local = (1/N) / edgeCount); every step is one rank update
 * (iterations 2..max_iterations) from the gathered contributions; end returns the owned ranks
 * (TGO_E_STATE unless exactly max_iterations - 1 steps ran: the rank property is written by
 * the last step only).  Plain layout: contrib_global = the rank-major all-gather of every
 * rank's contrib_local (n_global doubles). */
int tgo_part_pr_begin(tgo_ctx* ctx, const tgo_pr_args* args, double* contrib_local);
int tgo_part_pr_step(tgo_ctx* ctx, const double* contrib_global, double* contrib_local);
int tgo_part_pr_end(tgo_ctx* ctx, double* pr_local);
/* The fixed-point passes of the blocked layout (tgo_part_pr_blocked) are exact only inside a
 * range; a message outside it (+inf from a vertex whose row cut left it no OUT entry,
 * PageRankVertexProgram.java:80-88; NaN; a magnitude past 2^47 / longest row) sets a flag.
 * exact_check reads and clears it after end; when ANY rank reports bad = 1 every rank re-runs
 * the program with plain = 1 (the plain layout's fp64 gather, Java double sums), then sets
 * plain = 0.  tgo_part_pagerank_run does this itself. */
int tgo_part_pr_exact_check(tgo_ctx* ctx, int32_t* bad);
int tgo_part_pr_plain(tgo_ctx* ctx, int32_t on);

/* Device-resident level counts for the BFS / multi-source BFS steps: with dev_counts (a
 * device int64[3]) set, the steps that return counts write {next queue length, its push
 * entries} into [0..1] and this rank's own queue length into [2], stream-ordered, instead of
 * synchronising into the host `counts` (which may then be NULL).  The caller all-reduces
 * [0..1], reads the three values once per level and hands [2] back with
 * tgo_part_set_local_qlen, so the next step needs no read of its own.  NULL restores host
 * counts.  The SSSP steps always return host counts. */
int tgo_part_device_counts(tgo_ctx* ctx, int64_t* dev_counts);
/* The local queue length the caller read from dev_counts[2] after the last counting step. */
int tgo_part_set_local_qlen(tgo_ctx* ctx, int64_t qlen);

/* Rows of this rank holding any entry (the degree-grouped layout puts the others last). */
int tgo_part_active_rows(tgo_ctx* ctx, int64_t* n_active);

/* Cache-blocked partitioned PageRank (the one-GPU ColdBlocks over the job's sources).
 * active_span A = the maximum of every rank's tgo_part_active_rows; world = n_global/n_local.
 * *hot_per_rank = H > 0: the gathered vector is hot-first, W*A doubles —
 *     [rank 0 contrib_local[0,H)] ... [rank W-1 contrib_local[0,H)]
 *     [rank 0 contrib_local[H,A)] ... [rank W-1 contrib_local[H,A)]
 * i.e. two rank-major all-gathers (hot slices, then cold slices); rows >= A are no one's
 * source and are not exchanged.  A step may then be split so the hot all-gather overlaps
 * the cold phase: step_cold reads only the cold region of `gathered`, step_hot both.
 * *hot_per_rank = 0: blocking not applicable (bothE load, TGO_PR_BLOCKED=0, too small) —
 * keep the plain layout.  Building is host work on the downloaded in-lists (load time). */
int tgo_part_pr_blocked(tgo_ctx* ctx, int32_t world, int64_t active_span, int64_t* hot_per_rank);
int tgo_part_pr_step_cold(tgo_ctx* ctx, const double* gathered);
int tgo_part_pr_step_hot(tgo_ctx* ctx, const double* gathered, double* contrib_local);

/* The partitioned multi-source BFS sweep as ONE native call (part_driver.cpp): the protocol
 * of titan_amd/distributed.distributed_msbfs (dense level: in-place all-gather of the owned
 * frontier masks + tgo_part_ms_pull; sparse level: tgo_part_ms_push, then the fixed-capacity
 * pair exchange while world * (cap + 1) * 16 <= fixed_bytes (cap = the level's global frontier
 * entries, at most n_local), else sized pairs (one all-to-all of the split sizes, one of the
 * pairs); level counts all-reduced on the device) run as a C++ loop whose collectives go
 * through an exchange object on the ctx stream, without a Python step per level.
 *   tgo_exchange_rccl_id / _create : RCCL over xGMI (one process per GPU; rank 0 makes the
 *                                    128-byte id, the caller broadcasts it, every rank creates)
 *   tgo_exchange_local_group       : `world` ranks as threads of ONE process (tests on one
 *                                    device): collectives are device copies at a barrier; a
 *                                    rank that fails releases the others (60 s barrier limit)
 * The exchange's world / rank must match the partition (world * n_local == n_global, lo ==
 * rank * n_local).  reached / entries: per seed, global (NULL to skip); *levels = levels run.
 * The per-source levels are read with tgo_part_ms_levels afterwards, as after the Python
 * driver.  The ctx's device-counts setting (tgo_part_device_counts) is restored on return. */
typedef struct tgo_exchange tgo_exchange;
int  tgo_exchange_rccl_id(uint8_t* id_out /* 128 bytes */);
int  tgo_exchange_rccl_create(int32_t world, int32_t rank, const uint8_t* id, int32_t device, tgo_exchange** out);
int  tgo_exchange_local_group(int32_t world, tgo_exchange** ranks_out /* world handles */);
void tgo_exchange_destroy(tgo_exchange* x);
const char* tgo_exchange_last_error(const tgo_exchange* x);
int  tgo_part_msbfs_run(tgo_ctx* ctx, tgo_exchange* x, const int64_t* seeds, int32_t nseeds, int32_t max_depth,
                        double ms_alpha, int64_t fixed_bytes, int64_t* reached, int64_t* entries, int32_t* levels);

/* The other partitioned programs as ONE native call each (part_driver.cpp), same exchange
 * objects and preconditions as tgo_part_msbfs_run; outputs are host arrays, results equal the
 * Python drivers' (titan_amd/distributed.py) and the one-GPU programs':
 *   tgo_part_bfs_run      ShortestDistance with unit weights over bothE from global seed
 *                         (distributed_bfs): direction-optimizing levels (alpha / beta as
 *                         tgo_bfs), top-down = discovered-bitmap all-to-all + claim, bottom-up
 *                         = owned frontier slices all-gathered; dist_local = the owned
 *                         distances in row order (NULL to skip), reached = global {vertices,
 *                         entries} (NULL to skip), *levels = levels run.
 *   tgo_part_sssp_run     delta-stepping ShortestDistance (distributed_sssp): per phase a
 *                         relax, an all-to-all of the pair counts and an all-to-allv of the
 *                         (owner-local id, distance) pairs; an all-reduce(MIN) of the pending
 *                         minimum moves the bucket.  delta <= 0: the maximum of the ranks'
 *                         default widths.  *phases = relax phases run.
 *   tgo_part_pagerank_run PageRankVertexProgram (distributed_pagerank): layout agreed with an
 *                         all-reduce(MAX) of the active rows, tgo_part_pr_blocked, then per
 *                         update the gathered vector refreshed by exchange_mode 0 = all-gather
 *                         of every rank's slices, 1 = ghost exchange: only the contributions
 *                         this rank's in-lists read (lists built once per layout and kept with
 *                         the graph; pack -> all-to-allv -> unpack).  pr_local = owned ranks in
 *                         row order; *exchanged_bytes = bytes this rank received over the run. */
int  tgo_part_bfs_run(tgo_ctx* ctx, tgo_exchange* x, int64_t seed_global, int32_t max_depth, double alpha, double beta,
                      int64_t* dist_local, int64_t* reached, int32_t* levels);
int  tgo_part_sssp_run(tgo_ctx* ctx, tgo_exchange* x, int64_t seed_global, int64_t delta, int64_t* dist_local,
                       int64_t* reached, int32_t* phases);
int  tgo_part_pagerank_run(tgo_ctx* ctx, tgo_exchange* x, const tgo_pr_args* args, int32_t exchange_mode,
                           double* pr_local, int64_t* exchanged_bytes);

/* The partitioned load from edgestore rows: the multi-GPU form of tgo_load_rows +
 * tgo_finish_load (one scan, VertexJobConverter.java:109-129).  A Titan row holds a vertex's
 * OUT and IN entries, so the 1-D vertex partition is a row-range partition of the scan: rank r
 * of the exchange stages the rows of ITS vertices with tgo_load_rows (work blocks, local, any
 * split of the scan's rows over the ranks; edge-balanced ranges balance the work), then every
 * rank calls tgo_finish_partition_rows instead of tgo_finish_load (tgo_load_partition_rows =
 * one tgo_load_rows block + the finish; a failed stage still joins the collective).  Each rank decodes its rows with the one-GPU rules —
 * key filter, ghosts, typed scopes, and the hard-limit cut per row in column order
 * (QueryContainer.java:28,122; ColumnValueStore.java:47-69) — so its lists are exactly the
 * lists a one-GPU load keeps for those rows.  Collective (every rank calls it with the same
 * schema / opts / layout): the ranks agree on failure, the slot size S (the largest live row
 * count rounded up to 64; rank r's i-th live row is global id r * S + i, slots past its count are
 * entry-less), the global id map (all-gather of the live ids: entries to vertices no rank holds
 * are dropped, as on one GPU), the degree-grouped layout (layout = 1), and — when a cut single-
 * direction scope makes the push view no transpose of the stored lists — the push rows (every
 * rank's pull entries sent to their sources' owners).  part[0] = this rank's live rows (its
 * results are the first part[0] of the tgo_part_* outputs, in row order; tgo_vertex_ids gives
 * their ids), part[1] = S, part[2] = the live rows of every rank (the job's vertex count);
 * n_global = world * S, lo = rank * S for the tgo_part_* calls.
 * TGO_E_UNSUPPORTED for vertex cuts (they fold on one GPU) and non-Integer weight keys. */
int  tgo_finish_partition_rows(tgo_ctx* ctx, tgo_exchange* x, int32_t layout, int64_t* part);
int  tgo_load_partition_rows(tgo_ctx* ctx, tgo_exchange* x, const tgo_rows* rows, const tgo_schema* schema,
                             const tgo_load_opts* opts, int32_t layout, int64_t* part);

/* Bench / test input: the edges of an RMAT stream (tgo_synth.h) with an endpoint in
 * [lo, hi).  *count = edges written; if capacity is too small, nothing is written,
 * *count = required capacity and TGO_E_INVALID is returned. */
int tgo_rmat_partition(int32_t scale, int32_t edge_factor, uint64_t seed, int64_t lo, int64_t hi,
                       int32_t* src, int32_t* dst, int32_t* weight, int64_t capacity,
                       int64_t* count, int32_t threads);

#ifdef __cplusplus
}
#endif
#endif

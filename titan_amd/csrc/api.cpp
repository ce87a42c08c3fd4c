// api.cpp — the C-ABI (include/titan_gpu_olap.h): context, loads, program drivers.
//
// The program drivers replace FulgoraGraphComputer.submit's superstep loop
// (FulgoraGraphComputer.java:151-189): instead of one full edgestore scan per superstep,
// each iteration is one or two kernel launches over the device-resident adjacency, and
// only the frontier is touched for BFS/SSSP.
#include <algorithm>
#include <memory>
#include <numeric>
#include <atomic>
#include <chrono>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <new>
#include <thread>
#include <unordered_map>
#include <hip/hip_runtime_api.h>
#include "codec.hpp"
#include "engine.hpp"
#include "trace.hpp"
#include "../../include/titan_gpu_olap_part.h"

using namespace tgo;

struct tgo_ctx {
    tgo_options opts{};
    hipStream_t stream = nullptr;
    bool own_stream = false;
    std::string err;
    RowStaging staging;
    DevGraph g;
    bool loaded = false;
    std::vector<int64_t> titan_id;
    std::vector<int32_t> perm;                       // row-order dense -> internal
    // Titan id -> dense (seed lookups, tgo_dense_ids): binary search over titan_id when it is
    // strictly increasing (edge loads; row loads of an ordered scan usually), else over a
    // sorted copy built on the first lookup — no per-load hash map (16.8 M inserts at RMAT-24)
    bool id_sorted = false;
    std::vector<std::pair<int64_t, int32_t>> id_index;
    Scratch sc;
    tgo_stats st{};
    hipEvent_t ev0 = nullptr, ev1 = nullptr;
    int64_t dev_bytes = 0;
    std::vector<void*> allocs;
    int part_cur = 0;           // partitioned BFS: queue buffer holding the frontier
    int64_t part_qlen = 0;      // its length
    bool part_queued = true;    // q[part_cur] holds the frontier (pull / bottom-up levels only count it)
    // native multi-source sweep (part_driver.cpp): this rank's slice of the candidate words is
    // not packed but ORed in directly (tgo::part_ms_bypass); -1 = every slice packed
    int part_ms_self = -1;
    uint64_t* part_ms_cand = nullptr;
    const uint64_t* part_frontier = nullptr;   // after bottom-up: the caller's nb_local (queued lazily)
    int64_t* part_dcounts = nullptr;    // caller's device counts (tgo_part_device_counts)
    int64_t* part_qlen_dev = nullptr;   // device copy of the queue length (lazy host read)
    bool part_qlen_stale = false;       // part_qlen must be read from part_qlen_dev
    double part_alpha = 0.85, part_base = 0.0;
    int32_t part_pr_iter = 0;   // partitioned PageRank: iteration reached / program length
    int32_t part_pr_iters = 0;
    int32_t part_pr_world = 0;  // blocked gathered layout (tgo_part_pr_blocked): world, H, A
    bool part_pr_plain = false; // tgo_part_pr_plain: the plain layout although the blocked one is built
    int64_t part_pr_hot = 0, part_pr_span = 0;
    int64_t part_relaxed = 0;   // partitioned SSSP: entries relaxed, phases
    int32_t part_phases = 0;
    int64_t part_seed = -1;     // partitioned SSSP: the seed's internal id when owned here
    bool part_split = false;    // partitioned SSSP run on the light/heavy split (part_sssp_split)
    bool part_devloop = false;  // ... and on the device-sized loop (delta_loop.hip, part_sssp_dev_*)
    EdgeProg edge_prog;         // tgo_set_edge_program (TGO_EDGE_PROGRAM gathers)
    int64_t pv_max_out = 0, pv_max_in = 0;   // largest OUT / IN list of a vertex cut
    std::vector<int64_t> pv_rows;            // row ids of the vertex cuts
    // last finished program whose compute keys tgo_result_rows can encode (-1 = none)
    int res_kind = -1;
    bool host_decode = false;                // TGO_HOST_DECODE latched for the load in progress
    DecodeScratch dec;                       // device row decoder buffers (decode.hip)
    bool res_empty = false;                  // it set no property (PageRank iterations(0))
    ResultSource res_src;
    int num_cus = 256;          // compute units of the device (persistent launches)
    double ms_split = -1.0;     // tgo_set_tuning(TGO_TUNE_MS_SPLIT); < 0: TGO_MS_SPLIT / the default
    int ms_ghost = 1;           // tgo_set_tuning(TGO_TUNE_MS_GHOST): dense partitioned levels exchange ghosts
    int ds_bins = -1;           // tgo_set_tuning(TGO_TUNE_DS_BINS): 1 / 0; < 0: TGO_DS_BINS / on
    int64_t ds_pile_cap = 0;    // tgo_set_tuning(TGO_TUNE_DS_PILE_CAP): entries per pile; 0 = n
    int ds_done = -1;           // tgo_set_tuning(TGO_TUNE_DS_DONE): 1 / 0; < 0: TGO_DS_DONE / off
    double ds_pull = -1;        // tgo_set_tuning(TGO_TUNE_DS_PULL): member fraction; < 0: TGO_DS_PULL / off
    int ds_small = -1;          // tgo_set_tuning(TGO_TUNE_DS_SMALL): 1 / 0; < 0: TGO_DS_SMALL / off
    unsigned long long* part_srcent = nullptr;   // next settle's per-source sums (part_ms_settle_sums)
    bool part_count_only = false;               // next settle: no queue (part_ms_settle_sums)
    uint64_t* part_own_next = nullptr;          // next push: owned targets straight into these masks
    uint64_t* part_own_direct = nullptr;        // the last push did so (its settle skips the own OR)
    int64_t ms_cold = -1;       // tgo_set_tuning(TGO_TUNE_MS_COLD): 0 off, 1 on, > 1 on with that
                                // hot head (and segment); < 0: TGO_MS_COLD / on
    // state a native partitioned driver keeps between runs on this graph (part_driver.cpp:
    // the PageRank ghost lists); dropped with the graph
    std::shared_ptr<void> part_state;
};

namespace {

double env_double(const char* name, double dflt) {
    const char* v = std::getenv(name);
    return v ? std::atof(v) : dflt;
}

int fail(tgo_ctx* c, int code, const std::string& msg) {
    if (c) c->err = msg;
    return code;
}

#define HIP_TRY(call)                                                              \
    do {                                                                           \
        hipError_t e__ = (call);                                                   \
        if (e__ != hipSuccess)                                                     \
            return fail(ctx, e__ == hipErrorOutOfMemory ? TGO_E_OOM : TGO_E_HIP,   \
                        std::string(#call) + ": " + hipGetErrorString(e__));       \
    } while (0)

template <class T>
hipError_t dev_alloc(tgo_ctx* ctx, T*& p, int64_t count) {
    void* q = nullptr;
    const size_t bytes = static_cast<size_t>(std::max<int64_t>(count, 1)) * sizeof(T);
    hipError_t e = hipMalloc(&q, bytes);
    if (e != hipSuccess) return e;
    ctx->allocs.push_back(q);
    ctx->dev_bytes += static_cast<int64_t>(bytes);
    p = static_cast<T*>(q);
    return hipSuccess;
}

// Release one dev_alloc array of `count` elements before the graph goes (the stream is
// synchronised first: queued kernels may still use it).
template <class T>
void dev_free(tgo_ctx* ctx, T*& p, int64_t count) {
    if (!p) return;
    if (ctx->stream) (void)hipStreamSynchronize(ctx->stream);
    auto it = std::find(ctx->allocs.begin(), ctx->allocs.end(), static_cast<void*>(p));
    if (it != ctx->allocs.end()) {
        ctx->allocs.erase(it);
        ctx->dev_bytes -= static_cast<int64_t>(std::max<int64_t>(count, 1) * sizeof(T));
        (void)hipFree(p);
    }
    p = nullptr;
}

// Adopt a device array built on the device (DevArray): no copy, freed with the graph.
template <class T>
void adopt(tgo_ctx* ctx, T*& p, DevArray<T>& a) {
    p = a.p;
    if (a.p) {
        ctx->allocs.push_back(a.p);
        ctx->dev_bytes += static_cast<int64_t>(std::max<int64_t>(a.n, 1) * sizeof(T));
    }
    a.p = nullptr;
    a.n = -1;
}

template <class T>
hipError_t upload(tgo_ctx* ctx, T*& p, const std::vector<T>& h) {
    hipError_t e = dev_alloc(ctx, p, static_cast<int64_t>(h.size()));
    if (e != hipSuccess || h.empty()) return e;
    return copy_chunked(p, h.data(), h.size() * sizeof(T), hipMemcpyHostToDevice);
}

void free_graph(tgo_ctx* ctx) {
    if (ctx->stream) (void)hipStreamSynchronize(ctx->stream);
    if (ctx->sc.cub_tmp) (void)hipFree(ctx->sc.cub_tmp);       // grown by the scans, not in allocs
    if (ctx->sc.sort_tmp) (void)hipFree(ctx->sc.sort_tmp);
    for (void* p : ctx->allocs) (void)hipFree(p);
    ctx->allocs.clear();
    ctx->dev_bytes = 0;
    ctx->g = DevGraph();
    Scratch keep;                   // the mapped host counters outlive the graph (tgo_destroy frees them)
    keep.hcnt = ctx->sc.hcnt;
    keep.hcnt_dev = ctx->sc.hcnt_dev;
    keep.pub_seq = ctx->sc.pub_seq;
    ctx->sc = keep;
    ctx->loaded = false;
    ctx->res_kind = -1;         // the last program's results lived in the freed scratch
    ctx->part_state.reset();
}

int threads_of(const tgo_ctx* ctx) {
    int t = ctx->opts.host_threads;
    if (t <= 0) t = static_cast<int>(std::thread::hardware_concurrency());
    return std::max(1, std::min(t, 64));
}

// Cache-blocked PageRank in-lists (ColdBlocks, engine.hpp) for one-GPU PageRank.
// TGO_PR_BLOCKED=0 turns it off; TGO_PR_HOT / TGO_PR_SEG set the hot threshold and the cold
// segment size in sources (defaults: 384 K sources = 3 MB of fp64 messages each, under one
// XCD's 4 MB L2 so the row streams do not evict the head; swept on RMAT-24 in
// profiles/r02m_pr_probe.log and profiles/r02an_pr_hot_seg_probe*.log).
int64_t env_i64(const char* name, int64_t dflt) {
    const char* v = std::getenv(name);
    return v ? std::atoll(v) : dflt;
}
constexpr int64_t kPrSegDefault = 393216;   // 3 MB (profiles/r02an_pr_hot_seg_probe*.log)
// hot head: 3 MB for the slot tiles; 6 MB for the fixed-point super-tiles, whose source-sorted
// 380 K-entry tiles reuse lines enough that a head past one XCD's L2 still pays (RMAT-24
// ms/update: 384 K 0.852, 512 K 0.827, 768 K 0.814-0.818, 1 M 0.830, 1.5 M 0.913;
// profiles/r05j_pr_fx_hot_ab.log, r05k_pr_fx_hot_ab.log)
// The hot head (sources of the hot pass; the partitioned layout's gathered head, over every
// rank).  Round 5's source-split hot pass (TGO_PR_FX_SPLIT=2, 1 M sources, each half's 4 MB an
// XCD's L2) won with returning 128-bit LDS atomics; with the split non-returning accumulators
// the one-launch 768 K head is faster (same box, RMAT-24: split 1 M 0.897-0.902, unsplit 768 K
// 0.802-0.807, 655 K 0.806, 1 M 0.828 ms/update; profiles/r06r_*, r06s_pr_unsplit_sweep.log),
// so the split is off by default (TGO_PR_FX_SPLIT=1)
int64_t pr_fx_split_default() { return env_i64("TGO_PR_FX_SPLIT", 1); }
int64_t pr_hot_default() {
    if (env_i64("TGO_PR_FX", 1) == 0) return 393216;
    return pr_fx_split_default() > 1 ? 1048576 : 786432;
}
// LDS window of the hottest sources (lds_window, spmv.hip; TGO_PR_WIN, at most 12288 doubles =
// 96 KB beside the 16 waves' 4 KB item buffers).  Off by default: measured slower at every
// window size (negative result 13: 1.252 -> 1.385-1.476 ms/update at RMAT-24)
constexpr int64_t kPrWinDefault = 0, kPrWinMax = 12288;

// PageRank diagnostics (engine.hpp PrTuning): TGO_PR_DIAG=lo:hi gathers only sources in
// [lo, hi) — a timing attribution tool, its ranks are wrong (scripts/pr_probe.py).
PrTuning pr_tuning() {
    PrTuning t;
    if (const char* d = std::getenv("TGO_PR_DIAG")) {
        long lo = 0, hi = 0;
        if (std::sscanf(d, "%ld:%ld", &lo, &hi) == 2) { t.diag_lo = static_cast<int32_t>(lo); t.diag_hi = static_cast<int32_t>(hi); }
    }
    return t;
}

// CSR-adaptive row blocks of one CSR; `pack` (optional) source-sorts and packs the CSR's
// tiles first (spmv.hip gather_short_packed).
hipError_t upload_row_blocks(tgo_ctx* ctx, const std::vector<int64_t>& off, RowBlocks& rb,
                             std::vector<int32_t>* pack = nullptr, bool* packed = nullptr, int64_t tile = kTile,
                             int shift = kPackShift) {
    std::vector<int64_t> blk, crow, cbeg, cend, lrow, lch;
    build_row_blocks(off, tile, kMaxRows, blk, crow, cbeg, cend, lrow, lch);
    if (pack) *packed = pack_tiles(off, *pack, blk, cbeg, cend, tile, threads_of(ctx), shift);
    rb.nblocks = static_cast<int64_t>(blk.size()) - 1;
    rb.nchunks = static_cast<int64_t>(crow.size());
    rb.nlong = static_cast<int64_t>(lrow.size());
    hipError_t e;
    if ((e = upload(ctx, rb.blk, blk)) != hipSuccess) return e;
    if ((e = upload(ctx, rb.chunk_row, crow)) != hipSuccess) return e;
    if ((e = upload(ctx, rb.chunk_beg, cbeg)) != hipSuccess) return e;
    if ((e = upload(ctx, rb.chunk_end, cend)) != hipSuccess) return e;
    if ((e = upload(ctx, rb.long_row, lrow)) != hipSuccess) return e;
    if ((e = upload(ctx, rb.long_chunk, lch)) != hipSuccess) return e;
    std::vector<int64_t> desc(2 * blk.size());
    for (size_t b = 0; b < blk.size(); ++b) { desc[2 * b] = blk[b]; desc[2 * b + 1] = off[blk[b]]; }
    if ((e = upload(ctx, rb.bdesc, desc)) != hipSuccess) return e;
    return hipSuccess;
}

// upload_row_blocks with the tiles packed on the device, in place in d_adj (pr_layout.hip):
// the same blocks (built on the host from the offsets) and the same packed words.  *packed =
// false (d_adj untouched) when a source is too wide for the slot space (pack_tiles' rule).
int upload_row_blocks_dev(tgo_ctx* ctx, const std::vector<int64_t>& off, RowBlocks& rb, int32_t* d_adj,
                          int32_t max_src, bool* packed, int64_t tile, int shift, int64_t max_rows = kMaxRows) {
    std::vector<int64_t> blk, crow, cbeg, cend, lrow, lch;
    build_row_blocks(off, tile, max_rows, blk, crow, cbeg, cend, lrow, lch);
    *packed = false;
    const int64_t src_limit = shift == kPackShift ? (int64_t(1) << (31 - shift)) : (int64_t(1) << (32 - shift));
    if (d_adj && shift >= 1 && shift <= 20 && tile <= (int64_t(1) << shift) && max_src < src_limit) {
        // tiles in entry order: short blocks, and the chunks of each long row (they cover it)
        std::vector<std::pair<int64_t, int64_t>> t;
        for (size_t b = 0; b + 1 < blk.size(); ++b) {
            const int64_t s0 = off[blk[b]], s1 = off[blk[b + 1]];
            if (s1 - s0 <= tile) t.emplace_back(s0, s1);
        }
        for (size_t c = 0; c < cbeg.size(); ++c) t.emplace_back(cbeg[c], cend[c]);
        std::sort(t.begin(), t.end());
        std::vector<int64_t> ts(t.size());
        for (size_t i = 0; i < t.size(); ++i) ts[i] = t[i].first;
        std::string err;
        if (int rc = pack_tiles_device(d_adj, off.back(), ts, nullptr, shift, ctx->stream, err)) return fail(ctx, rc, err);
        *packed = true;
    }
    rb.nblocks = static_cast<int64_t>(blk.size()) - 1;
    rb.nchunks = static_cast<int64_t>(crow.size());
    rb.nlong = static_cast<int64_t>(lrow.size());
    HIP_TRY(upload(ctx, rb.blk, blk));
    HIP_TRY(upload(ctx, rb.chunk_row, crow));
    HIP_TRY(upload(ctx, rb.chunk_beg, cbeg));
    HIP_TRY(upload(ctx, rb.chunk_end, cend));
    HIP_TRY(upload(ctx, rb.long_row, lrow));
    HIP_TRY(upload(ctx, rb.long_chunk, lch));
    std::vector<int64_t> desc(2 * blk.size());
    for (size_t b = 0; b < blk.size(); ++b) { desc[2 * b] = blk[b]; desc[2 * b + 1] = off[blk[b]]; }
    HIP_TRY(upload(ctx, rb.bdesc, desc));
    return TGO_OK;
}

// Biased-exponent range [elo, ehi) in which the fixed-point PageRank sums are exact (spmv.hip
// kFxPoint): |v| >= 2^-53 (the 2^-80 resolution then costs < 2^-27 of a value), a row of
// max_len entries below 2^47 (|v| < 2^(47 - c) with 2^c >= max_len), and a tile's split H words
// (X >> 40, summed over at most min(max_len, kFxTileMax) entries of a row) below 2^63:
// |v| < 2^(23 - min(c, 22)); and |v| < 2^11 for the entry conversion (spmv.hip fx_hl).
constexpr int64_t kFxTileMax = int64_t(1) << 22;      // entries of a fixed-point tile / cold block
void fx_range(int64_t max_len, int& elo, int& ehi) {
    int c = 0;
    while ((int64_t(1) << c) < max_len && c < 47) ++c;
    elo = 1023 - 53;
    ehi = std::min({1023 + 47 - c, 1023 + 23 - std::min(c, 22), 1023 + 11});
}

// Cache-blocked PageRank in-lists of the rows [0, n_rows) (rows past n_rows have no entries)
// over sources [0, n_src): built on the device from the uploaded in-lists (d_off / d_adj,
// pr_layout.hip) unless TGO_HOST_ASSEMBLY=1 (or a row is not sorted by source), then on the
// host; uploaded into cb.
int upload_cold_blocks(tgo_ctx* ctx, const std::vector<int64_t>& off, const std::vector<int32_t>& adj,
                       int64_t n_src, int64_t hot, int64_t n_rows, ColdBlocks& cb, bool& ready,
                       const int64_t* d_off = nullptr, const int32_t* d_adj = nullptr, int64_t d_nnz = 0,
                       int64_t win = 0) {
    cb = ColdBlocks();
    ready = false;
    HostColdBlocks hc;
    static const bool trace = env_i64("TGO_TRACE", 0) != 0;
    auto t_last = std::chrono::steady_clock::now();
    auto lap = [&](const char* what) {
        if (!trace && !tracing()) return;
        const auto now = std::chrono::steady_clock::now();
        const double ms = std::chrono::duration<double, std::milli>(now - t_last).count();
        if (trace) std::fprintf(stderr, "[tgo]   cold %-18s %8.1f ms\n", what, ms);
        trace_complete(std::string("pagerank_layout.") + what, ms * 1e3);
        t_last = now;
    };
    bool on_dev = false;
    win = std::min<int64_t>(win, kPrWinMax);        // the window and the waves' item buffers share 160 KB of LDS
    // TGO_PR_FX_COLD (default on): fixed-point cold blocks (spmv.hip cold_fx) of up to 4096
    // pieces and TGO_PR_FX_CE entries
    const bool cold_fx = env_i64("TGO_PR_FX", 1) != 0 && env_i64("TGO_PR_FX_COLD", 1) != 0 && win == 0;
    if (d_off && d_adj && env_i64("TGO_HOST_ASSEMBLY", 0) == 0) {
        std::string err;
        if (int rc = build_cold_blocks_device(d_off, d_adj, static_cast<int64_t>(off.size()) - 1, d_nnz, n_src, hot,
                                              env_i64("TGO_PR_SEG", kPrSegDefault),
                                              cold_fx ? std::min(kFxTileMax, env_i64("TGO_PR_FX_CE", 65536)) : kTile,
                                              cold_fx ? std::min<int64_t>(env_i64("TGO_PR_FX_CP", 4096), int64_t(1) << (kPackShift + 1))
                                                      : kMaxRows,
                                              env_i64("TGO_PR_CPACK", 1) != 0, hc, on_dev, ctx->stream, err, win, cold_fx))
            return fail(ctx, rc, err);
        if (on_dev) lap("build (device)");
    }
    std::vector<int32_t> adj_dl;        // host copy of a device-resident list, for the host build
    if (!on_dev && d_adj && static_cast<int64_t>(adj.size()) != d_nnz) {
        adj_dl.resize(static_cast<size_t>(d_nnz));
        HIP_TRY(copy_chunked(adj_dl.data(), d_adj, static_cast<size_t>(d_nnz) * sizeof(int32_t), hipMemcpyDeviceToHost));
    }
    if (!on_dev) {
        if (!build_cold_blocks(off, adj_dl.empty() ? adj : adj_dl, n_src, hot, env_i64("TGO_PR_SEG", kPrSegDefault), kTile, kMaxRows,
                               threads_of(ctx), env_i64("TGO_PR_CPACK", 1) != 0, hc, win))
            return TGO_OK;                                // too small to block: plain gather
        lap("build (host)");
    }
    cb.hot = hc.hot;
    cb.seg = hc.seg;
    cb.npieces = static_cast<int64_t>(hc.cpid.size());
    cb.nblocks = static_cast<int64_t>(hc.bbeg.size());
    cb.max_xcd_blocks = hc.max_xcd_blocks;
    cb.xbase = hc.xbase;
    cb.n_rows = n_rows;
    const std::vector<int64_t> hoff_act(hc.hoff.begin(), hc.hoff.begin() + n_rows + 1);
    // hot tiles: 4096 entries (256 threads, 32 KB of LDS), 8192 (512 threads, 64 KB) or 16384
    // (1024 threads, 128 KB): a larger tile shares more 128-byte lines between the lanes of one
    // gather instruction (fewer L2 requests per entry) at fewer workgroups per CU
    const int64_t ht = env_i64("TGO_PR_HOT_TILE", 4096);
    cb.hot_tile = ht == 16384 ? 16384 : ht == 8192 ? 8192 : 4096;
    cb.hot_shift = cb.hot_tile == 16384 ? 14 : cb.hot_tile == 8192 ? 13 : kPackShift;
    cb.hot_pipe = static_cast<int>(env_i64("TGO_PR_HOT_PIPE", 0));
    cb.num_cus = ctx->num_cus;
    const bool pack = env_i64("TGO_PR_PACK", 1) != 0;
    if (!pack) cb.hot_tile = static_cast<int>(kTile), cb.hot_shift = kPackShift;
    // Fixed-point hot pass (TGO_PR_FX, default on; spmv.hip gather_hot_fx): super-tiles of
    // TGO_PR_FX_E entries, built on the device from the hot CSR (its sources must leave at least
    // 6 bits of the packed word for the row)
    if (on_dev && pack && env_i64("TGO_PR_FX", 1) != 0) {
        const int64_t hmax = std::min<int64_t>(hot, n_src);
        int sb = 1;
        while ((int64_t(1) << sb) < hmax) ++sb;         // sources < 2^sb
        // rows per super-tile: 2^12 (64 KB of LDS accumulators), or 2^13 with TGO_PR_FX_HROWS=8192
        // when the hot sources leave 13 bits of the packed word (hot <= 512 K)
        const int want_rbits = env_i64("TGO_PR_FX_HROWS", 4096) == 8192 ? 13 : 12;
        const int rbits = std::min(want_rbits, 32 - sb);
        if (rbits >= 6) {
            cb.hcsr.nnz = hc.d_hadj.n;
            adopt(ctx, cb.hcsr.adj, hc.d_hadj);
            HIP_TRY(upload(ctx, cb.hcsr.off, hc.hoff));
            std::vector<int64_t> tdesc, long_len;
            std::vector<int32_t> long_rows;
            std::string err;
            // entries per super-tile: larger tiles share more lines; about one tile a CU (hot
            // entries / 256, at most 1 M) — with the split accumulators and the one-launch head,
            // RMAT-24 (768 K head): 262 K 0.848, 430 K 0.802, 860 K 0.779, 1 M 0.772-0.786, 1.3 M
            // 0.832, 2 M 0.97 ms/update (profiles/r06t_pr_tile_entries_sweep.log, r06u_*); round 5
            // with returning atomics measured 512 K best (r05e_pr_fx_probe.log)
            const int64_t fx_e = std::min(kFxTileMax, env_i64("TGO_PR_FX_E", std::min<int64_t>(int64_t(1) << 20,
                                                                          std::max<int64_t>(int64_t(1) << 16, hc.hoff[n_rows] / 256))));
            if (int rc = pack_supertiles_device(cb.hcsr.adj, cb.hcsr.off, hc.hoff, n_rows, fx_e,
                                                rbits, tdesc, long_rows, long_len, ctx->stream, err))
                return fail(ctx, rc, err);
            cb.fx = true;
            cb.fx_rbits = rbits;
            cb.fx_ntiles = static_cast<int64_t>(tdesc.size() / 4);
            cb.fx_nlong = static_cast<int64_t>(long_rows.size());
            HIP_TRY(upload(ctx, cb.fx_desc, tdesc));
            HIP_TRY(upload(ctx, cb.fx_long_row, long_rows));
            HIP_TRY(dev_alloc(ctx, cb.fx_long_acc, 2 * std::max<int64_t>(cb.fx_nlong, 1)));
            HIP_TRY(hipMemset(cb.fx_long_acc, 0, 2 * std::max<int64_t>(cb.fx_nlong, 1) * sizeof(unsigned long long)));
            // TGO_PR_FX_SPLIT=S > 1: the hot pass in S launches over S ranges of the hot sources
            // (each range's messages fit an XCD's L2: 3 MB a half at 768 K hot sources)
            const int64_t split = std::min<int64_t>(8, std::max<int64_t>(1, pr_fx_split_default()));
            if (split > 1 && cb.fx_ntiles > 0) {
                HIP_TRY(dev_alloc(ctx, cb.fx_mid, cb.fx_ntiles * (split + 1)));
                HIP_TRY(dev_alloc(ctx, cb.fx_part, 2 * std::max<int64_t>(n_rows, 1)));
                const int64_t first = std::min<int64_t>(hmax, std::max<int64_t>(0, env_i64("TGO_PR_FX_SPLIT_AT", 0)));
                HIP_TRY(k_fx_split_points(reinterpret_cast<const uint32_t*>(cb.hcsr.adj), cb.fx_desc, cb.fx_ntiles, rbits,
                                          hmax, static_cast<int>(split), first, cb.fx_mid, ctx->stream));
                cb.fx_split = static_cast<int>(split);
            }
            lap("hot super-tiles");
        }
    }
    if (cb.fx) {
        // hot CSR adopted and packed above
    } else if (on_dev) {                            // hot tiles packed on the device
        cb.hcsr.nnz = hc.d_hadj.n;
        adopt(ctx, cb.hcsr.adj, hc.d_hadj);
        const int32_t max_src = static_cast<int32_t>(std::min<int64_t>(hot, n_src) - 1);
        if (int rc = upload_row_blocks_dev(ctx, hoff_act, cb.rb_hot, pack ? cb.hcsr.adj : nullptr, max_src, &cb.packed,
                                           cb.hot_tile, cb.hot_shift))
            return rc;
        if (pack && !cb.packed && cb.hot_tile != kTile) {
            cb.hot_tile = static_cast<int>(kTile);
            cb.hot_shift = kPackShift;
            cb.rb_hot = RowBlocks();
            if (int rc = upload_row_blocks_dev(ctx, hoff_act, cb.rb_hot, cb.hcsr.adj, max_src, &cb.packed, kTile,
                                               kPackShift))
                return rc;
        }
    } else {
        HIP_TRY(upload_row_blocks(ctx, hoff_act, cb.rb_hot, pack ? &hc.hadj : nullptr, &cb.packed, cb.hot_tile,
                                  cb.hot_shift));
        if (!cb.packed && cb.hot_tile != kTile) {  // sources too wide for the slot space: the 4096 form
            cb.hot_tile = static_cast<int>(kTile);
            cb.hot_shift = kPackShift;
            cb.rb_hot = RowBlocks();
            HIP_TRY(upload_row_blocks(ctx, hoff_act, cb.rb_hot, pack ? &hc.hadj : nullptr, &cb.packed));
        }
        HIP_TRY(upload(ctx, cb.hcsr.adj, hc.hadj));
        cb.hcsr.nnz = static_cast<int64_t>(hc.hadj.size());
    }
    lap("hot row blocks+pack");
    if (hc.win > 0) {                               // LDS window CSR: blocks over the active rows
        const std::vector<int64_t> woff_act(hc.woff.begin(), hc.woff.begin() + n_rows + 1);
        bool unused = false;
        // wave items of the window pass (lds_window): <= 512 entries, <= 64 rows
        if (int rc = upload_row_blocks_dev(ctx, woff_act, cb.rb_win, nullptr, 0, &unused, 512, kPackShift, 64)) return rc;
        HIP_TRY(upload(ctx, cb.woff, woff_act));
        if (hc.d_widx.present()) adopt(ctx, cb.widx, hc.d_widx);
        else HIP_TRY(upload(ctx, cb.widx, hc.widx));
        cb.win = hc.win;
    }
    if (!cb.fx) HIP_TRY(upload(ctx, cb.hcsr.off, hc.hoff));
    HIP_TRY(upload(ctx, cb.poff, hc.poff));
    if (hc.d_cadj.present()) adopt(ctx, cb.cadj, hc.d_cadj);
    else HIP_TRY(upload(ctx, cb.cadj, hc.cadj));
    HIP_TRY(upload(ctx, cb.cptr, hc.cptr));
    HIP_TRY(upload(ctx, cb.cpid, hc.cpid));
    HIP_TRY(upload(ctx, cb.bbeg, hc.bbeg));
    HIP_TRY(upload(ctx, cb.bend, hc.bend));
    HIP_TRY(upload(ctx, cb.xblk, hc.xblk));
    HIP_TRY(upload(ctx, cb.bsrc, hc.bsrc));
    if (hc.cfx) {                                   // cold_fx descriptors, launch-slot order
        std::vector<int64_t> desc(4 * hc.xblk.size());
        for (size_t j = 0; j < hc.xblk.size(); ++j) {
            const int32_t b = hc.xblk[j];
            const int64_t p0 = hc.bbeg[b], p1 = hc.bend[b];
            const int64_t src = hc.bsrc[b];
            if (p1 - p0 > (int64_t(1) << hc.cfx_shift) || src < 0) return fail(ctx, TGO_E_STATE, "cold block descriptor out of range");
            desc[4 * j] = hc.poff[p0]; desc[4 * j + 1] = hc.poff[p1]; desc[4 * j + 2] = p0;
            desc[4 * j + 3] = (src << 16) | (p1 - p0);
        }
        HIP_TRY(upload(ctx, cb.cfx_desc, desc));
        cb.cfx = true;
        cb.cfx_shift = hc.cfx_shift;
    } else {
        std::vector<int64_t> desc(4 * hc.xblk.size());
        for (size_t j = 0; j < hc.xblk.size(); ++j) {
            const int32_t b = hc.xblk[j];
            const int64_t p0 = hc.bbeg[b], p1 = hc.bend[b], s0 = hc.poff[p0], nnz = hc.poff[p1] - s0;
            const int64_t src = hc.bsrc.empty() ? 0 : hc.bsrc[b];
            if (nnz > kTile || src < 0) return fail(ctx, TGO_E_STATE, "cold block descriptor out of range");
            desc[4 * j] = p0; desc[4 * j + 1] = p1; desc[4 * j + 2] = s0; desc[4 * j + 3] = (src << 16) | nnz;
        }
        HIP_TRY(upload(ctx, cb.cdesc, desc));
    }
    cb.cpacked = hc.cpacked;
    HIP_TRY(dev_alloc(ctx, cb.partial, cb.npieces));
    HIP_TRY(dev_alloc(ctx, cb.csum, std::max<int64_t>(cb.n_rows, 1)));
    HIP_TRY(hipMemset(cb.csum, 0, std::max<int64_t>(cb.n_rows, 1) * sizeof(double)));
    cb.n_crows = static_cast<int64_t>(hc.crow.size());
    HIP_TRY(upload(ctx, cb.crow, hc.crow));
    if (cb.fx || cb.cfx) {                          // the fixed-point passes' range flag (FxGuard)
        int64_t max_len = 0;
        for (size_t r = 0; r + 1 < off.size(); ++r) max_len = std::max(max_len, off[r + 1] - off[r]);
        fx_range(max_len, cb.fx_elo, cb.fx_ehi);
        HIP_TRY(dev_alloc(ctx, cb.fx_bad, 1));
        HIP_TRY(hipMemset(cb.fx_bad, 0, sizeof(unsigned)));
    }
    lap("uploads");
    ready = true;
    return TGO_OK;
}

// After a program's updates: did any fixed-point pass see a message outside its exact range?
// Clears the flag.  (A synchronising read, once per program.)
int fx_take_bad(tgo_ctx* ctx, ColdBlocks& cb, bool* bad) {
    *bad = false;
    if (!cb.fx_bad) return TGO_OK;
    unsigned h = 0;
    HIP_TRY(hipMemcpyAsync(&h, cb.fx_bad, sizeof(unsigned), hipMemcpyDeviceToHost, ctx->stream));
    HIP_TRY(hipStreamSynchronize(ctx->stream));
    if (h) {
        HIP_TRY(hipMemsetAsync(cb.fx_bad, 0, sizeof(unsigned), ctx->stream));
        // a long row's accumulators may hold the discarded run's chunks: back to zero
        if (cb.fx_long_acc)
            HIP_TRY(hipMemsetAsync(cb.fx_long_acc, 0, 2 * std::max<int64_t>(cb.fx_nlong, 1) * sizeof(unsigned long long),
                                   ctx->stream));
        *bad = true;
    }
    return TGO_OK;
}

int upload_graph(tgo_ctx* ctx, HostGraph& h, bool allow_segments = true) {
    DevGraph& g = ctx->g;
    // TGO_TRACE=1: per-phase load times on stderr
    static const bool trace = env_i64("TGO_TRACE", 0) != 0;
    auto t_last = std::chrono::steady_clock::now();
    auto lap = [&](const char* what) {
        if (!trace && !tracing()) return;
        const auto now = std::chrono::steady_clock::now();
        const double ms = std::chrono::duration<double, std::milli>(now - t_last).count();
        if (trace) std::fprintf(stderr, "[tgo] upload %-14s %8.1f ms\n", what, ms);
        trace_complete(std::string("upload.") + what, ms * 1e3);
        t_last = now;
    };
    g.n = h.n;
    g.scope = h.scope;
    g.has_weight = h.has_weight;
    g.weight_dt = h.weight_dt;
    g.has_col = h.out.has_col() || h.in.has_col();
    g.has_transpose = h.has_transpose;
    g.n_active = 0;
    for (int64_t v = h.n - 1; v >= 0; --v)
        if (h.out.off[v + 1] > h.out.off[v] || h.in.off[v + 1] > h.in.off[v]) { g.n_active = v + 1; break; }
    g.min_weight = 0;
    g.max_weight = 0;
    double wsum = 0.0;
    int64_t wcnt = 0;
    const bool wide = h.has_weight && wide_weight_dt(h.weight_dt);   // the column holds value-table indices
    for (const HostCsr* c : {&h.out, &h.in})
        for (int32_t x : c->w)
            if (x != kMissingWeight && !wide) {
                g.min_weight = std::min(g.min_weight, x);
                g.max_weight = std::max(g.max_weight, x);
                wsum += x;
                ++wcnt;
            }
    g.mean_weight = wcnt ? wsum / static_cast<double>(wcnt) : 1.0;
    auto up = [&](HostCsr& src, DevCsr& dst) -> hipError_t {
        hipError_t e;
        dst.nnz = src.nnz();
        if ((e = upload(ctx, dst.off, src.off)) != hipSuccess) return e;
        // lists assembled on the device stay there (adopted); host-assembled ones are copied
        if (src.dadj.present()) adopt(ctx, dst.adj, src.dadj);
        else if ((e = upload(ctx, dst.adj, src.adj)) != hipSuccess) return e;
        if (h.has_weight) {
            if (src.dw.present()) adopt(ctx, dst.w, src.dw);
            else if ((e = upload(ctx, dst.w, src.w)) != hipSuccess) return e;
        }
        if (src.dcol.present()) adopt(ctx, dst.col, src.dcol);
        else if (!src.col.empty() && (e = upload(ctx, dst.col, src.col)) != hipSuccess) return e;
        return hipSuccess;
    };
    HIP_TRY(up(h.out, g.out));
    HIP_TRY(up(h.in, g.in));
    if (h.has_transpose) HIP_TRY(up(h.push_t, g.push_t));
    g.wval = nullptr;
    if (wide) {
        const int64_t nv = h.d_wval.present() ? h.d_wval.n : static_cast<int64_t>(h.wval.size());
        if (nv == 0 && (g.out.nnz > 0 || g.in.nnz > 0)) return fail(ctx, TGO_E_STATE, "wide weights: the value table is missing");
        if (h.d_wval.present()) adopt(ctx, g.wval, h.d_wval);
        else HIP_TRY(upload(ctx, g.wval, h.wval));
    }
    lap("csr");
    // CSR-adaptive blocks for the two pull gathers (walk counts: out; PageRank: in).
    HIP_TRY(upload_row_blocks(ctx, h.out.off, g.rb_out));
    HIP_TRY(upload_row_blocks(ctx, h.in.off, g.rb_in));
    g.rb_out_ready = g.rb_in_ready = true;
    lap("row blocks");
    g.push_ws = DevCsr();
    g.push_ws_ready = false;
    if (allow_segments && h.has_weight && !wide && env_i64("TGO_DS_SPLIT", 1) != 0) {
        HostCsr ws;                      // light/heavy delta-stepping: push entries sorted by weight
        weight_sorted_push(h, ws, threads_of(ctx));
        HIP_TRY(up(ws, g.push_ws));
        g.push_ws_ready = true;
        lap("weight-sorted");
    }
    g.cold_in = ColdBlocks();
    g.cold_in_ready = false;
    if (allow_segments && h.scope != TGO_SCOPE_BOTH_E && env_i64("TGO_PR_BLOCKED", 1) != 0) {
        // rows >= n_active have no entries at all: the hot pass skips them (their rank
        // after any update is (1-a)/N, written once at the end of the program)
        if (int rc = upload_cold_blocks(ctx, h.in.off, h.in.adj, h.n, env_i64("TGO_PR_HOT", pr_hot_default()), g.n_active,
                                        g.cold_in, g.cold_in_ready, g.in.off, g.in.adj, g.in.nnz,
                                        env_i64("TGO_PR_WIN", kPrWinDefault)))
            return rc;
        lap("cold blocks");
    }
    // scratch
    Scratch& s = ctx->sc;
    const int64_t n = h.n, words = (n + 63) / 64 + 1;
    s.n = n;
    HIP_TRY(dev_alloc(ctx, s.level, n));
    HIP_TRY(dev_alloc(ctx, s.q[0], n + 1));
    HIP_TRY(dev_alloc(ctx, s.q[1], n + 1));
    HIP_TRY(dev_alloc(ctx, s.qdeg, n + 2));
    HIP_TRY(dev_alloc(ctx, s.qpre, n + 2));
    HIP_TRY(dev_alloc(ctx, s.fb, words));
    HIP_TRY(dev_alloc(ctx, s.nb, words));
    HIP_TRY(dev_alloc(ctx, s.vb, words));
    HIP_TRY(dev_alloc(ctx, s.dist, n));
    HIP_TRY(dev_alloc(ctx, s.msg, n));
    for (int i = 0; i < 3; ++i) HIP_TRY(dev_alloc(ctx, s.vec[i], n));
    s.partial_cap = std::max<int64_t>({g.rb_out.nchunks, g.rb_in.nchunks, g.cold_in.rb_hot.nchunks, 1});
    HIP_TRY(dev_alloc(ctx, s.partial, s.partial_cap));
    HIP_TRY(dev_alloc(ctx, s.cnt, 1));
    if (!s.hcnt) {
        void* hp = nullptr;
        // fine-grained: the publish kernel's system-scope stores reach the spinning host
        HIP_TRY(hipHostMalloc(&hp, sizeof(Counters) + 64, hipHostMallocMapped | hipHostMallocCoherent));
        std::memset(hp, 0, sizeof(Counters) + 64);
        s.hcnt = static_cast<Counters*>(hp);
        void* dp = nullptr;
        HIP_TRY(hipHostGetDevicePointer(&dp, hp, 0));
        s.hcnt_dev = static_cast<unsigned long long*>(dp);
        s.pub_seq = 0;
    }
    HIP_TRY(hipDeviceSynchronize());
    // the host graph is dropped after the upload: its id and perm vectors move (1.5 GB at 2^27)
    ctx->titan_id = std::move(h.titan_id);
    ctx->perm = std::move(h.perm);
    if (ctx->perm.empty()) { ctx->perm.resize(n); for (int64_t v = 0; v < n; ++v) ctx->perm[v] = static_cast<int32_t>(v); }
    HIP_TRY(upload(ctx, g.perm, ctx->perm));
    ctx->id_index.clear();
    ctx->id_sorted = true;
    if (!h.ids_sorted)
        for (int64_t v = 1; v < n && ctx->id_sorted; ++v) ctx->id_sorted = ctx->titan_id[v] > ctx->titan_id[v - 1];
    ctx->st.num_vertices = n;
    ctx->st.out_entries = g.out.nnz;       // (the device lists were adopted: h's are empty)
    ctx->st.in_entries = g.in.nnz;
    ctx->st.ghost_vertices = h.ghost;
    ctx->st.truncated_results = h.truncated;
    ctx->st.skipped_rows = h.skipped;
    ctx->st.partitioned_vertices = h.partitioned;
    ctx->st.partition_rows = h.partition_rows;
    ctx->st.ghost_partition_rows = h.ghost_partition_rows;
    ctx->pv_max_out = h.pv_max_out;
    ctx->pv_max_in = h.pv_max_in;
    ctx->pv_rows.clear();
    for (size_t r = 0; r < h.pv_flags.size(); ++r)
        if (h.pv_flags[r]) ctx->pv_rows.push_back(static_cast<int64_t>(r));
    ctx->st.device_bytes = ctx->dev_bytes;
    ctx->loaded = true;
    lap("scratch, ids");
    return TGO_OK;
}

// Views of the loaded scope.
View make_view(const DevCsr* a, const DevCsr* b) {
    View v{};
    v.off0 = a->off; v.adj0 = a->adj; v.w0 = a->w;
    if (b) { v.off1 = b->off; v.adj1 = b->adj; v.w1 = b->w; v.nlists = 2; }
    else { v.off1 = a->off; v.adj1 = a->adj; v.w1 = a->w; v.nlists = 1; }
    return v;
}
View pull_view(const DevGraph& g, int scope) {
    if (scope == TGO_SCOPE_IN_E) return make_view(&g.out, nullptr);
    if (scope == TGO_SCOPE_OUT_E) return make_view(&g.in, nullptr);
    return make_view(&g.out, &g.in);
}
View push_view(const DevGraph& g, int scope) {
    if (g.has_transpose) return make_view(&g.push_t, nullptr);
    if (scope == TGO_SCOPE_IN_E) return make_view(&g.in, nullptr);
    if (scope == TGO_SCOPE_OUT_E) return make_view(&g.out, nullptr);
    return make_view(&g.out, &g.in);
}

// Row-order dense index of a Titan id, -1 when no executed vertex has it.
int64_t dense_of(tgo_ctx* ctx, int64_t id) {
    const std::vector<int64_t>& t = ctx->titan_id;
    if (ctx->id_sorted) {
        const auto it = std::lower_bound(t.begin(), t.end(), id);
        return it != t.end() && *it == id ? static_cast<int64_t>(it - t.begin()) : -1;
    }
    if (ctx->id_index.size() != t.size()) {
        ctx->id_index.resize(t.size());
        for (size_t v = 0; v < t.size(); ++v) ctx->id_index[v] = {t[v], static_cast<int32_t>(v)};
        std::sort(ctx->id_index.begin(), ctx->id_index.end());
    }
    const auto it = std::lower_bound(ctx->id_index.begin(), ctx->id_index.end(), std::make_pair(id, INT32_MIN));
    return it != ctx->id_index.end() && it->first == id ? it->second : -1;
}

int resolve_seed(tgo_ctx* ctx, int64_t seed, int is_dense, int64_t& out) {
    if (is_dense) {
        if (seed < 0 || seed >= ctx->g.n) return fail(ctx, TGO_E_INVALID, "dense seed out of range");
        out = ctx->perm[seed];
        return TGO_OK;
    }
    const int64_t d = dense_of(ctx, seed);
    out = d < 0 ? -1 : ctx->perm[d];                                 // unknown seed: nobody gets a distance
    return TGO_OK;
}

int check_program(tgo_ctx* ctx, int scope) {
    if (!ctx->loaded) return fail(ctx, TGO_E_STATE, "no graph loaded");
    if (scope < 0 || scope > 2) return fail(ctx, TGO_E_INVALID, "invalid scope");
    if (scope != ctx->g.scope)
        return fail(ctx, TGO_E_INVALID, "program scope differs from the scope the graph was loaded (preloaded) for");
    return TGO_OK;
}

// Counters of the work queued so far, without a copy + stream synchronisation: the publish
// kernel stores them and then a sequence number into host-mapped memory; the host spins on
// the sequence number (the level loops read a few words per level, so the wake-up latency of
// a blocking synchronisation dominated short levels).  A stream error ends the spin.
int wait_publish(tgo_ctx* ctx, unsigned long long seq);

int read_counters(tgo_ctx* ctx) {
    Scratch& s = ctx->sc;
    const unsigned long long seq = ++s.pub_seq;
    HIP_TRY(k_publish_counters(s.cnt, s.hcnt_dev, seq, ctx->stream));
    return wait_publish(ctx, seq);
}

// Spin on the publish sequence number (a periodic stream query ends the spin on a failure).
int wait_publish(tgo_ctx* ctx, unsigned long long seq) {
    Scratch& s = ctx->sc;
    const volatile unsigned long long* flag = reinterpret_cast<volatile unsigned long long*>(s.hcnt) + kCounterWords;
    for (uint64_t it = 1;; ++it) {
        if (*flag == seq) break;
        if ((it & 0x3FFF) == 0) {
            const hipError_t q = hipStreamQuery(ctx->stream);
            if (q != hipSuccess && q != hipErrorNotReady) return fail(ctx, TGO_E_HIP, hipGetErrorString(q));
            if (q == hipSuccess && *flag != seq) return fail(ctx, TGO_E_HIP, "counter publish not visible after the stream drained");
        }
        __builtin_ia32_pause();
    }
    std::atomic_thread_fence(std::memory_order_acquire);
    return TGO_OK;
}

// wait_publish for a publish that later ones may have overwritten: spin until the sequence
// word reaches seq (the words then hold that publish or a later one).
int wait_publish_at_least(tgo_ctx* ctx, unsigned long long seq) {
    Scratch& s = ctx->sc;
    const volatile unsigned long long* flag = reinterpret_cast<volatile unsigned long long*>(s.hcnt) + kCounterWords;
    for (uint64_t it = 1;; ++it) {
        if (*flag >= seq) break;
        if ((it & 0x3FFF) == 0) {
            const hipError_t q = hipStreamQuery(ctx->stream);
            if (q != hipSuccess && q != hipErrorNotReady) return fail(ctx, TGO_E_HIP, hipGetErrorString(q));
            if (q == hipSuccess && *flag < seq) return fail(ctx, TGO_E_HIP, "loop state publish not visible after the stream drained");
        }
        __builtin_ia32_pause();
    }
    std::atomic_thread_fence(std::memory_order_acquire);
    return TGO_OK;
}

// Exclusive scan of qdeg[0..qlen) into qpre[0..qlen] (qpre[qlen] = total).
int scan_frontier(tgo_ctx* ctx, int64_t qlen) {
    Scratch& s = ctx->sc;
    HIP_TRY(hipMemsetAsync(s.qdeg + qlen, 0, sizeof(int64_t), ctx->stream));
    HIP_TRY(scan_exclusive_i64(s.cub_tmp, s.cub_bytes, s.qdeg, s.qpre, qlen + 1, ctx->stream));
    return TGO_OK;
}

// Direction-optimizing level loop for unit weights (Beamer et al., SC'12 heuristics).
int run_bfs(tgo_ctx* ctx, int64_t seed, int max_depth, int scope) {
    DevGraph& g = ctx->g;
    Scratch& s = ctx->sc;
    hipStream_t st = ctx->stream;
    const int64_t n = g.n, words = (n + 63) / 64 + 1;
    const View pull = pull_view(g, scope), push = push_view(g, scope);
    HIP_TRY(k_fill_i32(s.level, -1, n, st));
    HIP_TRY(hipMemsetAsync(s.vb, 0, words * 8, st));
    HIP_TRY(hipMemsetAsync(s.fb, 0, words * 8, st));
    int levels = 0;
    if (seed >= 0) {
        HIP_TRY(k_bfs_seed(push, s.level, s.vb, s.fb, s.q[0], s.qdeg, seed, st));
        HIP_TRY(k_level_prep(s.cnt, s.nb, words, s.qdeg + 1, st));   // level 0: counters, nb, scan tail
        int64_t qlen = 1;
        int cur = 0;
        bool bottom_up = false;
        // Beamer's switch thresholds; TGO_BFS_ALPHA / TGO_BFS_BETA override for tuning.  Round 5:
        // alpha 30 (bottom-up once the frontier's entries pass 1/30 of the unexplored ones) and
        // beta 5000 (top-down again only below n/5000 frontier vertices), against Beamer's 15 / 18:
        // hmean 301-318 -> 327-338 GTEPS over the 64 bench roots (profiles/r05ab_bfs_switch_ab.log).
        // The roots that gain have a level-1 frontier of ~2300 hubs with ~18 M entries, just under
        // mu / 15: top-down spent ~0.68 ms on that level, where the bottom-up finds nearly every
        // vertex's parent among the hubs within a few entries.
        static const double alpha = env_double("TGO_BFS_ALPHA", 30.0);
        static const double beta = env_double("TGO_BFS_BETA", 5000.0);
        static const bool trace = env_double("TGO_TRACE", 0.0) != 0.0;
        // m_u: entries of unexplored vertices (push degrees); m_f: of the frontier.
        const int64_t total_push = push.nlists > 1 ? (g.out.nnz + g.in.nnz)
                                                   : (g.has_transpose ? g.push_t.nnz
                                                                      : (scope == TGO_SCOPE_IN_E ? g.in.nnz : g.out.nnz));
        int64_t mf = -1, mu = total_push;
        bool queued = true;         // q[cur] holds the frontier (bottom-up levels only count it)
        for (int L = 0; L < max_depth && qlen > 0; ++L) {
            if (mf < 0) {   // degree of the seed, through the mapped counter page (a copy and a
                            // stream synchronisation cost ~30 us before the first level)
                const unsigned long long seq = ++s.pub_seq;
                HIP_TRY(k_publish_words(s.qdeg, 1, s.hcnt_dev, seq, st));
                if (int rc = wait_publish(ctx, seq)) return rc;
                const int64_t d = static_cast<int64_t>(reinterpret_cast<volatile unsigned long long*>(s.hcnt)[0]);
                mf = d;
                mu -= d;
            }
            if (!bottom_up && static_cast<double>(mf) > static_cast<double>(mu) / alpha) bottom_up = true;
            else if (bottom_up && static_cast<double>(qlen) < static_cast<double>(n) / beta) bottom_up = false;
            // every level starts with zero counters, a clear nb and qdeg[qlen] = 0: level_turn
            // at the end of the previous level (the first: the level_prep before the loop)
            if (!bottom_up && !queued) {    // after bottom-up levels: queue the frontier bitmap
                HIP_TRY(k_bfs_queue(push, g.n_active, s.fb, s.q[cur], s.qdeg, s.cnt, st));
                HIP_TRY(k_level_prep(s.cnt, nullptr, 0, nullptr, st));   // the queue's counts out
            }
            queued = !bottom_up;
            DevSpan span(st, "bfs.level", {"level", L}, {"bottom_up", bottom_up ? 1 : 0});
            if (bottom_up) {
                // words past n_active hold only entry-less vertices: nothing to find there
                HIP_TRY(k_bu_step(pull, push, g.n_active, s.fb, s.vb, s.nb, s.level, s.cnt, L + 1, st));
            } else {
                HIP_TRY(scan_exclusive_i64(s.cub_tmp, s.cub_bytes, s.qdeg, s.qpre, qlen + 1, st));
                // qdeg is reused for the next queue's degrees after the scan consumed it
                HIP_TRY(k_td_expand(push, s.q[cur], s.qpre, qlen, s.level, s.vb, s.nb, s.q[cur ^ 1], s.qdeg, s.cnt, L + 1, st));
            }
            span.end();
            // the counters to the host, then the next level's prep (fb, consumed, is its nb)
            const unsigned long long seq = ++s.pub_seq;
            HIP_TRY(k_level_turn(s.cnt, s.hcnt_dev, seq, s.fb, words, s.qdeg, st));
            int rc = wait_publish(ctx, seq);
            if (rc) return rc;
            qlen = static_cast<int64_t>(s.hcnt->qlen);
            mf = static_cast<int64_t>(s.hcnt->mf);
            mu -= mf;
            if (trace) std::fprintf(stderr, "[tgo] level %d %s -> next frontier %lld vertices, %lld entries (unexplored %lld)\n",
                                    L, bottom_up ? "BU" : "TD", (long long)qlen, (long long)mf, (long long)mu);
            std::swap(s.fb, s.nb);
            cur ^= 1;
            ++levels;
        }
    }
    HIP_TRY(k_level_to_dist(s.level, s.dist, n, st));
    trace_resolve(st);
    ctx->st.levels = levels;
    ctx->st.iterations = max_depth;   // the reference always runs iterations 0..maxDepth
    return TGO_OK;
}

int run_sssp(tgo_ctx* ctx, int64_t seed, int max_depth, int scope, bool weighted) {
    DevGraph& g = ctx->g;
    Scratch& s = ctx->sc;
    hipStream_t st = ctx->stream;
    const int64_t n = g.n, words = (n + 63) / 64 + 1;
    const View push = push_view(g, scope);
    HIP_TRY(k_fill_i64(s.dist, INT64_MAX, n, st));
    HIP_TRY(hipMemsetAsync(s.vb, 0, words * 8, st));
    int levels = 0;
    if (seed >= 0) {
        HIP_TRY(k_sssp_seed(push, s.dist, s.msg, s.vb, s.q[0], s.qdeg, seed, st));
        int64_t qlen = 1;
        int cur = 0;
        for (int L = 0; L < max_depth && qlen > 0; ++L) {
            // counters, "improved this level" marks, scan tail
            DevSpan span(st, "sssp.superstep", {"superstep", L}, {"queue", qlen});
            HIP_TRY(k_level_prep(s.cnt, s.vb, words, s.qdeg + qlen, st));
            HIP_TRY(scan_exclusive_i64(s.cub_tmp, s.cub_bytes, s.qdeg, s.qpre, qlen + 1, st));
            int rc;
            HIP_TRY(k_sssp_relax(push, s.q[cur], s.qpre, qlen, s.msg, s.dist, s.vb, s.q[cur ^ 1], s.qdeg, s.cnt, weighted ? 1 : 0, st));
            span.end();
            rc = read_counters(ctx);
            if (rc) return rc;
            if (s.hcnt->err) return fail(ctx, TGO_E_PROGRAM,
                "vertex program failed: a traversed edge has no value for the weight property");
            qlen = static_cast<int64_t>(s.hcnt->qlen);
            // snapshot the improved vertices' distances: these are their messages
            if (qlen > 0) HIP_TRY(k_sssp_commit(s.q[cur ^ 1], qlen, s.dist, s.msg, s.vb, st));
            cur ^= 1;
            ++levels;
        }
    }
    HIP_TRY(k_dist_finalize(s.dist, n, st));
    trace_resolve(st);
    ctx->st.levels = levels;
    ctx->st.iterations = max_depth;
    return TGO_OK;
}

// Bucket width when the caller passes 0: TGO_DELTA, else a quarter of the mean edge weight
// (RMAT scale 24, weights 1..255: 39 ms at width 32 against 49 ms at 256 and 43 ms at one
// bucket per 2048 — profiles/r01_sssp_delta_sweep.log).
int64_t default_delta(const DevGraph& g, bool weighted) {
    const double env = env_double("TGO_DELTA", 0.0);
    if (env > 0) return static_cast<int64_t>(env);
    return std::max<int64_t>(1, static_cast<int64_t>(weighted ? 0.25 * g.mean_weight : 1.0));
}

// The light/heavy loop driven from the device (delta_loop.hip): the host enqueues steps in
// batches and reads the loop state once per batch (dist, pending and member bitmaps are
// initialised by the caller).
int run_delta_device(tgo_ctx* ctx, int64_t seed, int64_t delta, bool force_scan) {
    DevGraph& g = ctx->g;
    Scratch& s = ctx->sc;
    hipStream_t st = ctx->stream;
    const int64_t n = g.n;
    static const bool trace = env_double("TGO_TRACE", 0.0) != 0.0;
    static const int batch = static_cast<int>(std::max(1.0, env_double("TGO_DS_BATCH", 8.0)));
    // Piles (binned loop, TGO_DS_BINS=0 turns them off): a relaxation from bucket k reaches at
    // most bucket k + 1 + (max_weight - 1) / delta, so that many + 1 piles in a ring hold every
    // pending vertex; wider weight ranges keep the bitmap-scan loop.
    static const bool bins_env = env_double("TGO_DS_BINS", 1.0) != 0.0;
    const bool bins_on = ctx->ds_bins < 0 ? bins_env : ctx->ds_bins != 0;
    const int64_t reach = 2 + (std::max<int64_t>(g.max_weight, 1) - 1) / delta;
    const int nbins = (bins_on && !force_scan && reach <= kDsMaxBins) ? static_cast<int>(reach) : 0;
    // TGO_DS_DONE=1: the relax skips the distance read of done targets (measured neutral at
    // RMAT-24: the largest phases come before most vertices are done); TGO_DS_PILE_SCAN: piles
    // above this fraction of n are extracted by the bitmap scan
    static const bool done_env = env_double("TGO_DS_DONE", 0.0) != 0.0;
    const bool done_filter = ctx->ds_done < 0 ? done_env : ctx->ds_done != 0;
    static const double pile_scan = env_double("TGO_DS_PILE_SCAN", 1.0 / 16.0);
    const int64_t scan_above = static_cast<int64_t>(pile_scan * static_cast<double>(n));
    if (!s.ds_loop) {
        for (int b = 0; b < 2; ++b) {
            HIP_TRY(dev_alloc(ctx, s.ds_q[b], 2 * n + 2));
            HIP_TRY(dev_alloc(ctx, s.ds_qp[b], 2 * n + 2));
        }
        HIP_TRY(dev_alloc(ctx, s.ds_loop, 1));
        ctx->st.device_bytes = ctx->dev_bytes;
    }
    const int64_t cap = ctx->ds_pile_cap > 0 ? ctx->ds_pile_cap : std::max<int64_t>(n, 1024);
    if (nbins && s.ds_pile && s.ds_pile_cap != cap) {
        dev_free(ctx, s.ds_pile, kDsMaxBins * s.ds_pile_cap);
        s.ds_pile_cap = 0;
    }
    if (nbins && !s.ds_pile) {
        // a pile holds up to n appends per bucket (more drop to the bitmap scan of that bucket)
        s.ds_pile_cap = cap;
        HIP_TRY(dev_alloc(ctx, s.ds_pile, kDsMaxBins * s.ds_pile_cap));
        if (!s.ds_mlist) HIP_TRY(dev_alloc(ctx, s.ds_mlist, n + 1));
        if (!s.ds_done) HIP_TRY(dev_alloc(ctx, s.ds_done, (n + 63) / 64 + 1));
        ctx->st.device_bytes = ctx->dev_bytes;
    }
    if (nbins) HIP_TRY(hipMemsetAsync(s.ds_done, 0, ((n + 63) / 64 + 1) * 8, st));
    // Pull form (TGO_DS_PULL = members as a fraction of n, 0 = off): a finished bucket with at
    // least that many members has its heavy entries pulled by the vertices that can still
    // improve (delta_loop.hip ds_pull_heavy) instead of pushed entry by entry.
    static const double pull_env = env_double("TGO_DS_PULL", 0.0);
    const double pull_frac = ctx->ds_pull >= 0 ? ctx->ds_pull : pull_env;
    DsPull pull{};
    if (nbins && pull_frac > 0) {
        const int64_t words = (n + 63) / 64 + 1;
        for (int b = 0; b < 2; ++b) {
            if (!s.ds_pm[b]) HIP_TRY(dev_alloc(ctx, s.ds_pm[b], words));
            if (!s.ds_pl[b]) HIP_TRY(dev_alloc(ctx, s.ds_pl[b], n + 1));
            HIP_TRY(hipMemsetAsync(s.ds_pm[b], 0, words * 8, st));
            pull.pm[b] = s.ds_pm[b];
            pull.pl[b] = s.ds_pl[b];
        }
        ctx->st.device_bytes = ctx->dev_bytes;
        pull.view = pull_view(g, g.scope);
        pull.n_active = g.n_active > 0 ? std::min<int64_t>(g.n_active, n) : n;
        pull.min_members = std::max<int64_t>(1, static_cast<int64_t>(pull_frac * static_cast<double>(n)));
    }
    HIP_TRY(k_ds_loop_seed(g.push_ws, s.ds_light, s.dist, s.ds_q[0], s.ds_qp[0], s.ds_loop, seed, delta, st));
    DsLoop h{};
    int cur = 0;
    // Small steps (TGO_TUNE_DS_SMALL / TGO_DS_SMALL, default off; delta_loop.hip ds_small_steps):
    // the tiny steps run in one block inside one launch.  The binned loop without the done
    // filter or pulls.  Off by default: 12.6 -> 13.8 ms per RMAT-24 source
    // (profiles/r05ss1_sssp_small_ab.log) — a tiny step is a chain of dependent memory
    // round trips either way, and one block pays them with fewer loads in flight.
    static const bool small_env = env_double("TGO_DS_SMALL", 0.0) != 0.0;
    const bool small_on = ctx->ds_small < 0 ? small_env : ctx->ds_small != 0;
    const bool small = small_on && nbins && !done_filter && pull.min_members == 0;
    // every step either relaxes a non-empty queue or extracts (at most one extraction in a row
    // takes nothing); a run needs far fewer than 4n + 64 steps — the bound only stops a bug
    const int64_t max_steps = 4 * n + 64;
    // Pipelined stop checks (TGO_DS_PIPE, default on): each batch ends with a publish of the
    // stop flags to host-mapped words, and the host checks batch k while batch k + 1 runs (a
    // batch after the stop only runs steps that find nothing to do).  The stream no longer
    // drains at every check: one SSSP run had ~12 drains of ~60 us (profiles/r04v_sssp_timeline.txt).
    static const bool pipe = env_double("TGO_DS_PIPE", 1.0) != 0.0;
    if (pipe) {
        unsigned long long pending = 0;                       // publish to check next (0: none)
        bool stop = false;
        for (int64_t steps = 0; !stop;) {
            DevSpan span(st, "sssp.delta_steps", {"first_step", steps}, {"steps", batch});
            for (int k = 0; k < batch; ++k) {
                if (small)
                    HIP_TRY(k_ds_loop_step_small(g.push_ws, s.ds_light, s.vb, s.ds_member, n, s.dist, s.msg, s.ds_q,
                                                 s.ds_qp, s.ds_loop, delta, nbins, s.ds_pile, s.ds_pile_cap,
                                                 s.ds_mlist, s.ds_done, scan_above, st));
                else if (nbins)
                    HIP_TRY(k_ds_loop_step_bins(g.push_ws, s.ds_light, s.vb, s.ds_member, n, s.dist, s.msg, s.ds_q,
                                                s.ds_qp, s.ds_loop, cur, delta, nbins, s.ds_pile, s.ds_pile_cap,
                                                s.ds_mlist, s.ds_done, done_filter, scan_above, pull, st));
                else
                    HIP_TRY(k_ds_loop_step(g.push_ws, s.ds_light, s.vb, s.ds_member, n, s.dist, s.msg, s.ds_q, s.ds_qp,
                                           s.ds_loop, cur, delta, st));
                cur ^= 1;
            }
            steps += batch;
            span.end();
            const unsigned long long seq = ++s.pub_seq;
            HIP_TRY(k_ds_publish(s.ds_loop, s.hcnt_dev, seq, st));
            if (pending) {
                if (int rc = wait_publish_at_least(ctx, pending)) return rc;
                const volatile unsigned long long* hw = reinterpret_cast<volatile unsigned long long*>(s.hcnt);
                if (hw[1]) return fail(ctx, TGO_E_PROGRAM, "vertex program failed: a traversed edge has no value for the weight property");
                stop = hw[0] != 0 || hw[2] != 0;
            }
            pending = seq;
            if (!stop && steps > max_steps) return fail(ctx, TGO_E_HIP, "delta-stepping: the device loop did not converge");
        }
        HIP_TRY(hipMemcpyAsync(&h, s.ds_loop, sizeof(DsLoop), hipMemcpyDeviceToHost, st));
        HIP_TRY(hipStreamSynchronize(st));
        if (h.err) return fail(ctx, TGO_E_PROGRAM, "vertex program failed: a traversed edge has no value for the weight property");
    }
    for (int64_t steps = 0; !pipe;) {
        DevSpan span(st, "sssp.delta_steps", {"first_step", steps}, {"steps", batch});
        for (int k = 0; k < batch; ++k) {
            if (small)
                HIP_TRY(k_ds_loop_step_small(g.push_ws, s.ds_light, s.vb, s.ds_member, n, s.dist, s.msg, s.ds_q,
                                             s.ds_qp, s.ds_loop, delta, nbins, s.ds_pile, s.ds_pile_cap, s.ds_mlist,
                                             s.ds_done, scan_above, st));
            else if (nbins)
                HIP_TRY(k_ds_loop_step_bins(g.push_ws, s.ds_light, s.vb, s.ds_member, n, s.dist, s.msg, s.ds_q, s.ds_qp,
                                            s.ds_loop, cur, delta, nbins, s.ds_pile, s.ds_pile_cap, s.ds_mlist,
                                            s.ds_done, done_filter, scan_above, pull, st));
            else
                HIP_TRY(k_ds_loop_step(g.push_ws, s.ds_light, s.vb, s.ds_member, n, s.dist, s.msg, s.ds_q, s.ds_qp,
                                       s.ds_loop, cur, delta, st));
            cur ^= 1;
        }
        steps += batch;
        span.end();
        HIP_TRY(hipMemcpyAsync(&h, s.ds_loop, sizeof(DsLoop), hipMemcpyDeviceToHost, st));
        HIP_TRY(hipStreamSynchronize(st));
        if (h.err) return fail(ctx, TGO_E_PROGRAM, "vertex program failed: a traversed edge has no value for the weight property");
        if (h.spill) break;
        if (h.done) break;
        if (steps > max_steps) return fail(ctx, TGO_E_HIP, "delta-stepping: the device loop did not converge");
    }
    if (h.spill) {
        // a relaxation reached past the piles (the weight bound was wrong): start again with
        // the bitmap-scan loop (dist, pending and member state re-initialised by the caller)
        trace_resolve(st);
        return TGO_E_STATE;
    }
    HIP_TRY(k_dist_finalize(s.dist, n, st));
    trace_resolve(st);
    if (trace)
        std::fprintf(stderr, "[tgo] delta %lld (device loop, %d piles): %llu phases, %llu buckets, %llu extractions "
                     "(%llu bitmap scans), %llu entries relaxed\n", (long long)delta, nbins, h.phases, h.buckets,
                     h.extractions, h.full_scans, h.relaxed);
    ctx->st.levels = static_cast<int32_t>(h.phases);
    ctx->st.relaxed_entries = static_cast<int64_t>(h.relaxed);
    return TGO_OK;
}

// Light/heavy delta-stepping (delta.hip, weighted one-GPU loads): a bucket's phases relax
// light entries only; when its near queue runs dry the bucket's members relax their heavy
// entries once; then the threshold moves to the next non-empty bucket.
int run_delta_split(tgo_ctx* ctx, int64_t seed, int64_t delta) {
    DevGraph& g = ctx->g;
    Scratch& s = ctx->sc;
    hipStream_t st = ctx->stream;
    const int64_t n = g.n, words = (n + 63) / 64 + 1;
    static const bool trace = env_double("TGO_TRACE", 0.0) != 0.0;
    if (!s.ds_light) {
        HIP_TRY(dev_alloc(ctx, s.ds_light, n + 1));
        HIP_TRY(dev_alloc(ctx, s.ds_member, words));
        ctx->st.device_bytes = ctx->dev_bytes;
    }
    if (s.ds_light_delta != delta) {
        HIP_TRY(k_ds_light_end(g.push_ws, delta, n, s.ds_light, st));
        s.ds_light_delta = delta;
    }
    HIP_TRY(k_fill_i64(s.dist, INT64_MAX, n, st));
    HIP_TRY(hipMemsetAsync(s.vb, 0, words * 8, st));        // pending bitmap
    HIP_TRY(hipMemsetAsync(s.ds_member, 0, words * 8, st));
    // device-driven steps (delta_loop.hip) unless TGO_DS_HOSTLOOP=1 or the packed queue
    // counters could overflow: a queue holds up to 2n + 2 takes (a light and a heavy take per
    // vertex, ds_q / ds_qp are sized for that) in the count field above kDsCountShift, and up
    // to nnz entries below it
    static const bool host_loop = env_double("TGO_DS_HOSTLOOP", 0.0) != 0.0;
    constexpr int64_t kDsMaxCount = int64_t(1) << (64 - kDsCountShift);
    static_assert(kDsCountShift > 32 && kDsCountShift < 64, "queue counter layout");
    if (!host_loop && seed >= 0 && 2 * n + 2 < kDsMaxCount && g.push_ws.nnz < (int64_t(1) << kDsCountShift)) {
        const int rc = run_delta_device(ctx, seed, delta, false);
        if (rc != TGO_E_STATE) return rc;
        HIP_TRY(k_fill_i64(s.dist, INT64_MAX, n, st));
        HIP_TRY(hipMemsetAsync(s.vb, 0, words * 8, st));
        HIP_TRY(hipMemsetAsync(s.ds_member, 0, words * 8, st));
        return run_delta_device(ctx, seed, delta, true);
    }
    int phases = 0, buckets = 0;
    int64_t relaxed = 0;
    // TGO_DS_TRACE=1: one line per phase (queue, entries, wall time since the previous phase)
    static const bool phase_trace = env_double("TGO_DS_TRACE", 0.0) != 0.0;
    auto t_phase = std::chrono::steady_clock::now();
    if (seed >= 0) {
        HIP_TRY(k_ds_seed_ws(g.push_ws, s.ds_light, s.dist, s.q[0], s.qdeg, seed, st));
        int64_t qlen = 1, thr = delta;
        int cur = 0;
        for (;;) {
            if (qlen == 0) {
                // bucket settled: next near queue + the members' heavy entries, one extraction
                HIP_TRY(hipMemsetAsync(s.cnt, 0, sizeof(Counters), st));
                HIP_TRY(hipMemsetAsync(&s.cnt->red[0], 0x7F, sizeof(unsigned long long), st));   // ~INT64_MAX
                HIP_TRY(k_ds_pending_min_ws(s.vb, s.ds_member, words, s.dist, s.cnt, st));
                if (int rc = read_counters(ctx)) return rc;
                const int64_t pending = static_cast<int64_t>(s.hcnt->red[1]);
                const int64_t members = static_cast<int64_t>(s.hcnt->red2);
                if (pending == 0 && members == 0) break;        // converged
                if (pending > 0) {
                    const int64_t mn = static_cast<int64_t>(s.hcnt->red[0]);
                    if (mn >= thr) thr = (mn / delta + 1) * delta;
                    ++buckets;
                }
                HIP_TRY(hipMemsetAsync(s.cnt, 0, sizeof(Counters), st));
                HIP_TRY(k_ds_extract_ws(g.push_ws, s.ds_light, s.vb, s.ds_member, n, s.dist, thr, s.q[cur], s.qdeg, s.cnt,
                                        st));
                if (int rc = read_counters(ctx)) return rc;
                qlen = static_cast<int64_t>(s.hcnt->qlen);
                if (trace) std::fprintf(stderr, "[tgo] delta bucket thr %lld: %lld pending, %lld members, %lld queued\n",
                                        (long long)thr, (long long)pending, (long long)members, (long long)qlen);
                if (qlen == 0) {
                    if (pending > 0) return fail(ctx, TGO_E_HIP, "delta-stepping: extraction found no vertex below the threshold");
                    continue;                                   // members without heavy entries
                }
            }
            HIP_TRY(k_ds_commit_ws(s.q[cur], qlen, s.dist, s.msg, s.vb, s.ds_member, s.qdeg, s.cnt, st));
            HIP_TRY(scan_exclusive_i64(s.cub_tmp, s.cub_bytes, s.qdeg, s.qpre, qlen + 1, st));   // tail zeroed by commit
            HIP_TRY(k_ds_relax_ws(g.push_ws, s.ds_light, s.q[cur], s.qpre, qlen, s.msg, s.dist, s.vb, s.q[cur ^ 1], s.qdeg,
                                  s.cnt, thr, st));
            if (int rc = read_counters(ctx)) return rc;
            if (s.hcnt->err) return fail(ctx, TGO_E_PROGRAM,
                "vertex program failed: a traversed edge has no value for the weight property");
            relaxed += static_cast<int64_t>(s.hcnt->red[1]);
            if (phase_trace) {
                const auto now = std::chrono::steady_clock::now();
                std::fprintf(stderr, "[tgo] ds phase %d thr %lld: queue %lld, entries %llu, next %llu, %.1f us\n", phases,
                             (long long)thr, (long long)qlen, s.hcnt->red[1], s.hcnt->qlen,
                             std::chrono::duration<double, std::micro>(now - t_phase).count());
                t_phase = now;
            }
            qlen = static_cast<int64_t>(s.hcnt->qlen);
            cur ^= 1;
            ++phases;
        }
    }
    HIP_TRY(k_dist_finalize(s.dist, n, st));
    if (trace) std::fprintf(stderr, "[tgo] delta %lld (light/heavy): %d phases, %d buckets, %lld entries relaxed\n",
                            (long long)delta, phases, buckets, (long long)relaxed);
    ctx->st.levels = phases;
    ctx->st.relaxed_entries = relaxed;
    return TGO_OK;
}

// Delta-stepping (delta.hip): converged distances, near queue relaxed phase by phase,
// bucket threshold advanced from the minimum pending distance when the queue runs dry.
int run_delta(tgo_ctx* ctx, int64_t seed, int scope, bool weighted, int64_t delta) {
    DevGraph& g = ctx->g;
    Scratch& s = ctx->sc;
    hipStream_t st = ctx->stream;
    const int64_t n = g.n, words = (n + 63) / 64 + 1;
    const View push = push_view(g, scope);
    static const bool trace = env_double("TGO_TRACE", 0.0) != 0.0;
    if (delta <= 0) delta = default_delta(g, weighted);
    if (weighted && g.push_ws_ready && scope == g.scope) return run_delta_split(ctx, seed, delta);
    HIP_TRY(k_fill_i64(s.dist, INT64_MAX, n, st));
    HIP_TRY(hipMemsetAsync(s.vb, 0, words * 8, st));        // pending bitmap
    int phases = 0, buckets = 0;
    int64_t relaxed = 0;
    if (seed >= 0) {
        HIP_TRY(k_ds_seed(push, s.dist, s.q[0], s.qdeg, seed, st));
        int64_t qlen = 1, thr = delta;
        int cur = 0;
        for (;;) {
            if (qlen == 0) {
                HIP_TRY(hipMemsetAsync(s.cnt, 0, sizeof(Counters), st));
                HIP_TRY(hipMemsetAsync(&s.cnt->red[0], 0x7F, sizeof(unsigned long long), st));   // ~INT64_MAX
                HIP_TRY(k_ds_pending_min(s.vb, words, s.dist, s.cnt, st));
                if (int rc = read_counters(ctx)) return rc;
                if (s.hcnt->red[1] == 0) break;                 // nothing pending: converged
                const int64_t mn = static_cast<int64_t>(s.hcnt->red[0]);
                if (mn >= thr) thr = (mn / delta + 1) * delta;
                ++buckets;
                HIP_TRY(hipMemsetAsync(s.cnt, 0, sizeof(Counters), st));
                HIP_TRY(k_ds_extract(push, s.vb, n, s.dist, thr, s.q[cur], s.qdeg, s.cnt, st));
                if (int rc = read_counters(ctx)) return rc;
                qlen = static_cast<int64_t>(s.hcnt->qlen);
                if (trace) std::fprintf(stderr, "[tgo] delta bucket thr %lld: min pending %lld, %llu pending, %lld queued\n",
                                        (long long)thr, (long long)mn, s.hcnt->red[1], (long long)qlen);
                if (qlen == 0) return fail(ctx, TGO_E_HIP, "delta-stepping: extraction found no vertex below the threshold");
            }
            HIP_TRY(k_ds_commit(s.q[cur], qlen, s.dist, s.msg, s.vb, st));
            if (int rc = scan_frontier(ctx, qlen)) return rc;
            HIP_TRY(hipMemsetAsync(s.cnt, 0, sizeof(Counters), st));
            HIP_TRY(k_ds_relax(push, s.q[cur], s.qpre, qlen, s.msg, s.dist, s.vb, s.q[cur ^ 1], s.qdeg, s.cnt,
                               weighted ? 1 : 0, thr, st));
            if (int rc = read_counters(ctx)) return rc;
            if (s.hcnt->err) return fail(ctx, TGO_E_PROGRAM,
                "vertex program failed: a traversed edge has no value for the weight property");
            relaxed += static_cast<int64_t>(s.hcnt->red[1]);      // qpre[qlen], set by ds_relax
            qlen = static_cast<int64_t>(s.hcnt->qlen);
            cur ^= 1;
            ++phases;
        }
    }
    HIP_TRY(k_dist_finalize(s.dist, n, st));
    if (trace) std::fprintf(stderr, "[tgo] delta %lld: %d phases, %d buckets, %lld entries relaxed\n",
                            (long long)delta, phases, buckets, (long long)relaxed);
    ctx->st.levels = phases;
    ctx->st.relaxed_entries = relaxed;
    return TGO_OK;
}

int finish_distance_program(tgo_ctx* ctx, int scope, int flags, int64_t* dist_out) {
    Scratch& s = ctx->sc;
    HIP_TRY(hipEventRecord(ctx->ev1, ctx->stream));
    HIP_TRY(hipEventSynchronize(ctx->ev1));
    float ms = 0;
    HIP_TRY(hipEventElapsedTime(&ms, ctx->ev0, ctx->ev1));
    ctx->st.last_kernel_ms = ms;
    if (flags & TGO_FLAG_STATS) {
        // reached vertices and the entries of their pull lists (both lists for bothE)
        HIP_TRY(hipMemsetAsync(s.cnt, 0, sizeof(Counters), ctx->stream));
        HIP_TRY(k_reach_stats(pull_view(ctx->g, scope), s.dist, ctx->g.n, s.cnt->red, ctx->stream));
        int rc = read_counters(ctx);
        if (rc) return rc;
        ctx->st.reached = static_cast<int64_t>(s.hcnt->red[0]);
        ctx->st.reached_entries = static_cast<int64_t>(s.hcnt->red[1]);
    }
    if (dist_out) {
        HIP_TRY(k_unpermute_i64(s.dist, ctx->g.perm, s.msg, ctx->g.n, ctx->stream));
        HIP_TRY(hipMemcpyAsync(dist_out, s.msg, ctx->g.n * sizeof(int64_t), hipMemcpyDeviceToHost, ctx->stream));
        HIP_TRY(hipStreamSynchronize(ctx->stream));
    }
    (void)scope;
    return TGO_OK;
}

}  // namespace

// ============================================================================ C-ABI

namespace tgo { double ms_split_of(const tgo_ctx* ctx); int part_upload(tgo_ctx* ctx, HostGraph& h, int64_t n_global, int64_t lo); }

namespace {
struct TrimTemps {                  // tmp_cache.cpp: nothing stays reserved between loads
    ~TrimTemps() { tgo::tmp_trim(); }
};
}  // namespace

extern "C" {

void tgo_default_options(tgo_options* o) {
    std::memset(o, 0, sizeof(*o));
    o->abi_version = TGO_ABI_VERSION;
    o->device = 0;
    o->partition_bits = 5;
    o->host_threads = 0;
    o->hard_query_limit = 100000;
    o->stream = nullptr;
}

int tgo_set_tuning(tgo_ctx* ctx, int32_t key, double value) {
    if (!ctx) return TGO_E_INVALID;
    switch (key) {
    case TGO_TUNE_MS_SPLIT:
        if (!(value <= 1.0)) return fail(ctx, TGO_E_INVALID, "TGO_TUNE_MS_SPLIT: a fraction <= 1 (< 0: the default)");
        ctx->ms_split = value < 0.0 ? -1.0 : value;
        return TGO_OK;
    case TGO_TUNE_MS_GHOST:
        if (value != 0.0 && value != 1.0) return fail(ctx, TGO_E_INVALID, "TGO_TUNE_MS_GHOST: 0 or 1");
        ctx->ms_ghost = value != 0.0 ? 1 : 0;
        return TGO_OK;
    case TGO_TUNE_DS_BINS:
        if (value != 0.0 && value != 1.0 && value != -1.0) return fail(ctx, TGO_E_INVALID, "TGO_TUNE_DS_BINS: 0, 1 or -1");
        ctx->ds_bins = static_cast<int>(value);
        return TGO_OK;
    case TGO_TUNE_DS_DONE:
        if (value != 0.0 && value != 1.0 && value != -1.0) return fail(ctx, TGO_E_INVALID, "TGO_TUNE_DS_DONE: 0, 1 or -1");
        ctx->ds_done = static_cast<int>(value);
        return TGO_OK;
    case TGO_TUNE_DS_SMALL:
        if (value != 0.0 && value != 1.0 && value != -1.0) return fail(ctx, TGO_E_INVALID, "TGO_TUNE_DS_SMALL: 0, 1 or -1");
        ctx->ds_small = static_cast<int>(value);
        return TGO_OK;
    case TGO_TUNE_DS_PULL:
        if (!(value >= -1.0) || value > 1.0) return fail(ctx, TGO_E_INVALID, "TGO_TUNE_DS_PULL: a fraction in [0, 1] or -1");
        ctx->ds_pull = value;
        return TGO_OK;
    case TGO_TUNE_MS_COLD:
        if (!(value >= -1.0) || value >= 2147483647.0 || value != static_cast<double>(static_cast<int64_t>(value)))
            return fail(ctx, TGO_E_INVALID, "TGO_TUNE_MS_COLD: -1, 0, 1 or a hot-head size > 1");
        ctx->ms_cold = static_cast<int64_t>(value);
        return TGO_OK;
    case TGO_TUNE_DS_PILE_CAP:
        if (!(value >= 0.0) || value > 9.0e15) return fail(ctx, TGO_E_INVALID, "TGO_TUNE_DS_PILE_CAP: entries >= 0");
        ctx->ds_pile_cap = static_cast<int64_t>(value);
        return TGO_OK;
    default:
        return fail(ctx, TGO_E_INVALID, "tgo_set_tuning: unknown key");
    }
}

int tgo_create(const tgo_options* opts, tgo_ctx** out) {
    if (!opts || !out) return TGO_E_INVALID;
    *out = nullptr;
    if (opts->abi_version != TGO_ABI_VERSION) return TGO_E_INVALID;
    if (opts->partition_bits < 0 || opts->partition_bits > 16) return TGO_E_INVALID;
    int ndev = 0;
    if (hipGetDeviceCount(&ndev) != hipSuccess || ndev <= 0) return TGO_E_HIP;
    if (opts->device < 0 || opts->device >= ndev) return TGO_E_INVALID;
    if (hipSetDevice(opts->device) != hipSuccess) return TGO_E_HIP;
    hipDeviceProp_t prop;
    if (hipGetDeviceProperties(&prop, opts->device) != hipSuccess) return TGO_E_HIP;
    if (std::strncmp(prop.gcnArchName, "gfx950", 6) != 0) return TGO_E_HIP;   // gfx950 code objects only
    tgo_ctx* ctx = new (std::nothrow) tgo_ctx();
    if (!ctx) return TGO_E_OOM;
    ctx->opts = *opts;
    ctx->num_cus = prop.multiProcessorCount > 0 ? prop.multiProcessorCount : 256;
    if (ctx->opts.hard_query_limit <= 0) ctx->opts.hard_query_limit = 100000;
    if (opts->stream) {
        ctx->stream = static_cast<hipStream_t>(opts->stream);
    } else {
        if (hipStreamCreateWithFlags(&ctx->stream, hipStreamNonBlocking) != hipSuccess) { delete ctx; return TGO_E_HIP; }
        ctx->own_stream = true;
    }
    if (hipEventCreate(&ctx->ev0) != hipSuccess || hipEventCreate(&ctx->ev1) != hipSuccess) {
        delete ctx;
        return TGO_E_HIP;
    }
    *out = ctx;
    return TGO_OK;
}

void tgo_destroy(tgo_ctx* ctx) {
    if (!ctx) return;
    (void)hipSetDevice(ctx->opts.device);
    if (ctx->stream) (void)hipStreamSynchronize(ctx->stream);
    free_graph(ctx);
    ctx->dec.release();
    if (ctx->sc.hcnt) (void)hipHostFree(ctx->sc.hcnt);
    if (ctx->ev0) (void)hipEventDestroy(ctx->ev0);
    if (ctx->ev1) (void)hipEventDestroy(ctx->ev1);
    if (ctx->own_stream && ctx->stream) (void)hipStreamDestroy(ctx->stream);
    delete ctx;
}

const char* tgo_last_error(const tgo_ctx* ctx) { return ctx ? ctx->err.c_str() : "null ctx"; }

int tgo_decode_edge_entry(const tgo_schema* schema, const tgo_load_opts* opts, const uint8_t* entry,
                          int64_t len, int64_t value_pos, tgo_edge_entry* out) {
    if (!schema || !opts || !out) return TGO_E_INVALID;
    std::string err;
    return decode_one_entry(schema, opts, entry, len, value_pos, out, err);
}

int tgo_load_rows(tgo_ctx* ctx, const tgo_rows* rows, const tgo_schema* schema, const tgo_load_opts* opts) {
    if (!ctx) return TGO_E_INVALID;
    ctx->res_kind = -1;
    if (!rows || !schema || !opts) return fail(ctx, TGO_E_INVALID, "null argument");
    if (rows->nrows < 0 || (rows->nrows > 0 && (!rows->row_keys || !rows->row_entry_begin ||
        !rows->row_byte_begin || !rows->entry_bytes || !rows->entry_limit_valpos)))
        return fail(ctx, TGO_E_INVALID, "incomplete tgo_rows");
    if (opts->scope < 0 || opts->scope > 2) return fail(ctx, TGO_E_INVALID, "invalid scope");
    if (ctx->loaded && !ctx->staging.active) free_graph(ctx);
    (void)hipSetDevice(ctx->opts.device);
    const auto t0 = std::chrono::steady_clock::now();
    std::string err;
    // device decode (decode.hip) unless TGO_HOST_DECODE=1 picks the multi-threaded host decoder
    // (latched at the first batch of a load, so one load never mixes the two)
    if (!ctx->staging.active) {
        const char* host = std::getenv("TGO_HOST_DECODE");
        ctx->host_decode = host && std::atoi(host) != 0;
    }
    int rc = ctx->host_decode ? decode_rows(ctx->staging, rows, schema, opts, ctx->opts.partition_bits,
                                       ctx->opts.hard_query_limit, threads_of(ctx), err)
                         : stage_rows_raw(ctx->staging, rows, schema, opts, ctx->dec, ctx->stream, err);
    ctx->st.load_ms += std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
    if (rc) { ctx->staging = RowStaging(); return fail(ctx, rc, err); }
    return TGO_OK;
}

int tgo_finish_load(tgo_ctx* ctx) {
    Span load_span("load.finish_rows");
    TrimTemps trim_temps;   // the build temporaries are released when the load returns
    if (!ctx) return TGO_E_INVALID;
    if (!ctx->staging.active) return fail(ctx, TGO_E_STATE, "tgo_finish_load without tgo_load_rows");
    (void)hipSetDevice(ctx->opts.device);
    const auto t0 = std::chrono::steady_clock::now();
    HostGraph h;
    std::string err;
    // the staged work blocks, decoded in one device pass (decode.hip); the kept entries stay
    // on the device for the device assembly
    const bool dev_asm = env_i64("TGO_HOST_ASSEMBLY", 0) == 0;
    int rc = decode_staged_raw(ctx->staging, ctx->opts.partition_bits, ctx->opts.hard_query_limit, ctx->dec,
                               ctx->stream, err, dev_asm);
    ctx->dec.release();
    if (rc) { ctx->staging = RowStaging(); return fail(ctx, rc, err); }
    if (env_i64("TGO_TRACE", 0))
        std::fprintf(stderr, "[tgo] finish_load decode %8.1f ms\n",
                     std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count());
    // CSR assembly on the device (assemble.hip) unless TGO_HOST_ASSEMBLY=1 or the scan holds
    // vertex cuts (their representative rows fold on the host, graph_build.cpp)
    const RowStaging& stg = ctx->staging;
    const bool cuts = stg.n_rep > 0 || std::any_of(stg.vid.begin(), stg.vid.end(), [](int64_t v) { return (v & 7) == 2; });
    const bool on_dev = dev_asm && !cuts;
    if (!on_dev) rc = staging_entries_to_host(ctx->staging, ctx->stream, err);
    // a wide (Long / Double) weight key: the staged values become the graph's value table (taken
    // before the assembly, which consumes the staging)
    std::vector<int64_t> wval = std::move(ctx->staging.wv);
    DevArray<int64_t> d_wval = std::move(ctx->staging.d_wv);
    if (!rc)
        rc = on_dev ? assemble_rows_device(ctx->staging, h, ctx->stream, err)
                    : assemble_from_rows(ctx->staging, h, threads_of(ctx), err);
    if (rc) { ctx->staging = RowStaging(); return fail(ctx, rc, err); }
    h.wval = std::move(wval);
    h.d_wval = std::move(d_wval);
    if (env_i64("TGO_TRACE", 0))
        std::fprintf(stderr, "[tgo] finish_load decode + assembly (%s) %8.1f ms\n", on_dev ? "device" : "host",
                     std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count());
    free_graph(ctx);
    rc = upload_graph(ctx, h);
    ctx->st.load_ms += std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
    return rc;
}

int tgo_load_edges(tgo_ctx* ctx, const tgo_edges* edges, const tgo_load_opts* opts) {
    Span load_span("load.edges");
    TrimTemps trim_temps;   // the build temporaries are released when the load returns
    if (!ctx) return TGO_E_INVALID;
    ctx->res_kind = -1;
    if (!edges || !opts || (edges->m > 0 && (!edges->src || !edges->dst)))
        return fail(ctx, TGO_E_INVALID, "null argument");
    if (opts->scope < 0 || opts->scope > 2) return fail(ctx, TGO_E_INVALID, "invalid scope");
    (void)hipSetDevice(ctx->opts.device);
    const auto t0 = std::chrono::steady_clock::now();
    HostGraph h;
    std::string err;
    // device assembly (assemble.hip) unless TGO_HOST_ASSEMBLY=1
    const bool on_dev = env_i64("TGO_HOST_ASSEMBLY", 0) == 0;
    int rc = on_dev ? assemble_edges_device(edges, opts, ctx->opts.hard_query_limit, h, ctx->stream, err)
                    : assemble_from_edges(edges, opts, ctx->opts.hard_query_limit, h, threads_of(ctx), err);
    if (rc) return fail(ctx, rc, err);
    if (env_i64("TGO_TRACE", 0))
        std::fprintf(stderr, "[tgo] load_edges assembly (%s) %8.1f ms\n", on_dev ? "device" : "host",
                     std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count());
    free_graph(ctx);
    ctx->staging = RowStaging();
    rc = upload_graph(ctx, h);
    ctx->st.load_ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
    return rc;
}

int tgo_load_csr(tgo_ctx* ctx, int64_t n, const int64_t* titan_ids, const int64_t* out_off, const int32_t* out_idx,
                 const int32_t* out_w, const int64_t* in_off, const int32_t* in_idx, const int32_t* in_w,
                 const tgo_load_opts* opts) {
    if (!ctx) return TGO_E_INVALID;
    Span load_span("load.csr");
    TrimTemps trim_temps;   // the build temporaries are released when the load returns
    ctx->res_kind = -1;
    if (!opts || !out_off || !in_off) return fail(ctx, TGO_E_INVALID, "null argument");
    if (opts->scope < 0 || opts->scope > 2) return fail(ctx, TGO_E_INVALID, "invalid scope");
    if (opts->n_labels != 0) return fail(ctx, TGO_E_INVALID, "tgo_load_csr takes no label_ids (the rows are already sliced)");
    if (ctx->staging.active)            // a tgo_load_rows scan is in progress: finish (or destroy) it first
        return fail(ctx, TGO_E_STATE, "tgo_load_csr during a row load (tgo_load_rows without tgo_finish_load)");
    (void)hipSetDevice(ctx->opts.device);
    const auto t0 = std::chrono::steady_clock::now();
    // the rows as a staging of decoded rows (each row's OUT entries, then its IN entries), on
    // the device; then the row assembly of tgo_finish_load
    RowStaging st;
    st.active = true;
    st.opts = *opts;
    st.opts.label_ids = nullptr;
    const bool weighted = opts->weight_key != 0;
    const CsrInput in{n, titan_ids, {out_off, in_off}, {out_idx, in_idx}, {out_w, in_w}};
    std::string err;
    int rc = stage_csr_device(in, weighted, st, ctx->stream, err);
    if (rc) return fail(ctx, rc, err);
    HostGraph h;
    const bool on_dev = env_i64("TGO_HOST_ASSEMBLY", 0) == 0;
    if (!on_dev) rc = staging_entries_to_host(st, ctx->stream, err);
    if (!rc) rc = on_dev ? assemble_rows_device(st, h, ctx->stream, err) : assemble_from_rows(st, h, threads_of(ctx), err);
    if (rc) return fail(ctx, rc, err);
    free_graph(ctx);
    ctx->staging = RowStaging();
    rc = upload_graph(ctx, h);
    ctx->st.load_ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
    return rc;
}

int64_t tgo_num_vertices(const tgo_ctx* ctx) { return ctx && ctx->loaded ? ctx->g.n : 0; }

int tgo_vertex_ids(tgo_ctx* ctx, int64_t* out) {
    if (!ctx || !out) return TGO_E_INVALID;
    if (!ctx->loaded) return fail(ctx, TGO_E_STATE, "no graph loaded");
    std::memcpy(out, ctx->titan_id.data(), ctx->titan_id.size() * sizeof(int64_t));
    return TGO_OK;
}

int tgo_graph_csr(tgo_ctx* ctx, int32_t which, int64_t* nnz, int64_t* off, int32_t* adj, int32_t* w, uint32_t* col) {
    if (!ctx || !nnz || which < 0 || which > 2) return TGO_E_INVALID;
    if (!ctx->loaded) return fail(ctx, TGO_E_STATE, "no graph loaded");
    const DevGraph& g = ctx->g;
    if (which == 2 && !g.has_transpose) { *nnz = -1; return TGO_OK; }
    const DevCsr& c = which == 0 ? g.out : which == 1 ? g.in : g.push_t;
    *nnz = c.nnz;
    (void)hipSetDevice(ctx->opts.device);
    if (off) HIP_TRY(copy_chunked(off, c.off, (g.n + 1) * sizeof(int64_t), hipMemcpyDeviceToHost));
    if (adj && c.nnz) HIP_TRY(copy_chunked(adj, c.adj, c.nnz * sizeof(int32_t), hipMemcpyDeviceToHost));
    if (w && c.w && c.nnz) HIP_TRY(copy_chunked(w, c.w, c.nnz * sizeof(int32_t), hipMemcpyDeviceToHost));
    if (col && c.col && c.nnz) HIP_TRY(copy_chunked(col, c.col, c.nnz * sizeof(uint32_t), hipMemcpyDeviceToHost));
    return TGO_OK;
}

int tgo_graph_perm(tgo_ctx* ctx, int32_t* perm) {
    if (!ctx || !perm) return TGO_E_INVALID;
    if (!ctx->loaded) return fail(ctx, TGO_E_STATE, "no graph loaded");
    (void)hipSetDevice(ctx->opts.device);
    HIP_TRY(hipMemcpy(perm, ctx->g.perm, ctx->g.n * sizeof(int32_t), hipMemcpyDeviceToHost));
    return TGO_OK;
}

int tgo_bfs(tgo_ctx* ctx, const tgo_bfs_args* a, int64_t* dist_out) {
    if (!ctx) return TGO_E_INVALID;
    ctx->res_kind = -1;
    if (!a) return fail(ctx, TGO_E_INVALID, "null args");
    int rc = check_program(ctx, a->scope);
    if (rc) return rc;
    if (a->max_depth < 0) return fail(ctx, TGO_E_INVALID, "max_depth < 0");
    (void)hipSetDevice(ctx->opts.device);
    int64_t seed;
    if ((rc = resolve_seed(ctx, a->seed, a->seed_is_dense, seed))) return rc;
    HIP_TRY(hipEventRecord(ctx->ev0, ctx->stream));
    if ((rc = run_bfs(ctx, seed, a->max_depth, a->scope))) return rc;
    if ((rc = finish_distance_program(ctx, a->scope, a->flags, dist_out))) return rc;
    ctx->res_kind = TGO_RESULT_DISTANCE;
    ctx->res_empty = false;
    ctx->res_src = ResultSource{ctx->sc.dist, nullptr};
    return TGO_OK;
}

int tgo_sssp(tgo_ctx* ctx, const tgo_sssp_args* a, int64_t* dist_out) {
    if (!ctx) return TGO_E_INVALID;
    ctx->res_kind = -1;
    if (!a) return fail(ctx, TGO_E_INVALID, "null args");
    int rc = check_program(ctx, a->scope);
    if (rc) return rc;
    if (a->max_depth < 0) return fail(ctx, TGO_E_INVALID, "max_depth < 0");
    if (a->mode != TGO_SSSP_HOP_BOUNDED && a->mode != TGO_SSSP_DELTA) return fail(ctx, TGO_E_INVALID, "invalid mode");
    if (ctx->g.has_weight && ctx->g.weight_dt != TGO_DT_INTEGER)
        return fail(ctx, TGO_E_UNSUPPORTED, "ShortestDistanceVertexProgram reads edge.<Integer>value(weight): the weight "
                                            "property is not an Integer key (ClassCastException in the reference)");
    (void)hipSetDevice(ctx->opts.device);
    int64_t seed;
    if ((rc = resolve_seed(ctx, a->seed, a->seed_is_dense, seed))) return rc;
    HIP_TRY(hipEventRecord(ctx->ev0, ctx->stream));
    ctx->st.relaxed_entries = 0;
    if (a->mode == TGO_SSSP_DELTA) {
        // converged distances (== the reference's whenever maxDepth >= the hop count of
        // every shortest path); max_depth only sets the reported iteration count
        if (ctx->g.has_weight && ctx->g.min_weight < 0)
            return fail(ctx, TGO_E_INVALID, "DELTA mode needs non-negative weights");
        if ((rc = run_delta(ctx, seed, a->scope, ctx->g.has_weight, a->delta))) return rc;
        ctx->st.iterations = a->max_depth;
    } else {
        if ((rc = run_sssp(ctx, seed, a->max_depth, a->scope, ctx->g.has_weight))) return rc;
    }
    if ((rc = finish_distance_program(ctx, a->scope, a->flags, dist_out))) return rc;
    ctx->res_kind = TGO_RESULT_DISTANCE;
    ctx->res_empty = false;
    ctx->res_src = ResultSource{ctx->sc.dist, nullptr};
    return TGO_OK;
}

// ------------------------------------------------------------------ multi-source BFS
static LevelPlanes ms_planes(tgo_ctx* ctx) { return LevelPlanes{ctx->sc.ms_lvl, ctx->g.n}; }

// Zero the level planes a discovery at `level` writes (planes 0..floor(log2(level))) that
// this sweep has not zeroed yet: vertices reached earlier have levels < 2^k, whose bit k
// is 0, so a plane is valid from the moment it is zeroed.
static int ms_planes_for(tgo_ctx* ctx, int32_t level) {
    Scratch& s = ctx->sc;
    while (s.ms_nplanes < kLevelPlanes && (level >> s.ms_nplanes) != 0) {
        HIP_TRY(hipMemsetAsync(s.ms_lvl + static_cast<int64_t>(s.ms_nplanes) * ctx->g.n, 0,
                               ctx->g.n * sizeof(uint64_t), ctx->stream));
        ++s.ms_nplanes;
    }
    return TGO_OK;
}

static int ms_alloc(tgo_ctx* ctx) {
    Scratch& s = ctx->sc;
    if (s.ms_vis) return TGO_OK;
    const int64_t n = ctx->g.n;
    HIP_TRY(dev_alloc(ctx, s.ms_vis, n + 1));
    HIP_TRY(dev_alloc(ctx, s.ms_fr, n + 1));
    HIP_TRY(dev_alloc(ctx, s.ms_nx, n + 1));
    HIP_TRY(dev_alloc(ctx, s.ms_lvl, n * kLevelPlanes + 1));
    HIP_TRY(dev_alloc(ctx, s.ms_fbm, (n + 63) / 64 + 1));
    HIP_TRY(dev_alloc(ctx, s.ms_seeds, TGO_MAX_SOURCES));
    HIP_TRY(dev_alloc(ctx, s.ms_stat, 2 * TGO_MAX_SOURCES));
    HIP_TRY(dev_alloc(ctx, s.ms_srcent, TGO_MAX_SOURCES));
    ctx->st.device_bytes = ctx->dev_bytes;
    return TGO_OK;
}

// The cold layout of the scope's pull view for the split first pull level (built once per
// graph and scope, on first use): neighbours >= hot (TGO_MS_COLD_HOT, 384 K = 3 MB of masks,
// the hot head every XCD's L2 keeps) in segments of TGO_MS_COLD_SEG (384 K) neighbours.
static int ms_cold_layout(tgo_ctx* ctx, int32_t scope, const View& pull, int64_t hot_req) {
    DevGraph& g = ctx->g;
    Scratch& s = ctx->sc;
    static const int64_t hot_env = static_cast<int64_t>(env_double("TGO_MS_COLD_HOT", 393216.0));
    static const int64_t seg_env = static_cast<int64_t>(env_double("TGO_MS_COLD_SEG", 393216.0));
    const int64_t hot = hot_req > 1 ? hot_req : hot_env, seg = hot_req > 1 ? hot_req : seg_env;
    if (g.msc_scope == scope && g.msc_req == hot) return TGO_OK;
    g.msc_scope = scope;
    g.msc_req = hot;
    g.msc_C = 0;
    if (hot <= 0 || hot >= INT32_MAX || seg <= 0) return TGO_OK;
    Span span("msbfs.cold_layout");
    DevArray<int32_t> cadj, crow;
    int64_t C = 0;
    std::string err;
    if (int rc = build_ms_cold(pull, g.n, static_cast<int32_t>(hot), seg, cadj, crow, C, ctx->stream, err))
        return fail(ctx, rc, err);
    if (C == 0) return TGO_OK;
    adopt(ctx, g.msc_adj, cadj);
    adopt(ctx, g.msc_row, crow);
    if (!s.ms_cacc) {
        HIP_TRY(dev_alloc(ctx, s.ms_cacc, g.n + 1));
        HIP_TRY(dev_alloc(ctx, s.ms_need, g.n + 1));
        HIP_TRY(hipMemsetAsync(s.ms_need, 0, g.n + 1, ctx->stream));
    }
    g.msc_C = C;
    g.msc_hot = static_cast<int32_t>(hot);
    ctx->st.device_bytes = ctx->dev_bytes;
    return TGO_OK;
}

int tgo_bfs_multi(tgo_ctx* ctx, const int64_t* seeds, int32_t nseeds, const tgo_bfs_args* a, int64_t* dist_out) {
    if (!ctx) return TGO_E_INVALID;
    ctx->res_kind = -1;
    if (!a || !seeds) return fail(ctx, TGO_E_INVALID, "null args");
    if (nseeds < 1 || nseeds > TGO_MAX_SOURCES) return fail(ctx, TGO_E_INVALID, "nseeds must be in [1, 64]");
    int rc = check_program(ctx, a->scope);
    if (rc) return rc;
    if (a->max_depth < 0) return fail(ctx, TGO_E_INVALID, "max_depth < 0");
    (void)hipSetDevice(ctx->opts.device);
    if ((rc = ms_alloc(ctx))) return rc;
    DevGraph& g = ctx->g;
    Scratch& s = ctx->sc;
    hipStream_t st = ctx->stream;
    const int64_t n = g.n;
    const View pull = pull_view(g, a->scope), push = push_view(g, a->scope);
    std::vector<int64_t> in(nseeds);
    std::vector<int32_t> uniq;
    for (int r = 0; r < nseeds; ++r) {
        if ((rc = resolve_seed(ctx, seeds[r], a->seed_is_dense, in[r]))) return rc;
        if (in[r] < 0) return fail(ctx, TGO_E_INVALID, "multi-source BFS needs seeds that are executed vertices");
        if (std::find(uniq.begin(), uniq.end(), static_cast<int32_t>(in[r])) == uniq.end())
            uniq.push_back(static_cast<int32_t>(in[r]));
    }
    s.ms_nsrc = nseeds;
    HIP_TRY(hipEventRecord(ctx->ev0, st));
    HIP_TRY(hipMemcpyAsync(s.ms_seeds, in.data(), nseeds * sizeof(int64_t), hipMemcpyHostToDevice, st));
    HIP_TRY(hipMemcpyAsync(s.q[0], uniq.data(), uniq.size() * sizeof(int32_t), hipMemcpyHostToDevice, st));
    HIP_TRY(hipMemsetAsync(s.ms_vis, 0, n * 8, st));
    HIP_TRY(hipMemsetAsync(s.ms_fr, 0, n * 8, st));
    s.ms_nplanes = 0;
    HIP_TRY(k_ms_seed(s.ms_seeds, nseeds, s.ms_vis, s.ms_fr, INT64_MAX, st));
    HIP_TRY(k_degree_i64(push, s.q[0], static_cast<int64_t>(uniq.size()), s.qdeg, st));
    const uint64_t full = nseeds == 64 ? ~0ULL : ((1ULL << nseeds) - 1ULL);
    const int64_t total = pull.nlists > 1 ? g.out.nnz + g.in.nnz : (a->scope == TGO_SCOPE_IN_E ? g.out.nnz : g.in.nnz);
    static const double ms_alpha = env_double("TGO_MS_ALPHA", 12.0);
    static const bool trace = env_double("TGO_TRACE", 0.0) != 0.0;
    // frontier-bitmap filter of pull levels: measured slower (every pull level: 3.07 -> 3.99 ms,
    // 0.95 -> 1.25, 0.18 -> 0.19; MS-BFS 3146 -> 2471 GTEPS, profiles/r02ad_*): the mask gathers
    // mostly hit L2 / the Infinity Cache already and the probe adds a dependent load.  Opt-in.
    // TGO_MS_FILTER_FROM=H probes the bitmap only for neighbours >= H (the cold ids whose
    // gathers miss L2); TGO_MS_FILTER=1 is H=0, the filter for every neighbour.  Measured on
    // RMAT-24 (profiles/r03h_ms_filter.log): off 5.59 ms/sweep; H = 0 7.05, 128K 6.32, 256K 6.10,
    // 384K 5.93, 1M 5.62 — monotone towards no filter, so the probe's dependent load costs more
    // than the cold gathers it saves.  Off by default.
    static const int32_t filter_from = env_double("TGO_MS_FILTER", 0.0) != 0.0
        ? 0 : static_cast<int32_t>(env_double("TGO_MS_FILTER_FROM", -1.0));
    const bool filter = filter_from >= 0 && filter_from < n;
    // TGO_MS_SPLIT: push budget of the pull levels' sparse sources, as a fraction of the
    // list entries (0 = every source pulled)
    const double split_frac = tgo::ms_split_of(ctx);
    int64_t qlen = static_cast<int64_t>(uniq.size());
    int64_t mf = 0;             // the seeds' entries are not read back: level 0 always pushes (a
                                // direction is policy only; the read cost a stream drain, ~45 us)
    int64_t reached = qlen;     // vertices reached by any source so far
    bool srcent_ready = false;  // ms_srcent holds the current frontier's push entries per source
    static const double push_light = env_double("TGO_MS_PUSH_LIGHT", 1.0 / 16.0);
    static const bool push_probe = env_double("TGO_MS_PUSH_PROBE", 1.0) != 0.0;
    // measured slower at RMAT-24 (second level 446 -> 561 us, profiles/r04t_ms_push_ab.log): off
    static const int push_range_log2 = static_cast<int>(env_double("TGO_MS_PUSH_RANGE", 0.0));
    static const int64_t push_range_min = static_cast<int64_t>(env_double("TGO_MS_PUSH_RANGE_MIN", 1048576.0));
    const int depth = std::min(a->max_depth, 65534);
    uint64_t* fr = s.ms_fr;
    uint64_t* nx = s.ms_nx;
    int cur = 0, levels = 0;
    bool queued = true;         // q[cur] holds the frontier (pull levels only count it)
    bool pulled = false;        // the previous level pulled
    bool cnt_zero = false;      // the counters were zeroed after the last publish
    for (int L = 0; L < depth && qlen > 0; ++L) {
        const bool use_pull = static_cast<double>(mf) * ms_alpha > static_cast<double>(total);
        DevSpan span(st, "msbfs.level", {"level", L}, {"pull", use_pull ? 1 : 0});
        if ((rc = ms_planes_for(ctx, L + 1))) return rc;
        const bool queued_before = queued;
        if (!use_pull && !queued) {     // the frontier's queue, for the push level's scan
            HIP_TRY(hipMemsetAsync(s.cnt, 0, sizeof(Counters), st));
            HIP_TRY(k_ms_queue(push, g.n_active, fr, s.q[cur], s.qdeg, s.cnt, st));
        }
        queued = !use_pull;
        const bool prev_pull = pulled;
        pulled = use_pull;
        bool sums = false;          // this push level's settle sums the per-source entries
        if (!use_pull && !queued_before) cnt_zero = false;      // ms_queue counted into them
        if (use_pull) {
            if (!cnt_zero) HIP_TRY(hipMemsetAsync(s.cnt, 0, sizeof(Counters), st));
            // Split the sources: the pull's walk of a vertex stops once every open source is
            // covered, and one source whose frontier never reaches the vertex (a source far
            // from it, or one whose sweep is over) makes every walk scan its whole list.  The
            // sources with the smallest frontiers (exact push entries per source, within a
            // budget of split_frac of the list entries; every source with an empty frontier)
            // are pushed into candidate masks instead, and the pull covers only the rest.
            // (tried at the first pull level of a run of pull levels, where the frontiers
            // are most unequal; later pull levels found nothing to split on RMAT-24)
            uint64_t sparse = 0;
            if (split_frac > 0.0 && !prev_pull) {
                // every source's exact push entries in one pass, then the smallest within the budget
                // after a push level its settle summed them already (srcent_ready)
                if (!srcent_ready) HIP_TRY(k_ms_source_entries(push, fr, g.n_active, full, s.ms_srcent, st));
                static const bool srcent_check = env_double("TGO_MS_SRCENT_CHECK", 0.0) != 0.0;
                if (srcent_ready && srcent_check) {     // dev check: the settle's sums = a pass of their own
                    HIP_TRY(k_ms_source_entries(push, fr, g.n_active, full, s.ms_stat, st));
                    unsigned long long x[2][TGO_MAX_SOURCES];
                    HIP_TRY(hipMemcpyAsync(x[0], s.ms_srcent, sizeof(x[0]), hipMemcpyDeviceToHost, st));
                    HIP_TRY(hipMemcpyAsync(x[1], s.ms_stat, sizeof(x[1]), hipMemcpyDeviceToHost, st));
                    HIP_TRY(hipStreamSynchronize(st));
                    if (std::memcmp(x[0], x[1], sizeof(x[0])) != 0)
                        return fail(ctx, TGO_E_HIP, "multi-source BFS: settle per-source entries differ from ms_source_entries");
                    if (trace) std::fprintf(stderr, "[tgo] ms level %d: settle per-source entries checked\n", L);
                }
                unsigned long long se[TGO_MAX_SOURCES];
                HIP_TRY(hipMemcpyAsync(se, s.ms_srcent, sizeof(se), hipMemcpyDeviceToHost, st));
                HIP_TRY(hipStreamSynchronize(st));
                int order[TGO_MAX_SOURCES];
                for (int r = 0; r < nseeds; ++r) order[r] = r;
                std::sort(order, order + nseeds, [&](int a, int b) { return se[a] < se[b]; });
                const double budget = split_frac * static_cast<double>(total);
                double used = 0.0;
                for (int i = 0; i < nseeds; ++i) {
                    const int r = order[i];
                    if (used + static_cast<double>(se[r]) > budget) break;
                    used += static_cast<double>(se[r]);
                    sparse |= 1ULL << r;
                }
                if (sparse == full) sparse = 0;            // nothing left to pull: plain pull
                if (sparse) {
                    bool any = false;
                    for (int r = 0; r < nseeds; ++r) any |= ((sparse >> r) & 1ULL) && se[r] > 0;
                    HIP_TRY(hipMemsetAsync(nx, 0, g.n_active * 8, st));
                    if (any) {                           // push the sparse sources' frontiers
                        HIP_TRY(hipMemsetAsync(s.cnt, 0, sizeof(Counters), st));
                        HIP_TRY(k_ms_queue(push, g.n_active, fr, s.q[cur ^ 1], s.qdeg, s.cnt, st, sparse));
                        if ((rc = read_counters(ctx))) return rc;
                        const int64_t sq = static_cast<int64_t>(s.hcnt->qlen);
                        HIP_TRY(hipMemsetAsync(s.cnt, 0, sizeof(Counters), st));
                        if (sq > 0) {
                            if ((rc = scan_frontier(ctx, sq))) return rc;
                            HIP_TRY(k_ms_push(push, s.q[cur ^ 1], s.qpre, sq, fr, s.ms_vis, nx, st, PackTouch{}, sparse));
                        }
                    }
                    if (trace) std::fprintf(stderr, "[tgo] ms level %d split: %d sparse sources, %.0f push entries\n", L,
                                            __builtin_popcountll(sparse), used);
                }
            }
            if (filter) HIP_TRY(k_ms_fbitmap(fr, n, s.ms_fbm, st));
            // The first pull level of a run walks long lists to their end (its frontiers are the
            // most unequal: few walks are covered early).  Opt-in split (TGO_TUNE_MS_COLD /
            // TGO_MS_COLD=1): the walk covers the hot head only, a blocked pass over the cold
            // entries in (segment, row) order ORs the open rows' cold masks from L2, ms_finish
            // settles those rows — same masks, same result.  Measured slower at RMAT-24 (level 2
            // 2.01 -> 2.69 ms, sweep 4.54 -> 5.22 ms, gpurun_out/r04m): of the level's 227 M
            // gathers only 44 M are cold (profiles/r04l_ms_diag.log), and the pass streams every
            // cold entry of every row to reach them.
            MsColdSplit cs;
            static const bool cold_env = env_double("TGO_MS_COLD", 0.0) != 0.0;
            const bool cold_on = ctx->ms_cold < 0 ? cold_env : ctx->ms_cold != 0;
            if (cold_on && !prev_pull && !filter) {
                if ((rc = ms_cold_layout(ctx, a->scope, pull, ctx->ms_cold))) return rc;
                if (g.msc_C > 0) {
                    cs.hot_lim = g.msc_hot;
                    cs.acc = s.ms_cacc;
                    cs.need = s.ms_need;
                }
            }
            HIP_TRY(k_ms_pull(pull, push, g.n_active, full, fr, filter ? s.ms_fbm : nullptr, s.ms_vis, nx,
                              ms_planes(ctx), s.cnt, L + 1, st, filter ? filter_from : 0, full & ~sparse,
                              sparse ? nx : nullptr, cs));
            if (cs.acc) {
                HIP_TRY(k_ms_cold(g.msc_adj, g.msc_row, g.msc_C, fr, s.ms_need, s.ms_cacc, st));
                HIP_TRY(k_ms_finish(push, g.n_active, full, s.ms_vis, nx, sparse ? nx : nullptr, ms_planes(ctx), s.cnt,
                                    L + 1, s.ms_need, s.ms_cacc, st));
            }
        } else {
            // candidates only land on rows with entries (< n_active); the tail is never read
            // one kernel zeroes the counters, the candidate masks and the scan's tail entry
            // (three fills of ~5 us launch each before)
            HIP_TRY(k_level_prep(s.cnt, nx, g.n_active, s.qdeg + qlen, st));
            // A small frontier of long lists pushes target-ranged (k_ms_push_ranged: XCD x on
            // the x-th eighth of the (target range, entry) enumeration, its ranges' masks in
            // its L2); TGO_MS_PUSH_RANGE = log2 of the range (0 = off).
            const int64_t rng = static_cast<int64_t>(1) << std::min(40, std::max(0, push_range_log2));
            const int64_t nr = (g.n_active + rng - 1) / rng;
            const bool ranged = push_range_log2 > 0 && mf >= push_range_min && nr > 1 &&
                                (nr + 1) * qlen <= kMsRangePairs && nr * qlen + 1 <= n + 2;
            if (ranged) {
                for (int b = 0; b < 2; ++b)
                    if (!s.ms_rp[b]) HIP_TRY(dev_alloc(ctx, s.ms_rp[b], kMsRangePairs));
                const bool light = static_cast<double>(reached) < push_light * static_cast<double>(n);
                HIP_TRY(k_ms_push_ranged(push, s.q[cur], qlen, g.n_active, rng, s.ms_rp[0], s.ms_rp[1], s.qdeg, s.qpre,
                                         s.cub_tmp, s.cub_bytes, fr, light ? nullptr : s.ms_vis, nx, st));
            } else {
            HIP_TRY(scan_exclusive_i64(s.cub_tmp, s.cub_bytes, s.qdeg, s.qpre, qlen + 1, st));   // tail zeroed above
            // While few vertices are reached the push skips the reached-mask read of its
            // targets (ms_settle drops the reached bits anyway): one random 8-byte read less
            // per entry at the second level's 12.7 M entries (RMAT-24).  TGO_MS_PUSH_PROBE=0
            // also drops the read of the candidate mask before the atomic there.
            const bool light = static_cast<double>(reached) < push_light * static_cast<double>(n);
            HIP_TRY(k_ms_push(push, s.q[cur], s.qpre, qlen, fr, light ? nullptr : s.ms_vis, nx, st, PackTouch{}, ~0ULL,
                              light ? push_probe : true));
            }
            // the new frontier's push entries per source, for the next level's split — when that
            // level may pull (this frontier's entries within 64x of the pull threshold; a
            // frontier grows at most ~40x a level on RMAT-24), else the split computes them
            // (level 0: the seeds' entries are not known, so always)
            sums = split_frac > 0.0 && (L == 0 || static_cast<double>(mf) * ms_alpha * 64.0 > static_cast<double>(total));
            if (sums) HIP_TRY(hipMemsetAsync(s.ms_srcent, 0, 64 * sizeof(unsigned long long), st));
            // a frontier within 8x of the pull threshold: the next level will likely pull and
            // needs no queue — settle and count only (ms_queue builds it if the level pushes)
            const bool next_pull = static_cast<double>(mf) * ms_alpha * 8.0 > static_cast<double>(total);
            if (next_pull) {
                HIP_TRY(k_ms_settle_count(push, g.n_active, s.ms_vis, nx, ms_planes(ctx), s.cnt, L + 1, st,
                                          sums ? s.ms_srcent : nullptr));
                queued = false;
            } else {
                HIP_TRY(k_ms_settle(push, g.n_active, s.ms_vis, nx, ms_planes(ctx), s.q[cur ^ 1], s.qdeg, s.cnt, L + 1,
                                    st, sums ? s.ms_srcent : nullptr));
            }
        }
        srcent_ready = !use_pull && sums;
        {
            // publish the counts, then queue the next level's direction-independent prefix (its
            // level planes, zeroed counters) before the host waits: the GPU runs it during the
            // host's round trip (≈ 10–25 us a level)
            const unsigned long long seq = ++s.pub_seq;
            HIP_TRY(k_publish_counters(s.cnt, s.hcnt_dev, seq, st));
            if (L + 1 < depth) {
                if ((rc = ms_planes_for(ctx, L + 2))) return rc;
                HIP_TRY(hipMemsetAsync(s.cnt, 0, sizeof(Counters), st));
                cnt_zero = true;
            }
            if ((rc = wait_publish(ctx, seq))) return rc;
        }
        qlen = static_cast<int64_t>(s.hcnt->qlen);
        mf = static_cast<int64_t>(s.hcnt->mf);
        reached += qlen;
        if (trace) std::fprintf(stderr, "[tgo] ms level %d %s -> %lld vertices, %lld entries, %llu source-bits\n", L,
                                use_pull ? "pull" : "push", (long long)qlen, (long long)mf, s.hcnt->red[0]);
        static const bool diag = env_double("TGO_MS_DIAG", 0.0) != 0.0;
        if (trace && diag && use_pull) {
            unsigned long long d[10] = {};
            HIP_TRY(k_ms_diag_take(d, st));
            std::fprintf(stderr, "[tgo]   pull: %llu entries examined, %llu hot / %llu cold mask gathers, %llu open vertices, "
                         "%llu stopped early; long lists: %llu, %llu entries examined (%llu hot / %llu cold gathers), "
                         "%llu stopped early\n", d[0], d[1], d[2], d[3], d[4], d[6], d[5], d[8], d[9], d[7]);
        }
        std::swap(fr, nx);
        cur ^= 1;
        ++levels;
    }
    if (qlen > 0 && a->max_depth > depth)
        return fail(ctx, TGO_E_UNSUPPORTED, "multi-source BFS stores levels as uint16: depth > 65534");
    HIP_TRY(hipEventRecord(ctx->ev1, st));
    HIP_TRY(hipEventSynchronize(ctx->ev1));
    trace_resolve(st);
    float ms = 0;
    HIP_TRY(hipEventElapsedTime(&ms, ctx->ev0, ctx->ev1));
    ctx->st.last_kernel_ms = ms;
    ctx->st.levels = levels;
    ctx->st.iterations = a->max_depth;
    if (a->flags & TGO_FLAG_STATS) {
        HIP_TRY(hipMemsetAsync(s.ms_stat, 0, 2 * TGO_MAX_SOURCES * sizeof(unsigned long long), st));
        HIP_TRY(k_ms_reach(pull, s.ms_vis, n, nseeds, s.ms_stat, s.ms_stat + TGO_MAX_SOURCES, st));
        HIP_TRY(hipStreamSynchronize(st));
    }
    if (dist_out)
        for (int r = 0; r < nseeds; ++r) {
            HIP_TRY(k_ms_extract(ms_planes(ctx), s.ms_nplanes, s.ms_vis, g.perm, r, s.msg, n, st));
            HIP_TRY(hipMemcpyAsync(dist_out + static_cast<int64_t>(r) * n, s.msg, n * sizeof(int64_t),
                                   hipMemcpyDeviceToHost, st));
            HIP_TRY(hipStreamSynchronize(st));
        }
    return TGO_OK;
}

int tgo_copy_multi_distances(tgo_ctx* ctx, int32_t source, int64_t* dist_out) {
    if (!ctx || !dist_out) return TGO_E_INVALID;
    Scratch& s = ctx->sc;
    if (!ctx->loaded || !s.ms_vis) return fail(ctx, TGO_E_STATE, "no multi-source BFS has run");
    if (source < 0 || source >= s.ms_nsrc) return fail(ctx, TGO_E_INVALID, "source index out of range");
    (void)hipSetDevice(ctx->opts.device);
    HIP_TRY(k_ms_extract(ms_planes(ctx), s.ms_nplanes, s.ms_vis, ctx->g.perm, source, s.msg, ctx->g.n, ctx->stream));
    HIP_TRY(hipMemcpyAsync(dist_out, s.msg, ctx->g.n * sizeof(int64_t), hipMemcpyDeviceToHost, ctx->stream));
    HIP_TRY(hipStreamSynchronize(ctx->stream));
    return TGO_OK;
}

int tgo_multi_stats(tgo_ctx* ctx, int64_t* reached, int64_t* reached_entries) {
    if (!ctx) return TGO_E_INVALID;
    Scratch& s = ctx->sc;
    if (!ctx->loaded || !s.ms_vis) return fail(ctx, TGO_E_STATE, "no multi-source BFS has run");
    (void)hipSetDevice(ctx->opts.device);
    std::vector<unsigned long long> h(2 * TGO_MAX_SOURCES);
    HIP_TRY(hipMemcpy(h.data(), s.ms_stat, h.size() * sizeof(unsigned long long), hipMemcpyDeviceToHost));
    for (int r = 0; r < s.ms_nsrc; ++r) {
        if (reached) reached[r] = static_cast<int64_t>(h[r]);
        if (reached_entries) reached_entries[r] = static_cast<int64_t>(h[TGO_MAX_SOURCES + r]);
    }
    return TGO_OK;
}

int tgo_copy_distances(tgo_ctx* ctx, int64_t* dist_out) {
    if (!ctx || !dist_out) return TGO_E_INVALID;
    if (!ctx->loaded) return fail(ctx, TGO_E_STATE, "no graph loaded");
    HIP_TRY(hipStreamSynchronize(ctx->stream));
    HIP_TRY(k_unpermute_i64(ctx->sc.dist, ctx->g.perm, ctx->sc.msg, ctx->g.n, ctx->stream));
    HIP_TRY(hipMemcpyAsync(dist_out, ctx->sc.msg, ctx->g.n * sizeof(int64_t), hipMemcpyDeviceToHost, ctx->stream));
    HIP_TRY(hipStreamSynchronize(ctx->stream));
    return TGO_OK;
}

int tgo_pagerank(tgo_ctx* ctx, const tgo_pr_args* a, double* pr_out) {
    if (!ctx) return TGO_E_INVALID;
    ctx->res_kind = -1;
    if (!a) return fail(ctx, TGO_E_INVALID, "null args");
    if (!ctx->loaded) return fail(ctx, TGO_E_STATE, "no graph loaded");
    if (ctx->g.scope == TGO_SCOPE_BOTH_E)
        return fail(ctx, TGO_E_INVALID, "PageRank uses the inE/outE scopes; load the graph with a single-direction scope");
    if (a->max_iterations < 0) return fail(ctx, TGO_E_INVALID, "max_iterations < 0");
    // PageRankVertexProgram has no combiner: two messages of one scope meeting at a vertex cut
    // hit FulgoraUtil's ThrowingCombiner (:80-91) and the job fails.  Iteration 1 receives the
    // inE messages over OUT entries, iterations >= 2 the outE messages over IN entries.
    if ((a->max_iterations >= 1 && ctx->pv_max_out >= 2) || (a->max_iterations >= 2 && ctx->pv_max_in >= 2))
        return fail(ctx, TGO_E_PROGRAM, "The VertexProgram needs to define a message combiner in order to "
                                        "preserve memory and handle partitioned vertices");
    (void)hipSetDevice(ctx->opts.device);
    DevGraph& g = ctx->g;
    Scratch& s = ctx->sc;
    const int64_t n = g.n;
    hipStream_t st = ctx->stream;
    HIP_TRY(hipEventRecord(ctx->ev0, st));
    double* edge_count = s.vec[0];
    double* contrib = s.vec[1];
    double* contrib_next = s.vec[2];
    double* pr = reinterpret_cast<double*>(s.dist);    // int64-sized scratch reused for PR
    const double N = static_cast<double>(a->vertex_count);
    ctx->st.exact_reruns = 0;
    const PrTuning tune = pr_tuning();
    bool blocked = g.cold_in_ready && tune.diag_hi <= tune.diag_lo;
    if (a->max_iterations == 0) {
        HIP_TRY(k_fill_f64(pr, NAN, n, st));           // iteration 0 sets no PAGE_RANK property
    } else for (;;) {
        contrib = s.vec[1];
        contrib_next = s.vec[2];
        HIP_TRY(k_pr_init(g.out, edge_count, contrib, pr, 1.0 / N, n, st));
        const double base = (1.0 - a->alpha) / N;
        for (int it = 2; it <= a->max_iterations; ++it) {
            // the PAGE_RANK property is only read after the last superstep: write it there
            double* pr_it = it == a->max_iterations ? pr : nullptr;
            DevSpan span(st, "pagerank.update", {"iteration", it});
            if (blocked) {
                {
                    DevSpan ph(st, "pagerank.window_cold_phase", {"iteration", it});
                    HIP_TRY(k_pr_cold_phase(g.cold_in, contrib, st, it == 2));
                }
                DevSpan ph(st, "pagerank.hot_phase", {"iteration", it});
                HIP_TRY(k_pr_hot_phase(g.cold_in, contrib, edge_count, pr_it, contrib_next, s.partial, a->alpha, base,
                                       st, it == 2));
            } else
                HIP_TRY(k_pr_iter(g.in, g.rb_in, contrib, edge_count, pr_it, contrib_next, s.partial, a->alpha, base,
                                  n, tune, st));
            std::swap(contrib, contrib_next);
        }
        if (blocked && a->max_iterations >= 2 && g.cold_in.n_rows < n)   // entry-less rows: PR = (1-a)/N
            HIP_TRY(k_fill_f64(pr + g.cold_in.n_rows, base, n - g.cold_in.n_rows, st));
        // a message outside the fixed-point passes' exact range (an infinity from edgeCount 0,
        // NaN, or a magnitude the 128-bit form cannot hold): the whole program again on the
        // plain fp64 gather, whose sums are Java double sums
        bool bad = false;
        if (blocked && a->max_iterations >= 2)
            if (int rc = fx_take_bad(ctx, g.cold_in, &bad)) return rc;
        if (!bad) break;
        blocked = false;
        ++ctx->st.exact_reruns;
    }
    HIP_TRY(hipEventRecord(ctx->ev1, st));
    HIP_TRY(hipEventSynchronize(ctx->ev1));
    trace_resolve(st);
    float ms = 0;
    HIP_TRY(hipEventElapsedTime(&ms, ctx->ev0, ctx->ev1));
    ctx->st.last_kernel_ms = ms;
    ctx->st.iterations = a->max_iterations;
    if (pr_out) {
        HIP_TRY(k_unpermute_i64(reinterpret_cast<const int64_t*>(pr), g.perm, s.msg, n, st));
        HIP_TRY(hipMemcpyAsync(pr_out, s.msg, n * sizeof(double), hipMemcpyDeviceToHost, st));
        HIP_TRY(hipStreamSynchronize(st));
    }
    ctx->res_kind = TGO_RESULT_PAGERANK;
    ctx->res_empty = a->max_iterations == 0;        // PAGE_RANK / OUTGOING_EDGE_COUNT set at iteration 1
    ctx->res_src = ResultSource{pr, edge_count};
    return TGO_OK;
}

int tgo_walkcount(tgo_ctx* ctx, int32_t k, int32_t* out) {
    if (!ctx) return TGO_E_INVALID;
    ctx->res_kind = -1;
    if (!ctx->loaded) return fail(ctx, TGO_E_STATE, "no graph loaded");
    if (k <= 0) return fail(ctx, TGO_E_INVALID, "DegreeCounter length must be > 0");   // OLAPTest.java:347
    if (ctx->g.scope != TGO_SCOPE_IN_E)
        return fail(ctx, TGO_E_INVALID, "DegreeCounter uses the inE scope; load the graph with TGO_SCOPE_IN_E");
    (void)hipSetDevice(ctx->opts.device);
    DevGraph& g = ctx->g;
    Scratch& s = ctx->sc;
    const int64_t n = g.n;
    hipStream_t st = ctx->stream;
    HIP_TRY(hipEventRecord(ctx->ev0, st));
    int32_t* a = reinterpret_cast<int32_t*>(s.vec[0]);
    int32_t* b = reinterpret_cast<int32_t*>(s.vec[1]);
    HIP_TRY(k_fill_i32(a, 1, n, st));                  // iteration 0: every vertex sends 1
    for (int it = 1; it <= k; ++it) {
        DevSpan span(st, "degree_counter.superstep", {"iteration", it});
        HIP_TRY(k_walk_iter(g.out, g.rb_out, a, b, reinterpret_cast<int32_t*>(s.partial), n, st));
        std::swap(a, b);
    }
    HIP_TRY(hipEventRecord(ctx->ev1, st));
    HIP_TRY(hipEventSynchronize(ctx->ev1));
    trace_resolve(st);
    float ms = 0;
    HIP_TRY(hipEventElapsedTime(&ms, ctx->ev0, ctx->ev1));
    ctx->st.last_kernel_ms = ms;
    ctx->st.iterations = k;
    if (out) {
        HIP_TRY(k_unpermute_i32(a, g.perm, s.level, n, st));
        HIP_TRY(hipMemcpyAsync(out, s.level, n * sizeof(int32_t), hipMemcpyDeviceToHost, st));
        HIP_TRY(hipStreamSynchronize(st));
    }
    ctx->res_kind = TGO_RESULT_DEGREE;
    ctx->res_empty = false;
    ctx->res_src = ResultSource{a, nullptr};
    return TGO_OK;
}

static int result_rows_impl(tgo_ctx* ctx, const tgo_result_args* a, const ResultSource& src, bool empty,
                            tgo_result_size* size, const tgo_rows_buf* out) {
    if (out && (!out->row_keys || !out->row_entry_begin || !out->row_byte_begin || !out->entry_bytes ||
                !out->entry_limit_valpos))
        return fail(ctx, TGO_E_INVALID, "incomplete tgo_rows_buf");
    (void)hipSetDevice(ctx->opts.device);
    const int64_t n = ctx->g.n;
    const tgo_result_size want = *size;
    if (empty) {
        *size = tgo_result_size{0, 0, 0};
        if (out) out->row_entry_begin[0] = out->row_byte_begin[0] = 0;
        return TGO_OK;
    }
    int64_t* scratch[4] = {nullptr, nullptr, nullptr, nullptr};
    auto release = [&] { for (auto* p : scratch) if (p) (void)hipFree(p); };
    for (auto*& p : scratch)
        if (hipMalloc(&p, (n + 1) * sizeof(int64_t)) != hipSuccess) { release(); return fail(ctx, TGO_E_OOM, "result scratch"); }
    ResultRows rr;
    std::vector<int64_t> row_src;
    std::string err;
    int rc = encode_results(src, a, ctx->g.perm, n, scratch, ctx->sc.cub_tmp, ctx->sc.cub_bytes, &rr,
                            ctx->stream, err);
    if (!rc && out) {
        if (want.nrows < rr.nrows || want.nentries < rr.nentries || want.nbytes < rr.nbytes) {
            release();
            *size = tgo_result_size{rr.nrows, rr.nentries, rr.nbytes};
            return fail(ctx, TGO_E_INVALID, "result buffers smaller than the sizes of the first call");
        }
        row_src.resize(static_cast<size_t>(std::max<int64_t>(1, rr.nrows)));
        rr.write = true;
        rr.row_src = row_src.data();
        rr.row_entry_begin = out->row_entry_begin;
        rr.row_byte_begin = out->row_byte_begin;
        rr.entry_bytes = out->entry_bytes;
        rr.entry_limit_valpos = out->entry_limit_valpos;
        rc = encode_results(src, a, ctx->g.perm, n, scratch, ctx->sc.cub_tmp, ctx->sc.cub_bytes, &rr,
                            ctx->stream, err);
        // row keys: IDManager.getKey of each vertex id (IDManager.java:461-473)
        const int pb = ctx->opts.partition_bits;
        for (int64_t i = 0; !rc && i < rr.nrows; ++i) {
            const uint64_t vid = static_cast<uint64_t>(ctx->titan_id[static_cast<size_t>(row_src[i])]);
            const uint64_t part = pb ? (vid >> 3) & ((1ULL << pb) - 1) : 0;
            const uint64_t count = vid >> (3 + pb);
            out->row_keys[i] = static_cast<int64_t>((pb ? part << (64 - pb) : 0) | (count << 3) | (vid & 7));
        }
    }
    release();
    if (rc) return fail(ctx, rc, err);
    *size = tgo_result_size{rr.nrows, rr.nentries, rr.nbytes};
    return TGO_OK;
}

int tgo_result_rows(tgo_ctx* ctx, const tgo_result_args* a, tgo_result_size* size, const tgo_rows_buf* out) {
    if (!ctx) return TGO_E_INVALID;
    if (!a || !size) return fail(ctx, TGO_E_INVALID, "null args");
    if (a->kind < TGO_RESULT_DISTANCE || a->kind > TGO_RESULT_DEGREE) return fail(ctx, TGO_E_INVALID, "invalid result kind");
    if (ctx->res_kind != a->kind)
        return fail(ctx, TGO_E_STATE, "no finished program of that kind is the last one run on this ctx");
    return result_rows_impl(ctx, a, ctx->res_src, ctx->res_empty, size, out);
}

static int generic_alloc(tgo_ctx* ctx);

int tgo_result_rows_values(tgo_ctx* ctx, const tgo_result_args* a, const void* values, const uint8_t* present,
                           tgo_result_size* size, const tgo_rows_buf* out) {
    if (!ctx) return TGO_E_INVALID;
    if (!a || !size || !values || !present) return fail(ctx, TGO_E_INVALID, "null args");
    if (!ctx->loaded) return fail(ctx, TGO_E_STATE, "no graph loaded");
    if (a->kind != TGO_RESULT_VALUES) return fail(ctx, TGO_E_INVALID, "tgo_result_rows_values takes kind TGO_RESULT_VALUES");
    if (ctx->g.partitioned) return fail(ctx, TGO_E_UNSUPPORTED, "generic programs run on a one-GPU load");
    const int64_t n = ctx->g.n;
    if (a->reserved == TGO_VAL_INT64 && a->datatypes[0] == TGO_DT_INTEGER) {
        const int64_t* v = static_cast<const int64_t*>(values);
        for (int64_t i = 0; i < n; ++i)
            if (present[i] && (v[i] < INT32_MIN || v[i] > INT32_MAX))
                return fail(ctx, TGO_E_INVALID, "a value of an Integer compute key is out of int range");
    }
    (void)hipSetDevice(ctx->opts.device);
    int rc = generic_alloc(ctx);
    if (rc) return rc;
    Scratch& s = ctx->sc;
    hipStream_t st = ctx->stream;
    HIP_TRY(hipMemcpyAsync(s.gv[0], values, n * 8, hipMemcpyHostToDevice, st));
    HIP_TRY(hipMemcpyAsync(s.gh[0], present, n, hipMemcpyHostToDevice, st));
    HIP_TRY(k_to_internal(s.gv[0], s.gh[0], ctx->g.perm, s.gv[1], s.gh[1], n, st));
    HIP_TRY(hipStreamSynchronize(st));
    return result_rows_impl(ctx, a, ResultSource{s.gv[1], s.gh[1]}, false, size, out);
}

// ------------------------------------------------------------------ 1-D partitioned (multi-GPU)
int tgo_part_layout(const tgo_edges* edges, int64_t n_global, int64_t lo, int64_t hi, int32_t threads,
                    int32_t* layout_local) {
    if (!edges || !layout_local || (edges->m > 0 && (!edges->src || !edges->dst))) return TGO_E_INVALID;
    std::string err;
    return partition_layout(edges, n_global, lo, hi, threads > 0 ? threads : 1, layout_local, err);
}

int tgo_load_partition(tgo_ctx* ctx, int64_t n_global, int64_t lo, int64_t hi, const tgo_edges* edges,
                       const tgo_load_opts* opts) {
    return tgo_load_partition_layout(ctx, n_global, lo, hi, edges, opts, nullptr);
}

int tgo_load_partition_layout(tgo_ctx* ctx, int64_t n_global, int64_t lo, int64_t hi, const tgo_edges* edges,
                              const tgo_load_opts* opts, const int32_t* layout_global) {
    if (!ctx) return TGO_E_INVALID;
    Span load_span("load.partition");
    TrimTemps trim_temps;   // the build temporaries are released when the load returns
    if (!edges || !opts || (edges->m > 0 && (!edges->src || !edges->dst))) return fail(ctx, TGO_E_INVALID, "null argument");
    if ((hi - lo) % 64 != 0) return fail(ctx, TGO_E_INVALID, "partition size must be a multiple of 64");
    (void)hipSetDevice(ctx->opts.device);
    const auto t0 = std::chrono::steady_clock::now();
    HostGraph h;
    std::string err;
    // device assembly (assemble.hip) unless TGO_HOST_ASSEMBLY=1
    const bool on_dev = env_i64("TGO_HOST_ASSEMBLY", 0) == 0;
    int rc = on_dev ? assemble_partition_device(edges, n_global, lo, hi, opts, ctx->opts.hard_query_limit, layout_global,
                                                h, ctx->stream, err)
                    : assemble_partition(edges, n_global, lo, hi, opts, ctx->opts.hard_query_limit, layout_global, h,
                                         threads_of(ctx), err);
    if (rc == TGO_OK && env_i64("TGO_TRACE", 0))
        std::fprintf(stderr, "[tgo] load_partition assembly (%s) %8.1f ms\n", on_dev ? "device" : "host",
                     std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count());
    if (rc) return fail(ctx, rc, err);
    rc = tgo::part_upload(ctx, h, n_global, lo);
    ctx->st.load_ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
    return rc;
}

static int part_check(tgo_ctx* ctx);


static int part_check(tgo_ctx* ctx) {
    if (!ctx) return TGO_E_INVALID;
    if (!ctx->loaded || !ctx->g.partitioned) return fail(ctx, TGO_E_STATE, "no partitioned graph loaded");
    (void)hipSetDevice(ctx->opts.device);
    return TGO_OK;
}

// Entry points that leave work queued: on a ctx-owned stream the caller cannot order its
// collectives after that work, so finish it before returning; on the caller's stream the
// work stays stream-ordered (the caller's collectives follow it on the same stream).
static int part_done(tgo_ctx* ctx) {
    if (ctx->own_stream) HIP_TRY(hipStreamSynchronize(ctx->stream));
    return TGO_OK;
}

// Level counters {next queue length, its push entries}.  Host mode: read (one stream sync)
// into counts.  Device mode (tgo_part_device_counts): published to the caller's device
// buffer without a sync — the caller all-reduces it and reads the global counts once; the
// local queue length is fetched lazily by the next call that needs it (part_qlen_now).
static int part_counts(tgo_ctx* ctx, int64_t* counts, bool device_ok = true) {
    if (ctx->part_dcounts && device_ok) {
        HIP_TRY(k_publish_counts(ctx->sc.cnt, ctx->part_dcounts, ctx->part_qlen_dev, ctx->stream));
        ctx->part_qlen_stale = true;
        return part_done(ctx);
    }
    int rc = read_counters(ctx);
    if (rc) return rc;
    ctx->part_qlen = static_cast<int64_t>(ctx->sc.hcnt->qlen);
    ctx->part_qlen_stale = false;
    if (counts) {
        counts[0] = ctx->part_qlen;
        counts[1] = static_cast<int64_t>(ctx->sc.hcnt->mf);
    }
    return TGO_OK;
}

static int part_qlen_now(tgo_ctx* ctx, int64_t& q) {
    if (ctx->part_qlen_stale) {
        HIP_TRY(hipMemcpyAsync(&ctx->part_qlen, ctx->part_qlen_dev, sizeof(int64_t), hipMemcpyDeviceToHost, ctx->stream));
        HIP_TRY(hipStreamSynchronize(ctx->stream));
        ctx->part_qlen_stale = false;
    }
    q = ctx->part_qlen;
    return TGO_OK;
}

int tgo_part_device_counts(tgo_ctx* ctx, int64_t* dev_counts) {
    int rc = part_check(ctx);
    if (rc) return rc;
    if (dev_counts) ctx->part_qlen_dev = dev_counts + 2;        // [2]: this rank's queue length
    if (!dev_counts && ctx->part_qlen_stale) {
        int64_t q;
        if ((rc = part_qlen_now(ctx, q))) return rc;
    }
    ctx->part_dcounts = dev_counts;
    return TGO_OK;
}

int tgo_part_set_local_qlen(tgo_ctx* ctx, int64_t qlen) {
    int rc = part_check(ctx);
    if (rc) return rc;
    if (!ctx->part_qlen_stale) return TGO_OK;               // nothing pending
    if (qlen < 0 || qlen > ctx->g.n) return fail(ctx, TGO_E_INVALID, "local queue length out of range");
    ctx->part_qlen = qlen;
    ctx->part_qlen_stale = false;
    return TGO_OK;
}

int tgo_part_bfs_begin(tgo_ctx* ctx, int64_t seed_global, uint64_t* nb_local, int64_t* counts) {
    int rc = part_check(ctx);
    if (rc) return rc;
    if (ctx->g.scope != TGO_SCOPE_BOTH_E) return fail(ctx, TGO_E_UNSUPPORTED, "partitioned BFS runs over bothE");
    DevGraph& g = ctx->g;
    Scratch& s = ctx->sc;
    hipStream_t st = ctx->stream;
    const int64_t n = g.n, words = n / 64;
    const View push = push_view(g, TGO_SCOPE_BOTH_E);
    HIP_TRY(hipEventRecord(ctx->ev0, st));
    HIP_TRY(k_fill_i32(s.level, -1, n, st));
    HIP_TRY(hipMemsetAsync(s.vb, 0, (words + 1) * 8, st));
    HIP_TRY(hipMemsetAsync(nb_local, 0, words * 8, st));
    HIP_TRY(hipMemsetAsync(s.cnt, 0, sizeof(Counters), st));
    ctx->part_cur = 0;
    ctx->part_queued = true;
    ctx->part_qlen = 0;
    ctx->part_qlen_stale = false;
    int64_t deg = 0;
    int64_t seed = seed_global - g.lo;
    if (seed >= 0 && seed < n) {
        seed = ctx->perm[seed];
        // the owner seeds: level 0, visited, in the frontier bitmap slice and the queue
        HIP_TRY(k_bfs_seed(push, s.level, s.vb, nb_local, s.q[0], s.qdeg, seed, st));
        HIP_TRY(hipMemcpyAsync(&deg, s.qdeg, sizeof(int64_t), hipMemcpyDeviceToHost, st));
        ctx->part_qlen = 1;
    }
    HIP_TRY(hipStreamSynchronize(st));
    if (counts) { counts[0] = ctx->part_qlen; counts[1] = deg; }
    return TGO_OK;
}

int tgo_part_bfs_td(tgo_ctx* ctx, int32_t level, uint64_t* disc_global) {
    int rc = part_check(ctx);
    if (rc) return rc;
    (void)level;
    DevGraph& g = ctx->g;
    Scratch& s = ctx->sc;
    hipStream_t st = ctx->stream;
    const View push = push_view(g, TGO_SCOPE_BOTH_E);
    int64_t qlen = 0;
    if ((rc = part_qlen_now(ctx, qlen))) return rc;
    if (qlen > 0 && !ctx->part_queued) {
        HIP_TRY(hipMemsetAsync(s.cnt, 0, sizeof(Counters), st));
        HIP_TRY(k_bfs_queue(push, g.n_active, ctx->part_frontier, s.q[ctx->part_cur], s.qdeg, s.cnt, st));
        ctx->part_queued = true;
    }
    if (qlen > 0) {
        if ((rc = scan_frontier(ctx, ctx->part_qlen))) return rc;
        HIP_TRY(k_part_td_mark(push, s.q[ctx->part_cur], s.qpre, ctx->part_qlen, disc_global, s.vb, g.lo, g.n, st));
    }
    return part_done(ctx);
}

int tgo_part_bfs_claim(tgo_ctx* ctx, int32_t level, const uint64_t* recv, int32_t nslices,
                       uint64_t* nb_local, int64_t* counts) {
    int rc = part_check(ctx);
    if (rc) return rc;
    DevGraph& g = ctx->g;
    Scratch& s = ctx->sc;
    hipStream_t st = ctx->stream;
    const View push = push_view(g, TGO_SCOPE_BOTH_E);
    HIP_TRY(hipMemsetAsync(s.cnt, 0, sizeof(Counters), st));
    const int nxt = ctx->part_cur ^ 1;
    HIP_TRY(k_part_claim(push, recv, nslices, g.n / 64, g.n, s.vb, nb_local, s.level, s.q[nxt], s.qdeg, s.cnt,
                         level + 1, st));
    ctx->part_cur = nxt;
    ctx->part_queued = true;
    return part_counts(ctx, counts);
}

}  // extern "C" (the fused level helpers below are C++, used by part_driver.cpp)
namespace tgo {
// tgo_part_bfs_run's top-down level, fused: the current queue (built from the frontier bitmap
// when the last level was bottom-up), then ONE expansion that claims owned targets in place —
// the one-GPU td_expand — and marks only remote ones in disc; nb_local is zeroed first.  With
// world 1 nothing is remote, and the level needs no exchange and no claim pass over the whole
// bitmap (the C-ABI's td / all-to-all / claim protocol makes two passes over every word).
int part_bfs_td_fused(tgo_ctx* ctx, int32_t level, uint64_t* disc, uint64_t* nb_local) {
    int rc = part_check(ctx);
    if (rc) return rc;
    DevGraph& g = ctx->g;
    Scratch& s = ctx->sc;
    hipStream_t st = ctx->stream;
    const View push = push_view(g, TGO_SCOPE_BOTH_E);
    int64_t qlen = 0;
    if ((rc = part_qlen_now(ctx, qlen))) return rc;
    if (qlen > 0 && !ctx->part_queued) {
        HIP_TRY(hipMemsetAsync(s.cnt, 0, sizeof(Counters), st));
        HIP_TRY(k_bfs_queue(push, g.n_active, ctx->part_frontier, s.q[ctx->part_cur], s.qdeg, s.cnt, st));
        ctx->part_queued = true;
    }
    if (qlen > 0 && (rc = scan_frontier(ctx, qlen))) return rc;
    HIP_TRY(hipMemsetAsync(s.cnt, 0, sizeof(Counters), st));
    HIP_TRY(hipMemsetAsync(nb_local, 0, (g.n / 64) * 8, st));
    const int nxt = ctx->part_cur ^ 1;
    if (qlen > 0)
        HIP_TRY(k_part_td_claim(push, s.q[ctx->part_cur], s.qpre, qlen, disc, s.vb, nb_local, s.level, s.q[nxt], s.qdeg,
                                s.cnt, level + 1, g.lo, g.n, st));
    ctx->part_cur = nxt;
    ctx->part_queued = true;
    return part_done(ctx);
}
// The remote discoveries (received slices) into the queue part_bfs_td_fused started.
int part_bfs_claim_remote(tgo_ctx* ctx, int32_t level, const uint64_t* recv, int32_t nslices, uint64_t* nb_local) {
    int rc = part_check(ctx);
    if (rc) return rc;
    DevGraph& g = ctx->g;
    Scratch& s = ctx->sc;
    const View push = push_view(g, TGO_SCOPE_BOTH_E);
    HIP_TRY(k_part_claim(push, recv, nslices, g.n / 64, g.n, s.vb, nb_local, s.level, s.q[ctx->part_cur], s.qdeg, s.cnt,
                         level + 1, ctx->stream, true));
    return part_done(ctx);
}
// The level's counts (device counts when set, as tgo_part_bfs_claim).
int part_bfs_level_done(tgo_ctx* ctx) { return part_counts(ctx, nullptr); }
}  // namespace tgo
extern "C" {

int tgo_part_bfs_bu(tgo_ctx* ctx, int32_t level, const uint64_t* fb_global, uint64_t* nb_local, int64_t* counts) {
    int rc = part_check(ctx);
    if (rc) return rc;
    DevGraph& g = ctx->g;
    Scratch& s = ctx->sc;
    hipStream_t st = ctx->stream;
    const View pull = pull_view(g, TGO_SCOPE_BOTH_E), push = push_view(g, TGO_SCOPE_BOTH_E);
    HIP_TRY(hipMemsetAsync(s.cnt, 0, sizeof(Counters), st));
    HIP_TRY(hipMemsetAsync(nb_local, 0, (g.n / 64) * 8, st));
    const int nxt = ctx->part_cur ^ 1;
    HIP_TRY(k_bu_step(pull, push, g.n_active, fb_global, s.vb, nb_local, s.level, s.cnt, level + 1, st));
    ctx->part_cur = nxt;
    ctx->part_queued = false;       // counted only: bfs_td queues nb_local if it runs next
    ctx->part_frontier = nb_local;
    return part_counts(ctx, counts);
}

int tgo_part_bfs_end(tgo_ctx* ctx, int64_t* dist_local, int64_t* reached) {
    int rc = part_check(ctx);
    if (rc) return rc;
    DevGraph& g = ctx->g;
    Scratch& s = ctx->sc;
    hipStream_t st = ctx->stream;
    HIP_TRY(k_level_to_dist(s.level, s.dist, g.n, st));
    HIP_TRY(hipEventRecord(ctx->ev1, st));
    if (reached) {
        HIP_TRY(hipMemsetAsync(s.cnt, 0, sizeof(Counters), st));
        HIP_TRY(k_reach_stats(pull_view(g, TGO_SCOPE_BOTH_E), s.dist, g.n, s.cnt->red, st));
        if ((rc = read_counters(ctx))) return rc;
        reached[0] = static_cast<int64_t>(s.hcnt->red[0]);
        reached[1] = static_cast<int64_t>(s.hcnt->red[1]);
    }
    if (dist_local) {   // back to row order
        HIP_TRY(k_unpermute_i64(s.dist, g.perm, s.msg, g.n, st));
        HIP_TRY(hipMemcpyAsync(dist_local, s.msg, g.n * sizeof(int64_t), hipMemcpyDeviceToHost, st));
    }
    HIP_TRY(hipStreamSynchronize(st));
    float ms = 0;
    HIP_TRY(hipEventElapsedTime(&ms, ctx->ev0, ctx->ev1));
    ctx->st.last_kernel_ms = ms;
    return TGO_OK;
}

// ---- partitioned multi-source BFS
int tgo_part_ms_begin(tgo_ctx* ctx, const int64_t* seeds, int32_t nseeds, uint64_t* fr_local, int64_t* counts) {
    int rc = part_check(ctx);
    if (rc) return rc;
    if (!seeds || nseeds < 1 || nseeds > TGO_MAX_SOURCES) return fail(ctx, TGO_E_INVALID, "nseeds must be in [1, 64]");
    if (ctx->g.scope != TGO_SCOPE_BOTH_E) return fail(ctx, TGO_E_UNSUPPORTED, "partitioned BFS runs over bothE");
    if ((rc = ms_alloc(ctx))) return rc;
    DevGraph& g = ctx->g;
    Scratch& s = ctx->sc;
    hipStream_t st = ctx->stream;
    const int64_t n = g.n;
    const View push = push_view(g, TGO_SCOPE_BOTH_E);
    // owned seeds, as local ids; sources keep their global bit position r
    std::vector<int64_t> local(nseeds, -1);
    std::vector<int32_t> uniq;
    for (int r = 0; r < nseeds; ++r) {
        int64_t l = seeds[r] - g.lo;
        if (l >= 0 && l < n) {
            l = ctx->perm[l];
            local[r] = l;
            if (std::find(uniq.begin(), uniq.end(), static_cast<int32_t>(l)) == uniq.end()) uniq.push_back(static_cast<int32_t>(l));
        }
    }
    s.ms_nsrc = nseeds;
    HIP_TRY(hipEventRecord(ctx->ev0, st));
    HIP_TRY(hipMemsetAsync(s.ms_vis, 0, n * 8, st));
    HIP_TRY(hipMemsetAsync(fr_local, 0, n * 8, st));
    if (!s.pk_ovf) HIP_TRY(dev_alloc(ctx, s.pk_ovf, 1));
    HIP_TRY(hipMemsetAsync(s.pk_ovf, 0, sizeof(int), st));
    const int64_t touch_n = g.n_global / kPackChunk + kMaxRanks + 1;
    if (!s.pk_touch) HIP_TRY(dev_alloc(ctx, s.pk_touch, touch_n));
    HIP_TRY(hipMemsetAsync(s.pk_touch, 0, touch_n, st));
    s.ms_nplanes = 0;
    // seeds owned elsewhere stay -1 (skipped by the seed kernel; their bit is set by the owner)
    HIP_TRY(hipMemcpyAsync(s.ms_seeds, local.data(), nseeds * sizeof(int64_t), hipMemcpyHostToDevice, st));
    // entry-less seeds stay out of the masks: the pull levels never write the masks' tail
    // [n_active, n), which therefore stays zero in both alternating buffers
    HIP_TRY(k_ms_seed(s.ms_seeds, nseeds, s.ms_vis, fr_local, g.n_active, st));
    ctx->part_cur = 0;
    ctx->part_queued = true;
    ctx->part_qlen = static_cast<int64_t>(uniq.size());
    ctx->part_qlen_stale = false;
    int64_t mf = 0;
    if (!uniq.empty()) {
        HIP_TRY(hipMemcpyAsync(s.q[0], uniq.data(), uniq.size() * sizeof(int32_t), hipMemcpyHostToDevice, st));
        HIP_TRY(k_degree_i64(push, s.q[0], static_cast<int64_t>(uniq.size()), s.qdeg, st));
        std::vector<int64_t> d(uniq.size());
        HIP_TRY(hipMemcpyAsync(d.data(), s.qdeg, d.size() * sizeof(int64_t), hipMemcpyDeviceToHost, st));
        HIP_TRY(hipStreamSynchronize(st));
        for (int64_t x : d) mf += x;
    }
    HIP_TRY(hipStreamSynchronize(st));
    if (counts) { counts[0] = ctx->part_qlen; counts[1] = mf; }
    return TGO_OK;
}

// ---- source split of a dense level (tgo_bfs_multi's split, partitioned; titan_gpu_olap_part.h)
int tgo_part_ms_source_counts(tgo_ctx* ctx, const uint64_t* fr_local, int64_t* counts_dev) {
    int rc = part_check(ctx);
    if (rc) return rc;
    if (!fr_local || !counts_dev) return fail(ctx, TGO_E_INVALID, "null argument");
    HIP_TRY(k_ms_source_counts(fr_local, ctx->g.n_active, reinterpret_cast<unsigned long long*>(counts_dev), ctx->stream));
    return part_done(ctx);
}

int tgo_part_ms_source_entries(tgo_ctx* ctx, const uint64_t* fr_local, uint64_t cand, int64_t* entries_dev) {
    int rc = part_check(ctx);
    if (rc) return rc;
    if (!fr_local || !entries_dev) return fail(ctx, TGO_E_INVALID, "null argument");
    HIP_TRY(k_ms_source_entries(push_view(ctx->g, TGO_SCOPE_BOTH_E), fr_local, ctx->g.n_active, cand,
                                reinterpret_cast<unsigned long long*>(entries_dev), ctx->stream));
    return part_done(ctx);
}

// The sparse sources' frontiers pushed into cand_global: a masked queue of this rank's
// frontier in the idle queue buffer (a dense level builds no queue), the pack's touch flags.
int tgo_part_ms_push_masked(tgo_ctx* ctx, const uint64_t* fr_local, uint64_t* cand_global, uint64_t mask) {
    int rc = part_check(ctx);
    if (rc) return rc;
    if (!fr_local || !cand_global) return fail(ctx, TGO_E_INVALID, "null argument");
    DevGraph& g = ctx->g;
    Scratch& s = ctx->sc;
    hipStream_t st = ctx->stream;
    const View push = push_view(g, TGO_SCOPE_BOTH_E);
    int32_t* q = s.q[ctx->part_cur ^ 1];
    HIP_TRY(hipMemsetAsync(s.cnt, 0, sizeof(Counters), st));
    HIP_TRY(k_ms_queue(push, g.n_active, fr_local, q, s.qdeg, s.cnt, st, mask));
    if ((rc = read_counters(ctx))) return rc;
    const int64_t qlen = static_cast<int64_t>(s.hcnt->qlen);
    if (qlen > 0) {
        if ((rc = scan_frontier(ctx, qlen))) return rc;
        const PackTouch touch{s.pk_touch, g.n, (g.n + kPackChunk - 1) / kPackChunk};
        HIP_TRY(k_ms_push(push, q, s.qpre, qlen, fr_local, nullptr, cand_global, st, touch, mask));
    }
    return part_done(ctx);
}

// The received candidate pairs OR-ed into fr_next (zeroed first), no settle: the pull of the
// same level reads them (tgo_part_ms_pull_split).
// With the own-slice bypass on: this rank's candidate words into the owned next masks.
static hipError_t ms_or_own(tgo_ctx* ctx, uint64_t* fr_next) {
    if (ctx->part_ms_self < 0 || !ctx->part_ms_cand) return hipSuccess;
    const int64_t nl = ctx->g.n, cps = (nl + kPackChunk - 1) / kPackChunk;
    uint8_t* touched = ctx->sc.pk_touch ? ctx->sc.pk_touch + static_cast<int64_t>(ctx->part_ms_self) * cps : nullptr;
    return k_ms_or_local(ctx->part_ms_cand + static_cast<int64_t>(ctx->part_ms_self) * nl, nl, cps, touched, fr_next,
                         ctx->stream);
}

int tgo_part_ms_or_fixed(tgo_ctx* ctx, const int64_t* recv, int32_t nslices, int64_t cap, uint64_t* fr_next) {
    int rc = part_check(ctx);
    if (rc) return rc;
    if (!recv || !fr_next || nslices < 1 || nslices > kMaxRanks || cap < 1 || cap > ctx->g.n)
        return fail(ctx, TGO_E_INVALID, "ms_or_fixed: bad arguments");
    HIP_TRY(hipMemsetAsync(fr_next, 0, ctx->g.n_active * 8, ctx->stream));
    HIP_TRY(k_ms_or_fixed(recv, nslices, cap, fr_next, ctx->stream));
    HIP_TRY(ms_or_own(ctx, fr_next));
    return part_done(ctx);
}

int tgo_part_ms_or_pairs(tgo_ctx* ctx, const int64_t* recv, const int64_t* recv_counts, int32_t nslices,
                         uint64_t* fr_next) {
    int rc = part_check(ctx);
    if (rc) return rc;
    if (!recv || !recv_counts || !fr_next || nslices < 1 || nslices > kMaxRanks)
        return fail(ctx, TGO_E_INVALID, "ms_or_pairs: bad arguments");
    int64_t npairs = 0;
    for (int r = 0; r < nslices; ++r) {
        if (recv_counts[r] < 0 || recv_counts[r] > ctx->g.n) return fail(ctx, TGO_E_INVALID, "ms_or_pairs: bad count");
        npairs += recv_counts[r];
    }
    HIP_TRY(hipMemsetAsync(fr_next, 0, ctx->g.n_active * 8, ctx->stream));
    HIP_TRY(k_ms_or_pairs(recv, npairs, fr_next, ctx->stream));
    HIP_TRY(ms_or_own(ctx, fr_next));
    return part_done(ctx);
}

int tgo_part_ms_pull_split(tgo_ctx* ctx, int32_t level, const uint64_t* fr_global, uint64_t* fr_next, uint64_t sparse,
                           int32_t cand_in_next, int64_t* counts) {
    int rc = part_check(ctx);
    if (rc) return rc;
    DevGraph& g = ctx->g;
    Scratch& s = ctx->sc;
    hipStream_t st = ctx->stream;
    const View pull = pull_view(g, TGO_SCOPE_BOTH_E), push = push_view(g, TGO_SCOPE_BOTH_E);
    const uint64_t full = s.ms_nsrc == 64 ? ~0ULL : ((1ULL << s.ms_nsrc) - 1ULL);
    if (level + 1 >= (1 << kLevelPlanes)) return fail(ctx, TGO_E_UNSUPPORTED, "multi-source BFS levels are < 65536");
    if ((rc = ms_planes_for(ctx, level + 1))) return rc;
    HIP_TRY(hipMemsetAsync(s.cnt, 0, sizeof(Counters), st));
    const int nxt = ctx->part_cur ^ 1;
    HIP_TRY(k_ms_pull(pull, push, g.n_active, full, fr_global, nullptr, s.ms_vis, fr_next, ms_planes(ctx), s.cnt,
                      level + 1, st, 0, full & ~sparse, cand_in_next ? fr_next : nullptr));
    ctx->part_cur = nxt;
    ctx->part_queued = false;
    return part_counts(ctx, counts);
}

int tgo_part_ms_pull(tgo_ctx* ctx, int32_t level, const uint64_t* fr_global, uint64_t* fr_next, int64_t* counts) {
    int rc = part_check(ctx);
    if (rc) return rc;
    DevGraph& g = ctx->g;
    Scratch& s = ctx->sc;
    hipStream_t st = ctx->stream;
    const View pull = pull_view(g, TGO_SCOPE_BOTH_E), push = push_view(g, TGO_SCOPE_BOTH_E);
    const uint64_t full = s.ms_nsrc == 64 ? ~0ULL : ((1ULL << s.ms_nsrc) - 1ULL);
    if (level + 1 >= (1 << kLevelPlanes)) return fail(ctx, TGO_E_UNSUPPORTED, "multi-source BFS levels are < 65536");
    if ((rc = ms_planes_for(ctx, level + 1))) return rc;
    HIP_TRY(hipMemsetAsync(s.cnt, 0, sizeof(Counters), st));
    // the pull writes every active row's mask; the entry-less tail is zero already (no
    // entry-less seed enters a mask, tgo_part_ms_begin)
    const int nxt = ctx->part_cur ^ 1;
    HIP_TRY(k_ms_pull(pull, push, g.n_active, full, fr_global, nullptr, s.ms_vis, fr_next, ms_planes(ctx), s.cnt,
                      level + 1, st, 0));
    ctx->part_cur = nxt;
    ctx->part_queued = false;       // counted only: ms_push builds the queue if it needs one
    return part_counts(ctx, counts);
}

int tgo_part_ms_push(tgo_ctx* ctx, int32_t level, const uint64_t* fr_local, uint64_t* cand_global) {
    int rc = part_check(ctx);
    if (rc) return rc;
    (void)level;
    DevGraph& g = ctx->g;
    Scratch& s = ctx->sc;
    int64_t qlen = 0;
    if ((rc = part_qlen_now(ctx, qlen))) return rc;
    if (qlen > 0 && !ctx->part_queued) {
        HIP_TRY(hipMemsetAsync(s.cnt, 0, sizeof(Counters), ctx->stream));
        HIP_TRY(k_ms_queue(push_view(g, TGO_SCOPE_BOTH_E), g.n_active, fr_local, s.q[ctx->part_cur], s.qdeg, s.cnt,
                           ctx->stream));
        ctx->part_queued = true;
    }
    // bypass on and the next masks named (part_ms_own_next): the owned targets' candidates go
    // straight into them (zeroed here), so the settle neither zeroes them nor ORs the own slice
    uint64_t* own = nullptr;
    int64_t own_lo = 0;
    if (ctx->part_own_next && ctx->part_ms_self >= 0 && cand_global == ctx->part_ms_cand) {
        own = ctx->part_own_next;
        own_lo = static_cast<int64_t>(ctx->part_ms_self) * g.n;
        HIP_TRY(k_level_prep(nullptr, own, g.n_active, nullptr, ctx->stream));   // the tail stays zero
    }
    ctx->part_own_next = nullptr;
    ctx->part_own_direct = own;
    if (qlen > 0) {
        if ((rc = scan_frontier(ctx, ctx->part_qlen))) return rc;
        const PackTouch touch{s.pk_touch, g.n, (g.n + kPackChunk - 1) / kPackChunk};
        HIP_TRY(k_ms_push(push_view(g, TGO_SCOPE_BOTH_E), s.q[ctx->part_cur], s.qpre, ctx->part_qlen, fr_local,
                          nullptr, cand_global, ctx->stream, touch, ~0ULL, true, own, own_lo));
    }
    return part_done(ctx);
}

int tgo_part_ms_settle(tgo_ctx* ctx, int32_t level, const uint64_t* recv, int32_t nslices, uint64_t* fr_next,
                       int64_t* counts) {
    int rc = part_check(ctx);
    if (rc) return rc;
    DevGraph& g = ctx->g;
    Scratch& s = ctx->sc;
    hipStream_t st = ctx->stream;
    if (level + 1 >= (1 << kLevelPlanes)) return fail(ctx, TGO_E_UNSUPPORTED, "multi-source BFS levels are < 65536");
    if ((rc = ms_planes_for(ctx, level + 1))) return rc;
    HIP_TRY(hipMemsetAsync(s.cnt, 0, sizeof(Counters), st));
    HIP_TRY(k_or_slices(recv, nslices, g.n, fr_next, st));
    const int nxt = ctx->part_cur ^ 1;
    if (ctx->part_count_only) {
        HIP_TRY(k_ms_settle_count(push_view(g, TGO_SCOPE_BOTH_E), g.n_active, s.ms_vis, fr_next, ms_planes(ctx), s.cnt,
                                  level + 1, st, ctx->part_srcent));
    } else {
        HIP_TRY(k_ms_settle(push_view(g, TGO_SCOPE_BOTH_E), g.n_active, s.ms_vis, fr_next, ms_planes(ctx), s.q[nxt], s.qdeg,
                            s.cnt, level + 1, st, ctx->part_srcent));
    }
    ctx->part_queued = !ctx->part_count_only;
    ctx->part_srcent = nullptr;
    ctx->part_count_only = false;
    ctx->part_cur = nxt;
    return part_counts(ctx, counts);
}

int tgo_part_ms_pack(tgo_ctx* ctx, uint64_t* cand_global, int32_t nranks, int64_t* send, int64_t* send_counts) {
    int rc = part_check(ctx);
    if (rc) return rc;
    DevGraph& g = ctx->g;
    Scratch& s = ctx->sc;
    if (!cand_global || !send || !send_counts || nranks < 1 || nranks > kMaxRanks ||
        static_cast<int64_t>(nranks) * g.n != g.n_global)
        return fail(ctx, TGO_E_INVALID, "ms_pack: bad arguments (nranks * n_local must equal n_global)");
    hipStream_t st = ctx->stream;
    const int64_t cps = (g.n + kPackChunk - 1) / kPackChunk;     // chunks per slice
    const int64_t nchunks = cps * nranks;
    if (!s.pk_cnt) {
        HIP_TRY(dev_alloc(ctx, s.pk_cnt, g.n_global / kPackChunk + kMaxRanks + 1));
        HIP_TRY(dev_alloc(ctx, s.pk_off, g.n_global / kPackChunk + kMaxRanks + 1));
    }
    HIP_TRY(hipMemsetAsync(s.pk_cnt + nchunks, 0, sizeof(int64_t), st));
    HIP_TRY(k_ms_pack(false, cand_global, g.n, cps, nchunks, s.pk_cnt, s.pk_off, send, st, s.pk_touch));
    HIP_TRY(scan_exclusive_i64(s.cub_tmp, s.cub_bytes, s.pk_cnt, s.pk_off, nchunks + 1, st));
    std::vector<int64_t> off(nranks + 1);
    for (int r = 0; r <= nranks; ++r)     // offsets at the slice boundaries (pk_cnt[nchunks] is 0)
        HIP_TRY(hipMemcpyAsync(&off[r], s.pk_off + r * cps, sizeof(int64_t), hipMemcpyDeviceToHost, st));
    HIP_TRY(hipStreamSynchronize(st));
    for (int r = 0; r < nranks; ++r) send_counts[r] = off[r + 1] - off[r];
    if (off[nranks] > 0) HIP_TRY(k_ms_pack(true, cand_global, g.n, cps, nchunks, s.pk_cnt, s.pk_off, send, st, s.pk_touch));
    return part_done(ctx);
}

// Device form of tgo_part_ms_pack: no host synchronisation — the split sizes (int64
// elements, 2 per pair) go to send_elems_dev for the caller's device all-to-all.
int tgo_part_ms_pack_dev(tgo_ctx* ctx, uint64_t* cand_global, int32_t nranks, int64_t* send, int64_t* send_elems_dev) {
    int rc = part_check(ctx);
    if (rc) return rc;
    DevGraph& g = ctx->g;
    Scratch& s = ctx->sc;
    if (!cand_global || !send || !send_elems_dev || nranks < 1 || nranks > kMaxRanks ||
        static_cast<int64_t>(nranks) * g.n != g.n_global)
        return fail(ctx, TGO_E_INVALID, "ms_pack_dev: bad arguments (nranks * n_local must equal n_global)");
    hipStream_t st = ctx->stream;
    const int64_t cps = (g.n + kPackChunk - 1) / kPackChunk;
    const int64_t nchunks = cps * nranks;
    if (!s.pk_cnt) {
        HIP_TRY(dev_alloc(ctx, s.pk_cnt, g.n_global / kPackChunk + kMaxRanks + 1));
        HIP_TRY(dev_alloc(ctx, s.pk_off, g.n_global / kPackChunk + kMaxRanks + 1));
    }
    const int self = cand_global == ctx->part_ms_cand ? ctx->part_ms_self : -1;
    HIP_TRY(hipMemsetAsync(s.pk_cnt + nchunks, 0, sizeof(int64_t), st));
    HIP_TRY(k_ms_pack(false, cand_global, g.n, cps, nchunks, s.pk_cnt, s.pk_off, send, st, s.pk_touch, self));
    HIP_TRY(scan_exclusive_i64(s.cub_tmp, s.cub_bytes, s.pk_cnt, s.pk_off, nchunks + 1, st));
    HIP_TRY(k_slice_elems(s.pk_off, cps, nranks, send_elems_dev, st));
    HIP_TRY(k_ms_pack(true, cand_global, g.n, cps, nchunks, s.pk_cnt, s.pk_off, send, st, s.pk_touch, self));
    return part_done(ctx);
}

// Fixed-capacity sparse exchange (msbfs.hip ms_pack_fixed): owner r's slot of `send` is
// 2 * (cap + 1) int64 (header + pairs), so the caller's all-to-all has equal splits.
int tgo_part_ms_pack_fixed(tgo_ctx* ctx, uint64_t* cand_global, int32_t nranks, int64_t cap, int64_t* send) {
    int rc = part_check(ctx);
    if (rc) return rc;
    DevGraph& g = ctx->g;
    Scratch& s = ctx->sc;
    if (!cand_global || !send || nranks < 1 || nranks > kMaxRanks || cap < 1 || cap > g.n ||
        static_cast<int64_t>(nranks) * g.n != g.n_global)
        return fail(ctx, TGO_E_INVALID, "ms_pack_fixed: bad arguments (1 <= cap <= n_local, nranks * n_local == n_global)");
    if (!s.pk_ovf) return fail(ctx, TGO_E_STATE, "ms_pack_fixed before ms_begin");
    hipStream_t st = ctx->stream;
    const int64_t cps = (g.n + kPackChunk - 1) / kPackChunk;
    const int64_t nchunks = cps * nranks;
    if (!s.pk_cnt) {
        HIP_TRY(dev_alloc(ctx, s.pk_cnt, g.n_global / kPackChunk + kMaxRanks + 1));
        HIP_TRY(dev_alloc(ctx, s.pk_off, g.n_global / kPackChunk + kMaxRanks + 1));
    }
    const int self = cand_global == ctx->part_ms_cand ? ctx->part_ms_self : -1;
    HIP_TRY(hipMemsetAsync(s.pk_cnt + nchunks, 0, sizeof(int64_t), st));
    HIP_TRY(k_ms_pack(false, cand_global, g.n, cps, nchunks, s.pk_cnt, s.pk_off, send, st, s.pk_touch, self));
    HIP_TRY(scan_exclusive_i64(s.cub_tmp, s.cub_bytes, s.pk_cnt, s.pk_off, nchunks + 1, st));
    HIP_TRY(k_ms_pack_fixed(cand_global, g.n, cps, nchunks, s.pk_off, nranks, cap, send, s.pk_ovf, s.pk_touch, st,
                            self));
    return part_done(ctx);
}

int tgo_part_ms_settle_fixed(tgo_ctx* ctx, int32_t level, const int64_t* recv, int32_t nslices, int64_t cap,
                             uint64_t* fr_next, int64_t* counts) {
    int rc = part_check(ctx);
    if (rc) return rc;
    DevGraph& g = ctx->g;
    Scratch& s = ctx->sc;
    hipStream_t st = ctx->stream;
    if (!recv || !fr_next || nslices < 1 || nslices > kMaxRanks || cap < 1 || cap > g.n)
        return fail(ctx, TGO_E_INVALID, "ms_settle_fixed: bad arguments");
    if (level + 1 >= (1 << kLevelPlanes)) return fail(ctx, TGO_E_UNSUPPORTED, "multi-source BFS levels are < 65536");
    if ((rc = ms_planes_for(ctx, level + 1))) return rc;
    const bool direct = ctx->part_own_direct == fr_next;     // the push wrote the owned targets here
    ctx->part_own_direct = nullptr;
    HIP_TRY(k_level_prep(s.cnt, direct ? nullptr : fr_next, direct ? 0 : g.n_active, nullptr, st));   // tail stays zero
    HIP_TRY(k_ms_or_fixed(recv, nslices, cap, fr_next, st));
    if (!direct) HIP_TRY(ms_or_own(ctx, fr_next));
    const int nxt = ctx->part_cur ^ 1;
    if (ctx->part_count_only) {
        HIP_TRY(k_ms_settle_count(push_view(g, TGO_SCOPE_BOTH_E), g.n_active, s.ms_vis, fr_next, ms_planes(ctx), s.cnt,
                                  level + 1, st, ctx->part_srcent));
    } else {
        HIP_TRY(k_ms_settle(push_view(g, TGO_SCOPE_BOTH_E), g.n_active, s.ms_vis, fr_next, ms_planes(ctx), s.q[nxt], s.qdeg,
                            s.cnt, level + 1, st, ctx->part_srcent));
    }
    ctx->part_queued = !ctx->part_count_only;
    ctx->part_srcent = nullptr;
    ctx->part_count_only = false;
    ctx->part_cur = nxt;
    return part_counts(ctx, counts);
}

int tgo_part_ms_settle_pairs(tgo_ctx* ctx, int32_t level, const int64_t* recv, const int64_t* recv_counts,
                             int32_t nslices, uint64_t* fr_next, int64_t* counts) {
    int rc = part_check(ctx);
    if (rc) return rc;
    DevGraph& g = ctx->g;
    Scratch& s = ctx->sc;
    hipStream_t st = ctx->stream;
    if (!recv || !recv_counts || !fr_next || nslices < 1 || nslices > kMaxRanks)
        return fail(ctx, TGO_E_INVALID, "ms_settle_pairs: bad arguments");
    if (level + 1 >= (1 << kLevelPlanes)) return fail(ctx, TGO_E_UNSUPPORTED, "multi-source BFS levels are < 65536");
    if ((rc = ms_planes_for(ctx, level + 1))) return rc;
    const bool direct = ctx->part_own_direct == fr_next;     // the push wrote the owned targets here
    ctx->part_own_direct = nullptr;
    HIP_TRY(k_level_prep(s.cnt, direct ? nullptr : fr_next, direct ? 0 : g.n_active, nullptr, st));   // tail stays zero
    int64_t npairs = 0;
    for (int r = 0; r < nslices; ++r) {
        if (recv_counts[r] < 0 || recv_counts[r] > g.n) return fail(ctx, TGO_E_INVALID, "ms_settle_pairs: bad count");
        npairs += recv_counts[r];
    }
    HIP_TRY(k_ms_or_pairs(recv, npairs, fr_next, st));
    if (!direct) HIP_TRY(ms_or_own(ctx, fr_next));
    const int nxt = ctx->part_cur ^ 1;
    if (ctx->part_count_only) {
        HIP_TRY(k_ms_settle_count(push_view(g, TGO_SCOPE_BOTH_E), g.n_active, s.ms_vis, fr_next, ms_planes(ctx), s.cnt,
                                  level + 1, st, ctx->part_srcent));
    } else {
        HIP_TRY(k_ms_settle(push_view(g, TGO_SCOPE_BOTH_E), g.n_active, s.ms_vis, fr_next, ms_planes(ctx), s.q[nxt], s.qdeg,
                            s.cnt, level + 1, st, ctx->part_srcent));
    }
    ctx->part_queued = !ctx->part_count_only;
    ctx->part_srcent = nullptr;
    ctx->part_count_only = false;
    ctx->part_cur = nxt;
    return part_counts(ctx, counts);
}

int tgo_part_ms_end(tgo_ctx* ctx, int64_t* reached, int64_t* entries) {
    int rc = part_check(ctx);
    if (rc) return rc;
    Scratch& s = ctx->sc;
    hipStream_t st = ctx->stream;
    HIP_TRY(hipEventRecord(ctx->ev1, st));
    if (reached || entries) {
        HIP_TRY(hipMemsetAsync(s.ms_stat, 0, 2 * TGO_MAX_SOURCES * sizeof(unsigned long long), st));
        HIP_TRY(k_ms_reach(pull_view(ctx->g, TGO_SCOPE_BOTH_E), s.ms_vis, ctx->g.n, s.ms_nsrc, s.ms_stat,
                           s.ms_stat + TGO_MAX_SOURCES, st));
        std::vector<unsigned long long> h(2 * TGO_MAX_SOURCES);
        HIP_TRY(hipMemcpyAsync(h.data(), s.ms_stat, h.size() * sizeof(unsigned long long), hipMemcpyDeviceToHost, st));
        HIP_TRY(hipStreamSynchronize(st));
        for (int r = 0; r < s.ms_nsrc; ++r) {
            if (reached) reached[r] = static_cast<int64_t>(h[r]);
            if (entries) entries[r] = static_cast<int64_t>(h[TGO_MAX_SOURCES + r]);
        }
    }
    // the fixed-capacity exchange (tgo_part_ms_pack_fixed) drops the pairs past an owner's
    // capacity: a sweep that overflowed has wrong levels and fails here
    int ovf = 0;
    if (s.pk_ovf) HIP_TRY(hipMemcpyAsync(&ovf, s.pk_ovf, sizeof(int), hipMemcpyDeviceToHost, st));
    HIP_TRY(hipStreamSynchronize(st));
    if (ovf) return fail(ctx, TGO_E_STATE, "ms_pack_fixed: an owner's pairs exceeded the capacity (cap below the level's frontier entries)");
    float ms = 0;
    HIP_TRY(hipEventElapsedTime(&ms, ctx->ev0, ctx->ev1));
    ctx->st.last_kernel_ms = ms;
    return TGO_OK;
}

int tgo_part_ms_levels(tgo_ctx* ctx, int32_t source, int64_t* dist_local) {
    int rc = part_check(ctx);
    if (rc) return rc;
    Scratch& s = ctx->sc;
    if (!s.ms_vis || source < 0 || source >= s.ms_nsrc || !dist_local) return fail(ctx, TGO_E_INVALID, "bad source");
    HIP_TRY(k_ms_extract(ms_planes(ctx), s.ms_nplanes, s.ms_vis, ctx->g.perm, source, s.msg, ctx->g.n, ctx->stream));
    HIP_TRY(hipMemcpyAsync(dist_local, s.msg, ctx->g.n * sizeof(int64_t), hipMemcpyDeviceToHost, ctx->stream));
    HIP_TRY(hipStreamSynchronize(ctx->stream));
    return TGO_OK;
}

int tgo_part_active_rows(tgo_ctx* ctx, int64_t* n_active) {
    int rc = part_check(ctx);
    if (rc) return rc;
    if (!n_active) return fail(ctx, TGO_E_INVALID, "null argument");
    *n_active = ctx->g.n_active;
    return TGO_OK;
}

// Cache-blocked partitioned PageRank.  The gathered contribution vector is laid out hot-first
// across ranks: [rank 0 rows 0..H) ... [rank W-1 rows 0..H) | [rank 0 rows H..A) ... — the
// degree-grouped layout puts each rank's hottest rows first and its entry-less rows last, so
// the first W*H sources are the job's hot set and rows >= A are never anyone's source.  The
// owned in-lists are re-expressed in that index space and cache-blocked as on one GPU.
int tgo_part_pr_blocked(tgo_ctx* ctx, int32_t world, int64_t active_span, int64_t* hot_per_rank) {
    int rc = part_check(ctx);
    if (rc) return rc;
    DevGraph& g = ctx->g;
    const int64_t nl = g.n;
    if (!hot_per_rank || world < 1 || g.n_global != static_cast<int64_t>(world) * nl)
        return fail(ctx, TGO_E_INVALID, "tgo_part_pr_blocked: world must equal n_global / n_local");
    if (active_span < g.n_active || active_span > nl)
        return fail(ctx, TGO_E_INVALID, "tgo_part_pr_blocked: active_span must cover every rank's active rows");
    *hot_per_rank = 0;
    if (g.scope == TGO_SCOPE_BOTH_E || env_i64("TGO_PR_BLOCKED", 1) == 0) {
        ctx->part_pr_world = 0;
        return TGO_OK;                                  // plain layout: one rank-major all-gather
    }
    int64_t H = env_i64("TGO_PR_HOT", pr_hot_default()) / world;
    H = std::min(active_span, std::max<int64_t>(64, H / 64 * 64));
    if (ctx->part_pr_world == world && ctx->part_pr_hot == H && ctx->part_pr_span == active_span) {
        *hot_per_rank = H;
        return TGO_OK;                                  // already built for this layout
    }
    TrimTemps trim_temps;
    const int64_t A = active_span, W = world;
    std::vector<int64_t> off(nl + 1);
    HIP_TRY(hipMemcpy(off.data(), g.in.off, (nl + 1) * sizeof(int64_t), hipMemcpyDeviceToHost));
    // the in-lists' sources as positions in the blocked gathered vector, mapped on the device;
    // the cold layout is built from that device copy (pr_layout.hip), as on one GPU
    const int64_t nnz = g.in.nnz;
    int32_t* gidx = nullptr;
    int* bad = nullptr;
    HIP_TRY(hipMalloc(&gidx, std::max<int64_t>(nnz, 1) * sizeof(int32_t)));
    struct Free { void* p; ~Free() { if (p) (void)hipFree(p); } } free_gidx{gidx};
    HIP_TRY(hipMalloc(&bad, sizeof(int)));
    Free free_bad{bad};
    HIP_TRY(hipMemsetAsync(bad, 0, sizeof(int), ctx->stream));
    HIP_TRY(k_part_gathered_index(g.in.adj, nnz, nl, A, H, W, gidx, bad, ctx->stream));
    int hbad = 0;
    HIP_TRY(hipMemcpyAsync(&hbad, bad, sizeof(int), hipMemcpyDeviceToHost, ctx->stream));
    HIP_TRY(hipStreamSynchronize(ctx->stream));
    if (hbad) return fail(ctx, TGO_E_INVALID, "tgo_part_pr_blocked: a source row lies beyond active_span");
    // the mapping is not monotone in the global id: re-sort each row so the device build applies
    if (env_i64("TGO_HOST_ASSEMBLY", 0) == 0) {
        std::string err;
        if (int r = sort_rows_device(g.in.off, nl, gidx, nnz, ctx->stream, err)) return fail(ctx, r, err);
    }
    bool ready = false;
    const std::vector<int32_t> no_host_adj;
    if ((rc = upload_cold_blocks(ctx, off, no_host_adj, W * A, W * H, g.n_active, g.cold_in, ready, g.in.off, gidx, nnz)))
        return rc;
    HIP_TRY(hipStreamSynchronize(ctx->stream));
    g.cold_in_ready = ready;
    if (!ready) { ctx->part_pr_world = 0; return TGO_OK; }
    Scratch& s = ctx->sc;
    if (g.cold_in.rb_hot.nchunks > s.partial_cap) {
        s.partial_cap = g.cold_in.rb_hot.nchunks;
        HIP_TRY(dev_alloc(ctx, s.partial, s.partial_cap));
    }
    ctx->part_pr_world = world;
    ctx->part_pr_hot = H;
    ctx->part_pr_span = A;
    ctx->st.device_bytes = ctx->dev_bytes;
    *hot_per_rank = H;
    return TGO_OK;
}

int tgo_part_pr_begin(tgo_ctx* ctx, const tgo_pr_args* a, double* contrib_local) {
    int rc = part_check(ctx);
    if (rc) return rc;
    if (!a || a->max_iterations < 1) return fail(ctx, TGO_E_INVALID, "partitioned PageRank needs max_iterations >= 1");
    DevGraph& g = ctx->g;
    Scratch& s = ctx->sc;
    const double N = static_cast<double>(a->vertex_count);
    ctx->part_alpha = a->alpha;
    ctx->part_base = (1.0 - a->alpha) / N;
    ctx->part_pr_iter = 1;
    ctx->part_pr_iters = a->max_iterations;
    if (!ctx->part_pr_plain) ctx->st.exact_reruns = 0;
    HIP_TRY(hipEventRecord(ctx->ev0, ctx->stream));
    // iteration 1 (PageRankVertexProgram.java:78-83) on the owned rows
    HIP_TRY(k_pr_init(g.out, s.vec[0], contrib_local, reinterpret_cast<double*>(s.dist), 1.0 / N, g.n, ctx->stream));
    return part_done(ctx);
}

static bool part_pr_blocked_ready(const tgo_ctx* ctx) {
    return ctx->part_pr_world > 0 && ctx->g.cold_in_ready && !ctx->part_pr_plain;
}

// The fixed-point passes' range flag of the last partitioned PageRank (read and cleared).
int tgo_part_pr_exact_check(tgo_ctx* ctx, int32_t* bad) {
    int rc = part_check(ctx);
    if (rc) return rc;
    if (!bad) return fail(ctx, TGO_E_INVALID, "null argument");
    bool b = false;
    if (part_pr_blocked_ready(ctx) && (rc = fx_take_bad(ctx, ctx->g.cold_in, &b))) return rc;
    *bad = b ? 1 : 0;
    return TGO_OK;
}

// Run the next partitioned PageRank programs on the plain layout (rank-major n_local slices,
// fp64 gather) while on = 1, keeping the blocked layout for later ones.
int tgo_part_pr_plain(tgo_ctx* ctx, int32_t on) {
    int rc = part_check(ctx);
    if (rc) return rc;
    ctx->part_pr_plain = on != 0;
    if (on) ctx->st.exact_reruns = 1;                // the stats of the program that re-runs
    return TGO_OK;
}

// the PAGE_RANK property is only read after the last superstep: write it there
static double* part_pr_out(tgo_ctx* ctx) {
    return ctx->part_pr_iter + 1 == ctx->part_pr_iters ? reinterpret_cast<double*>(ctx->sc.dist) : nullptr;
}

int tgo_part_pr_step_cold(tgo_ctx* ctx, const double* gathered) {
    int rc = part_check(ctx);
    if (rc) return rc;
    if (!part_pr_blocked_ready(ctx)) return fail(ctx, TGO_E_STATE, "tgo_part_pr_step_cold needs tgo_part_pr_blocked");
    HIP_TRY(k_pr_cold_phase(ctx->g.cold_in, gathered, ctx->stream, ctx->part_pr_iter == 1));
    return part_done(ctx);
}

int tgo_part_pr_step_hot(tgo_ctx* ctx, const double* gathered, double* contrib_local) {
    int rc = part_check(ctx);
    if (rc) return rc;
    if (!part_pr_blocked_ready(ctx)) return fail(ctx, TGO_E_STATE, "tgo_part_pr_step_hot needs tgo_part_pr_blocked");
    if (ctx->part_pr_iter >= ctx->part_pr_iters) return fail(ctx, TGO_E_STATE, "PageRank program already complete");
    Scratch& s = ctx->sc;
    HIP_TRY(k_pr_hot_phase(ctx->g.cold_in, gathered, s.vec[0], part_pr_out(ctx), contrib_local, s.partial,
                           ctx->part_alpha, ctx->part_base, ctx->stream, ctx->part_pr_iter == 1));
    ++ctx->part_pr_iter;
    return part_done(ctx);
}

int tgo_part_pr_step(tgo_ctx* ctx, const double* contrib_global, double* contrib_local) {
    int rc = part_check(ctx);
    if (rc) return rc;
    if (part_pr_blocked_ready(ctx)) {
        if ((rc = tgo_part_pr_step_cold(ctx, contrib_global))) return rc;
        return tgo_part_pr_step_hot(ctx, contrib_global, contrib_local);
    }
    if (ctx->part_pr_iter >= ctx->part_pr_iters) return fail(ctx, TGO_E_STATE, "PageRank program already complete");
    DevGraph& g = ctx->g;
    Scratch& s = ctx->sc;
    // owned rows gather over their IN lists (global source ids) from the gathered vector
    HIP_TRY(k_pr_iter(g.in, g.rb_in, contrib_global, s.vec[0], part_pr_out(ctx), contrib_local, s.partial,
                      ctx->part_alpha, ctx->part_base, g.n, PrTuning{}, ctx->stream));
    ++ctx->part_pr_iter;
    return part_done(ctx);
}

int tgo_part_pr_end(tgo_ctx* ctx, double* pr_local) {
    int rc = part_check(ctx);
    if (rc) return rc;
    if (ctx->part_pr_iter != ctx->part_pr_iters)
        return fail(ctx, TGO_E_STATE, "partitioned PageRank ended before its last iteration");
    DevGraph& g = ctx->g;
    Scratch& s = ctx->sc;
    double* pr = reinterpret_cast<double*>(s.dist);
    // blocked updates skip the entry-less rows: their rank after any update is (1-a)/N
    if (part_pr_blocked_ready(ctx) && ctx->part_pr_iters >= 2 && g.cold_in.n_rows < g.n)
        HIP_TRY(k_fill_f64(pr + g.cold_in.n_rows, ctx->part_base, g.n - g.cold_in.n_rows, ctx->stream));
    HIP_TRY(hipEventRecord(ctx->ev1, ctx->stream));
    if (pr_local) {     // back to row order
        HIP_TRY(k_unpermute_i64(s.dist, g.perm, s.msg, g.n, ctx->stream));
        HIP_TRY(hipMemcpyAsync(pr_local, s.msg, g.n * sizeof(double), hipMemcpyDeviceToHost, ctx->stream));
    }
    HIP_TRY(hipStreamSynchronize(ctx->stream));
    float ms = 0;
    HIP_TRY(hipEventElapsedTime(&ms, ctx->ev0, ctx->ev1));
    ctx->st.last_kernel_ms = ms;
    return TGO_OK;
}

// ---- partitioned delta-stepping SSSP (delta.hip; exchange protocol: titan_amd/distributed.py)
static int ds_part_alloc(tgo_ctx* ctx) {
    Scratch& s = ctx->sc;
    if (s.ds_rbest) return TGO_OK;
    HIP_TRY(dev_alloc(ctx, s.ds_rbest, ctx->g.n_global));
    HIP_TRY(dev_alloc(ctx, s.ds_rmark, ctx->g.n_global / 64 + 1));
    HIP_TRY(dev_alloc(ctx, s.ds_pack, 3 * kMaxRanks + 2));
    return TGO_OK;
}
// the loop state words after the pack counters (delta.hip ds_track_reset)
static long long* ds_track(Scratch& s) { return reinterpret_cast<long long*>(s.ds_pack + 3 * kMaxRanks); }

int tgo_part_sssp_begin(tgo_ctx* ctx, int64_t seed_global, int64_t delta, int64_t* out) {
    int rc = part_check(ctx);
    if (rc) return rc;
    DevGraph& g = ctx->g;
    if (g.has_weight && g.min_weight < 0) return fail(ctx, TGO_E_INVALID, "delta-stepping needs non-negative weights");
    if ((rc = ds_part_alloc(ctx))) return rc;
    Scratch& s = ctx->sc;
    hipStream_t st = ctx->stream;
    const int64_t n = g.n;
    const View push = push_view(g, g.scope);
    HIP_TRY(hipEventRecord(ctx->ev0, st));
    HIP_TRY(k_fill_i64(s.dist, INT64_MAX, n, st));
    HIP_TRY(hipMemsetAsync(s.vb, 0, ((n + 63) / 64 + 1) * 8, st));
    HIP_TRY(k_fill_i64(s.ds_rbest, INT64_MAX, g.n_global, st));
    HIP_TRY(hipMemsetAsync(s.ds_rmark, 0, (g.n_global / 64 + 1) * 8, st));
    HIP_TRY(hipMemsetAsync(s.ds_pack, 0, 3 * kMaxRanks * sizeof(unsigned long long), st));
    HIP_TRY(k_ds_track_reset(ds_track(s), st));
    ctx->part_cur = 0;
    ctx->part_qlen = 0;
    ctx->part_qlen_stale = false;
    ctx->part_relaxed = 0;
    ctx->part_phases = 0;
    ctx->part_seed = -1;
    ctx->part_split = false;
    ctx->part_devloop = false;
    int64_t seed = seed_global - g.lo;
    if (seed >= 0 && seed < n) {
        seed = ctx->perm[seed];
        HIP_TRY(k_ds_seed(push, s.dist, s.q[0], s.qdeg, seed, st));
        ctx->part_qlen = 1;
        ctx->part_seed = seed;
    }
    HIP_TRY(hipStreamSynchronize(st));
    if (out) {
        out[0] = ctx->part_qlen;
        out[1] = delta > 0 ? delta : default_delta(g, g.has_weight);
    }
    return TGO_OK;
}

// The smallest weight of the rank's load (0 without weights).  Delta-stepping refuses negative
// weights; the drivers agree on the global minimum BEFORE the first collective, so every rank
// fails together instead of one rank failing while its peers wait in an exchange.
int tgo_part_weight_min(tgo_ctx* ctx, int64_t* min_weight) {
    int rc = part_check(ctx);
    if (rc) return rc;
    if (!min_weight) return fail(ctx, TGO_E_INVALID, "null argument");
    *min_weight = ctx->g.has_weight ? ctx->g.min_weight : 0;
    return TGO_OK;
}

// The relax half of a phase.  send_counts (host) set: the pair counts come back to the host
// (one stream synchronisation); sizes (device) set instead: the exchange header is written on
// the device (ds_mark_sizes) and nothing waits.
static int part_sssp_relax_impl(tgo_ctx* ctx, int64_t thr, int32_t nranks, int64_t* send, int64_t* send_counts,
                                int64_t* sizes) {
    int rc = part_check(ctx);
    if (rc) return rc;
    DevGraph& g = ctx->g;
    Scratch& s = ctx->sc;
    if (!s.ds_rbest) return fail(ctx, TGO_E_STATE, "tgo_part_sssp_begin has not run");
    if (nranks < 1 || nranks > kMaxRanks || g.n * nranks != g.n_global || !send || (!send_counts && !sizes))
        return fail(ctx, TGO_E_INVALID, "nranks * n_local must equal n_global (equal partitions, <= 64 ranks)");
    hipStream_t st = ctx->stream;
    const View push = push_view(g, g.scope);
    const int cur = ctx->part_cur;
    if (ctx->part_split && ctx->part_qlen > 0) {      // commit_ws zeroes the counters and the scan's tail
        const int64_t ql = ctx->part_qlen;
        HIP_TRY(k_ds_commit_ws(s.q[cur], ql, s.dist, s.msg, s.vb, s.ds_member, s.qdeg, s.cnt, st, ds_track(s)));
        HIP_TRY(scan_exclusive_i64(s.cub_tmp, s.cub_bytes, s.qdeg, s.qpre, ql + 1, st));
        HIP_TRY(k_ds_relax_ws_part(s.ds_pws, s.ds_light, s.q[cur], s.qpre, ql, s.msg, s.dist, s.vb, s.q[cur ^ 1], s.qdeg,
                                   s.cnt, thr, g.lo, g.n, s.ds_rbest, s.ds_rmark, ds_track(s), st));
    } else {
        HIP_TRY(hipMemsetAsync(s.cnt, 0, sizeof(Counters), st));
    }
    if (!ctx->part_split && ctx->part_qlen > 0) {
        HIP_TRY(k_ds_commit(s.q[cur], ctx->part_qlen, s.dist, s.msg, s.vb, st));
        if ((rc = scan_frontier(ctx, ctx->part_qlen))) return rc;
        HIP_TRY(k_ds_relax_part(push, s.q[cur], s.qpre, ctx->part_qlen, s.msg, s.dist, s.vb, s.q[cur ^ 1], s.qdeg,
                                s.cnt, g.has_weight ? 1 : 0, thr, g.lo, g.n, s.ds_rbest, s.ds_rmark, ds_track(s), st));
    }
    unsigned long long* counts = s.ds_pack;
    unsigned long long* offs = counts + kMaxRanks;
    unsigned long long* cursor = offs + kMaxRanks;
    // device header: the counts / cursors are zero here (begin, then every ds_mark_sizes)
    if (send_counts) HIP_TRY(hipMemsetAsync(counts, 0, 3 * kMaxRanks * sizeof(unsigned long long), st));
    const int64_t words = g.n_global / 64, wpr = g.n / 64;
    if (!send_counts && nranks == 1) {      // one rank owns every target: nothing is ever marked
        HIP_TRY(k_ds_mark_sizes(counts, nranks, ctx->part_qlen, offs, cursor, ds_track(s), sizes, st));
        return part_done(ctx);
    }
    HIP_TRY(k_ds_mark_count(s.ds_rmark, words, wpr, counts, st));
    if (!send_counts) {
        HIP_TRY(k_ds_mark_sizes(counts, nranks, ctx->part_qlen, offs, cursor, ds_track(s), sizes, st));
        HIP_TRY(k_ds_mark_pack(s.ds_rmark, words, wpr, g.n, s.ds_rbest, offs, cursor, send, st));
        return part_done(ctx);
    }
    unsigned long long h[kMaxRanks], ho[kMaxRanks];
    HIP_TRY(hipMemcpyAsync(h, counts, nranks * sizeof(unsigned long long), hipMemcpyDeviceToHost, st));
    HIP_TRY(hipStreamSynchronize(st));
    unsigned long long acc = 0;
    for (int r = 0; r < nranks; ++r) {
        ho[r] = acc;
        acc += h[r];
        send_counts[r] = static_cast<int64_t>(h[r]);
    }
    HIP_TRY(hipMemcpyAsync(offs, ho, nranks * sizeof(unsigned long long), hipMemcpyHostToDevice, st));
    HIP_TRY(k_ds_mark_pack(s.ds_rmark, words, wpr, g.n, s.ds_rbest, offs, cursor, send, st));
    return part_done(ctx);          // the caller's exchange follows on the same stream
}

int tgo_part_sssp_relax(tgo_ctx* ctx, int64_t thr, int32_t nranks, int64_t* send, int64_t* send_counts) {
    if (ctx && !send_counts) return fail(ctx, TGO_E_INVALID, "null send_counts");
    return part_sssp_relax_impl(ctx, thr, nranks, send, send_counts, nullptr);
}

int tgo_part_sssp_apply(tgo_ctx* ctx, int64_t thr, const int64_t* recv, int64_t npairs, int64_t* counts) {
    int rc = part_check(ctx);
    if (rc) return rc;
    DevGraph& g = ctx->g;
    Scratch& s = ctx->sc;
    if (!s.ds_rbest) return fail(ctx, TGO_E_STATE, "tgo_part_sssp_begin has not run");
    if (npairs < 0 || (npairs > 0 && !recv)) return fail(ctx, TGO_E_INVALID, "bad received pairs");
    hipStream_t st = ctx->stream;
    if (npairs > 0)
        HIP_TRY(k_ds_apply(push_view(g, g.scope), recv, npairs, s.dist, s.vb, s.q[ctx->part_cur ^ 1], s.qdeg, s.cnt,
                           thr, ctx->part_split ? s.ds_pws.off : nullptr, ctx->part_split ? s.ds_light : nullptr,
                           ds_track(s), st));
    if ((rc = read_counters(ctx))) return rc;
    if (s.hcnt->err) return fail(ctx, TGO_E_PROGRAM,
        "vertex program failed: a traversed edge has no value for the weight property");
    if (ctx->part_qlen > 0) ctx->part_relaxed += static_cast<int64_t>(s.hcnt->red[1]);
    ctx->part_cur ^= 1;
    ctx->part_qlen = static_cast<int64_t>(s.hcnt->qlen);
    ctx->part_qlen_stale = false;
    ++ctx->part_phases;
    if (counts) {
        counts[0] = ctx->part_qlen;
        counts[1] = static_cast<int64_t>(s.hcnt->mf);
    }
    return TGO_OK;
}

int tgo_part_sssp_pending_min(tgo_ctx* ctx, int64_t* out) {
    int rc = part_check(ctx);
    if (rc) return rc;
    Scratch& s = ctx->sc;
    if (!out) return fail(ctx, TGO_E_INVALID, "null output");
    hipStream_t st = ctx->stream;
    HIP_TRY(hipMemsetAsync(s.cnt, 0, sizeof(Counters), st));
    HIP_TRY(hipMemsetAsync(&s.cnt->red[0], 0x7F, sizeof(unsigned long long), st));
    HIP_TRY(k_ds_pending_min(s.vb, (ctx->g.n + 63) / 64, s.dist, s.cnt, st));
    if ((rc = read_counters(ctx))) return rc;
    out[1] = static_cast<int64_t>(s.hcnt->red[1]);
    out[0] = out[1] ? static_cast<int64_t>(s.hcnt->red[0]) : INT64_MAX;
    return TGO_OK;
}

int tgo_part_sssp_extract(tgo_ctx* ctx, int64_t thr, int64_t* counts) {
    int rc = part_check(ctx);
    if (rc) return rc;
    DevGraph& g = ctx->g;
    Scratch& s = ctx->sc;
    hipStream_t st = ctx->stream;
    HIP_TRY(hipMemsetAsync(s.cnt, 0, sizeof(Counters), st));
    if (!s.ds_rbest) return fail(ctx, TGO_E_STATE, "tgo_part_sssp_begin has not run");
    HIP_TRY(k_ds_track_reset(ds_track(s), st));     // the extraction sets the pending minimum afresh
    if (ctx->part_split)            // the new near queue (light) and the settled members' heavy entries
        HIP_TRY(k_ds_extract_ws(s.ds_pws, s.ds_light, s.vb, s.ds_member, g.n, s.dist, thr, s.q[ctx->part_cur], s.qdeg,
                                s.cnt, st, ds_track(s)));
    else
        HIP_TRY(k_ds_extract(push_view(g, g.scope), s.vb, g.n, s.dist, thr, s.q[ctx->part_cur], s.qdeg, s.cnt, st,
                             ds_track(s)));
    return part_counts(ctx, counts, false);   // the SSSP driver reads counts on the host
}

int tgo_part_sssp_end(tgo_ctx* ctx, int64_t* dist_local, int64_t* reached) {
    int rc = part_check(ctx);
    if (rc) return rc;
    DevGraph& g = ctx->g;
    Scratch& s = ctx->sc;
    hipStream_t st = ctx->stream;
    if (ctx->part_devloop) {            // the device loop's counts and failure flag
        DsLoop h{};
        HIP_TRY(hipMemcpyAsync(&h, s.ds_loop, sizeof(DsLoop), hipMemcpyDeviceToHost, st));
        HIP_TRY(hipStreamSynchronize(st));
        ctx->part_devloop = false;
        if (h.err) return fail(ctx, TGO_E_PROGRAM,
            "vertex program failed: a traversed edge has no value for the weight property");
        ctx->part_relaxed = static_cast<int64_t>(h.relaxed);
        ctx->part_phases = static_cast<int32_t>(h.phases);
    }
    HIP_TRY(k_dist_finalize(s.dist, g.n, st));
    HIP_TRY(hipEventRecord(ctx->ev1, st));
    if (reached) {
        HIP_TRY(hipMemsetAsync(s.cnt, 0, sizeof(Counters), st));
        HIP_TRY(k_reach_stats(pull_view(g, g.scope), s.dist, g.n, s.cnt->red, st));
        if ((rc = read_counters(ctx))) return rc;
        reached[0] = static_cast<int64_t>(s.hcnt->red[0]);
        reached[1] = static_cast<int64_t>(s.hcnt->red[1]);
    }
    if (dist_local) {   // back to row order
        HIP_TRY(k_unpermute_i64(s.dist, g.perm, s.msg, g.n, st));
        HIP_TRY(hipMemcpyAsync(dist_local, s.msg, g.n * sizeof(int64_t), hipMemcpyDeviceToHost, st));
    }
    HIP_TRY(hipStreamSynchronize(st));
    float ms = 0;
    HIP_TRY(hipEventElapsedTime(&ms, ctx->ev0, ctx->ev1));
    ctx->st.last_kernel_ms = ms;
    ctx->st.relaxed_entries = ctx->part_relaxed;
    ctx->st.levels = ctx->part_phases;
    return TGO_OK;
}

// ------------------------------------------------------------------ generic vertex programs
static int generic_alloc(tgo_ctx* ctx) {
    Scratch& s = ctx->sc;
    if (s.gv[0]) return TGO_OK;
    for (int i = 0; i < 3; ++i) {
        HIP_TRY(dev_alloc(ctx, s.gv[i], ctx->g.n + 1));
        HIP_TRY(dev_alloc(ctx, s.gh[i], ctx->g.n + 1));
    }
    ctx->st.device_bytes = ctx->dev_bytes;
    return TGO_OK;
}

// Whether the gather's edge function reads e.value(weight).
static bool weight_edge_fn(const tgo_ctx* ctx, int fn) {
    return (fn >= TGO_EDGE_ADD_WEIGHT && fn <= TGO_EDGE_DIV_WEIGHT) || (fn == TGO_EDGE_PROGRAM && ctx->edge_prog.uses_w);
}

// Validate a postfix edge-function program (stack effects, constant indices, one result).
int tgo_set_edge_program(tgo_ctx* ctx, const tgo_edge_program* p) {
    if (!ctx) return TGO_E_INVALID;
    if (!p) { ctx->edge_prog = EdgeProg(); return TGO_OK; }
    if (p->n_ops < 1 || p->n_ops > TGO_EDGE_PROGRAM_MAX_OPS || !p->ops)
        return fail(ctx, TGO_E_INVALID, "edge program: 1 to " + std::to_string(TGO_EDGE_PROGRAM_MAX_OPS) + " ops");
    if (p->n_consts < 0 || p->n_consts > TGO_EDGE_PROGRAM_MAX_CONSTS || (p->n_consts > 0 && !p->iconsts && !p->fconsts))
        return fail(ctx, TGO_E_INVALID, "edge program: 0 to " + std::to_string(TGO_EDGE_PROGRAM_MAX_CONSTS) +
                                        " constants, long and / or double values");
    EdgeProg pg;
    int depth = 0;
    for (int i = 0; i < p->n_ops; ++i) {
        const int op = p->ops[i] & 0xFF, arg = p->ops[i] >> 8;
        const std::string at = "edge program op " + std::to_string(i) + ": ";
        if (op < TGO_OP_MSG || op > TGO_OP_ABS) return fail(ctx, TGO_E_INVALID, at + "unknown op");
        if (op != TGO_OP_CONST && arg != 0) return fail(ctx, TGO_E_INVALID, at + "only CONST takes an argument");
        if (op == TGO_OP_CONST && (arg < 0 || arg >= p->n_consts)) return fail(ctx, TGO_E_INVALID, at + "constant index");
        const int pops = op <= TGO_OP_CONST ? 0 : op >= TGO_OP_NEG ? 1 : 2;
        if (depth < pops) return fail(ctx, TGO_E_INVALID, at + "stack underflow");
        depth += (op <= TGO_OP_CONST ? 1 : op >= TGO_OP_NEG ? 0 : -1);
        if (depth > TGO_EDGE_PROGRAM_MAX_STACK) return fail(ctx, TGO_E_INVALID, at + "stack deeper than " +
                                                            std::to_string(TGO_EDGE_PROGRAM_MAX_STACK));
        if (op == TGO_OP_WEIGHT) pg.uses_w = 1;
        pg.ops[i] = p->ops[i];
    }
    if (depth != 1) return fail(ctx, TGO_E_INVALID, "edge program must leave exactly one value");
    pg.n = p->n_ops;
    pg.has_i = p->n_consts == 0 || p->iconsts;
    pg.has_f = p->n_consts == 0 || p->fconsts;
    for (int i = 0; i < p->n_consts; ++i) {
        if (p->iconsts) pg.ic[i] = p->iconsts[i];
        if (p->fconsts) pg.fc[i] = p->fconsts[i];
    }
    ctx->edge_prog = pg;
    return TGO_OK;
}

// Scope, value type, combiner (when used) and edge function of a Local receive.
static int check_gather_args(tgo_ctx* ctx, const tgo_gather_args* a, bool combiner) {
    if (!ctx->loaded) return fail(ctx, TGO_E_STATE, "no graph loaded");
    if (ctx->g.partitioned) return fail(ctx, TGO_E_UNSUPPORTED, "generic gathers run on a one-GPU load");
    if (a->scope < 0 || a->scope > 2) return fail(ctx, TGO_E_INVALID, "invalid scope");
    if (a->scope != ctx->g.scope && ctx->g.scope != TGO_SCOPE_BOTH_E)
        return fail(ctx, TGO_E_INVALID, "message scope differs from the scope the graph was loaded (preloaded) for");
    if (a->value_type < 0 || a->value_type > 1 || (combiner && (a->combiner < 0 || a->combiner > 2)) ||
        a->edge_fn < TGO_EDGE_IDENTITY || a->edge_fn > TGO_EDGE_PROGRAM)
        return fail(ctx, TGO_E_INVALID, "invalid value type, combiner or edge function");
    if (a->edge_fn == TGO_EDGE_PROGRAM) {
        const EdgeProg& pg = ctx->edge_prog;
        if (pg.n == 0) return fail(ctx, TGO_E_STATE, "TGO_EDGE_PROGRAM without a program (tgo_set_edge_program)");
        if (a->value_type == TGO_VAL_INT64 ? !pg.has_i : !pg.has_f)
            return fail(ctx, TGO_E_INVALID, "the edge program has no constants of the message type");
    }
    if (weight_edge_fn(ctx, a->edge_fn) && !ctx->g.has_weight)
        return fail(ctx, TGO_E_INVALID, "weight edge function on a graph loaded without a weight property");
    if (weight_edge_fn(ctx, a->edge_fn) && (ctx->g.weight_dt == TGO_DT_FLOAT || ctx->g.weight_dt == TGO_DT_DOUBLE) &&
        a->value_type == TGO_VAL_INT64)
        return fail(ctx, TGO_E_INVALID, "a Float / Double weight needs fp64 messages (long op double is a double in Java)");
    return TGO_OK;
}

static WeightCol weight_col(const DevGraph& g) {
    WeightCol wc;
    wc.kind = g.weight_dt == TGO_DT_FLOAT ? 1 : g.weight_dt == TGO_DT_LONG ? 2 : g.weight_dt == TGO_DT_DOUBLE ? 3 : 0;
    wc.wide = g.wval;
    return wc;
}

static int gather_error(tgo_ctx* ctx, unsigned long long err) {
    if (err & 2) return fail(ctx, TGO_E_PROGRAM, "vertex program failed: integer division by zero in an edge function");
    if (err) return fail(ctx, TGO_E_PROGRAM, "vertex program failed: a traversed edge has no value for the weight property");
    return TGO_OK;
}

int tgo_gather(tgo_ctx* ctx, const tgo_gather_args* a, const void* msg, const uint8_t* has, void* out,
               uint8_t* out_has) {
    if (!ctx) return TGO_E_INVALID;
    ctx->res_kind = -1;
    if (!a || !msg || !out || !out_has) return fail(ctx, TGO_E_INVALID, "null argument");
    int rc;
    if ((rc = check_gather_args(ctx, a, true))) return rc;
    (void)hipSetDevice(ctx->opts.device);
    if ((rc = generic_alloc(ctx))) return rc;
    Scratch& s = ctx->sc;
    hipStream_t st = ctx->stream;
    const int64_t n = ctx->g.n;
    HIP_TRY(hipEventRecord(ctx->ev0, st));
    HIP_TRY(hipMemcpyAsync(s.gv[0], msg, n * 8, hipMemcpyHostToDevice, st));
    if (has) HIP_TRY(hipMemcpyAsync(s.gh[0], has, n, hipMemcpyHostToDevice, st));
    else HIP_TRY(hipMemsetAsync(s.gh[0], 1, n, st));
    HIP_TRY(hipMemsetAsync(s.cnt, 0, sizeof(Counters), st));
    HIP_TRY(k_to_internal(s.gv[0], s.gh[0], ctx->g.perm, s.gv[1], s.gh[1], n, st));
    HIP_TRY(k_local_gather(pull_view(ctx->g, a->scope), n, a->value_type, s.gv[1], s.gh[1], a->combiner, a->edge_fn,
                           weight_col(ctx->g), ctx->edge_prog, s.gv[2], s.gh[2], &s.cnt->err, st));
    HIP_TRY(k_to_rows(s.gv[2], s.gh[2], ctx->g.perm, s.gv[0], s.gh[0], n, st));
    HIP_TRY(hipEventRecord(ctx->ev1, st));
    HIP_TRY(hipMemcpyAsync(out, s.gv[0], n * 8, hipMemcpyDeviceToHost, st));
    HIP_TRY(hipMemcpyAsync(out_has, s.gh[0], n, hipMemcpyDeviceToHost, st));
    if ((rc = read_counters(ctx))) return rc;
    float ms = 0;
    HIP_TRY(hipEventElapsedTime(&ms, ctx->ev0, ctx->ev1));
    ctx->st.last_kernel_ms = ms;
    return gather_error(ctx, s.hcnt->err);
}

int tgo_gather_lists(tgo_ctx* ctx, const tgo_gather_args* a, const void* msg, const uint8_t* has, int64_t* row_offsets,
                     void* values) {
    if (!ctx) return TGO_E_INVALID;
    ctx->res_kind = -1;
    if (!a || !msg || !row_offsets) return fail(ctx, TGO_E_INVALID, "null argument");
    int rc;
    if ((rc = check_gather_args(ctx, a, false))) return rc;
    (void)hipSetDevice(ctx->opts.device);
    if ((rc = generic_alloc(ctx))) return rc;
    Scratch& s = ctx->sc;
    hipStream_t st = ctx->stream;
    const DevGraph& g = ctx->g;
    const int64_t n = g.n;
    const View pull = pull_view(g, a->scope);
    const WeightCol wc = weight_col(g);
    HIP_TRY(hipMemcpyAsync(s.gv[0], msg, n * 8, hipMemcpyHostToDevice, st));
    if (has) HIP_TRY(hipMemcpyAsync(s.gh[0], has, n, hipMemcpyHostToDevice, st));
    else HIP_TRY(hipMemsetAsync(s.gh[0], 1, n, st));
    HIP_TRY(hipMemsetAsync(s.cnt, 0, sizeof(Counters), st));
    HIP_TRY(k_to_internal(s.gv[0], s.gh[0], g.perm, s.gv[1], s.gh[1], n, st));
    // offsets: counts per row (s.gv[2] as int64 n+1), scanned into s.gv[0]
    int64_t* cnt = reinterpret_cast<int64_t*>(s.gv[2]);
    int64_t* off = reinterpret_cast<int64_t*>(s.gv[0]);
    HIP_TRY(k_list_count(pull, g.perm, n, s.gh[1], weight_edge_fn(ctx, a->edge_fn), cnt, &s.cnt->err, st));
    HIP_TRY(scan_exclusive_i64(s.cub_tmp, s.cub_bytes, cnt, off, n + 1, st));
    HIP_TRY(hipMemcpyAsync(row_offsets, off, (n + 1) * sizeof(int64_t), hipMemcpyDeviceToHost, st));
    if ((rc = read_counters(ctx))) return rc;
    if ((rc = gather_error(ctx, s.hcnt->err))) return rc;
    // a vertex cut that receives two messages meets FulgoraUtil's ThrowingCombiner (:80-91)
    for (int64_t r : ctx->pv_rows)
        if (row_offsets[r + 1] - row_offsets[r] >= 2)
            return fail(ctx, TGO_E_PROGRAM, "The VertexProgram needs to define a message combiner in order to preserve "
                                            "memory and handle partitioned vertices");
    const int64_t total = row_offsets[n];
    if (!values || total == 0) return TGO_OK;
    if (total >= (int64_t(1) << 31)) return fail(ctx, TGO_E_UNSUPPORTED, "more than 2^31 messages in one receive");
    // keys in/out (4 B each) + values in/out (8 B each) + the internal -> row map
    char* buf = nullptr;
    const size_t bytes = static_cast<size_t>(total) * 24 + static_cast<size_t>(n) * 4 + 64;
    HIP_TRY(hipMalloc(reinterpret_cast<void**>(&buf), bytes));
    uint64_t* val_in = reinterpret_cast<uint64_t*>(buf);
    uint64_t* val_out = val_in + total;
    uint32_t* key_in = reinterpret_cast<uint32_t*>(val_out + total);
    uint32_t* key_out = key_in + total;
    int32_t* inv = reinterpret_cast<int32_t*>(key_out + total);
    // column positions of the pull lists (pull_view: inE walks OUT entries, outE IN, bothE both)
    const uint32_t* col0 = !g.has_col ? nullptr : a->scope == TGO_SCOPE_OUT_E ? g.in.col : g.out.col;
    const uint32_t* col1 = !g.has_col || a->scope != TGO_SCOPE_BOTH_E ? nullptr : g.in.col;
    hipError_t e = k_list_fill_sort(pull, col0, col1, g.perm, inv, n,
                                    a->value_type, s.gv[1], s.gh[1], a->edge_fn, wc, ctx->edge_prog, off, total,
                                    key_in, key_out,
                                    val_in, val_out, s.sort_tmp, s.sort_bytes, &s.cnt->err, st);
    if (e == hipSuccess) e = hipMemcpyAsync(values, val_out, total * 8, hipMemcpyDeviceToHost, st);
    if (e == hipSuccess) e = hipStreamSynchronize(st);
    (void)hipFree(buf);
    HIP_TRY(e);
    if ((rc = read_counters(ctx))) return rc;
    return gather_error(ctx, s.hcnt->err);
}

int tgo_combine_global(tgo_ctx* ctx, int32_t value_type, int32_t combiner, int64_t nmsgs, const int64_t* targets,
                       const void* values, void* out, uint8_t* out_has) {
    if (!ctx) return TGO_E_INVALID;
    ctx->res_kind = -1;
    if (nmsgs < 0 || (nmsgs > 0 && (!targets || !values)) || !out || !out_has) return fail(ctx, TGO_E_INVALID, "null argument");
    if (!ctx->loaded) return fail(ctx, TGO_E_STATE, "no graph loaded");
    if (value_type < 0 || value_type > 1 || combiner < 0 || combiner > 2)
        return fail(ctx, TGO_E_INVALID, "invalid value type or combiner");
    if (nmsgs >= (int64_t(1) << 31)) return fail(ctx, TGO_E_UNSUPPORTED, "more than 2^31 global messages in one superstep");
    const int64_t n = ctx->g.n;
    for (int64_t i = 0; i < nmsgs; ++i)
        if (targets[i] < 0 || targets[i] >= n) return fail(ctx, TGO_E_INVALID, "global message target out of range");
    (void)hipSetDevice(ctx->opts.device);
    int rc = generic_alloc(ctx);
    if (rc) return rc;
    Scratch& s = ctx->sc;
    hipStream_t st = ctx->stream;
    HIP_TRY(hipMemsetAsync(s.gv[0], 0, n * 8, st));
    HIP_TRY(hipMemsetAsync(s.gh[0], 0, n, st));
    if (nmsgs > 0) {
        int64_t* buf = nullptr;          // targets, values, sort scratch (3 m): freed below
        HIP_TRY(hipMalloc(&buf, static_cast<size_t>(nmsgs) * 5 * sizeof(int64_t)));
        hipError_t e = hipMemcpyAsync(buf, targets, nmsgs * 8, hipMemcpyHostToDevice, st);
        if (e == hipSuccess) e = hipMemcpyAsync(buf + nmsgs, values, nmsgs * 8, hipMemcpyHostToDevice, st);
        if (e == hipSuccess)
            e = k_global_combine(s.sort_tmp, s.sort_bytes, buf, nmsgs, n, value_type, buf + nmsgs, combiner, buf + 2 * nmsgs,
                                 s.gv[0], s.gh[0], st);
        if (e == hipSuccess) e = hipStreamSynchronize(st);
        (void)hipFree(buf);
        HIP_TRY(e);
    }
    HIP_TRY(hipMemcpyAsync(out, s.gv[0], n * 8, hipMemcpyDeviceToHost, st));
    HIP_TRY(hipMemcpyAsync(out_has, s.gh[0], n, hipMemcpyDeviceToHost, st));
    HIP_TRY(hipStreamSynchronize(st));
    return TGO_OK;
}

int tgo_dense_ids(tgo_ctx* ctx, const int64_t* titan_ids, int64_t count, int64_t* dense_out) {
    if (!ctx) return TGO_E_INVALID;
    if (count < 0 || (count > 0 && (!titan_ids || !dense_out))) return fail(ctx, TGO_E_INVALID, "null argument");
    if (!ctx->loaded) return fail(ctx, TGO_E_STATE, "no graph loaded");
    const int pb = ctx->opts.partition_bits;
    for (int64_t i = 0; i < count; ++i) {
        int64_t id = titan_ids[i];
        if (is_partitioned_vertex(id, pb)) id = canonical_vertex_id(id, pb);    // getCanonicalId
        dense_out[i] = dense_of(ctx, id);
    }
    return TGO_OK;
}

int tgo_stats_get(tgo_ctx* ctx, tgo_stats* out) {
    if (!ctx || !out) return TGO_E_INVALID;
    *out = ctx->st;
    return TGO_OK;
}

int tgo_sync(tgo_ctx* ctx) {
    if (!ctx) return TGO_E_INVALID;
    HIP_TRY(hipStreamSynchronize(ctx->stream));
    return TGO_OK;
}

}  // extern "C"

// accessors for the C++ partitioned driver (part_driver.cpp)
namespace tgo {
hipStream_t part_stream(tgo_ctx* ctx) { return ctx->stream; }
// A partition's host graph onto the device (tgo_load_partition_layout, tgo_load_partition_rows).
int part_upload(tgo_ctx* ctx, HostGraph& h, int64_t n_global, int64_t lo) {
    free_graph(ctx);
    ctx->staging = RowStaging();
    int rc = upload_graph(ctx, h, false);     // partitioned PageRank gathers global ids: plain CSR
    if (rc) return rc;
    ctx->g.partitioned = true;
    ctx->part_pr_world = 0;
    ctx->part_pr_plain = false;
    ctx->part_pr_hot = ctx->part_pr_span = 0;
    ctx->part_pr_iter = ctx->part_pr_iters = 0;
    ctx->g.lo = lo;
    ctx->g.n_global = n_global;
    return TGO_OK;
}
// tgo_finish_partition_rows: the rows this rank staged with tgo_load_rows, decoded with the
// one-GPU rules (device decoder, or the host one under TGO_HOST_DECODE: key filter, ghosts,
// typed scopes, the cut in column order per row) into host vectors.  Vertex cuts fold on one GPU
// only; the partitioned programs read Integer weights.
int part_rows_take(tgo_ctx* ctx, RowStaging& st, std::string& err) {
    (void)hipSetDevice(ctx->opts.device);
    ctx->res_kind = -1;
    if (!ctx->staging.active) {          // no rows staged here: an empty range (the caller's scope agreed later)
        st = RowStaging();
        st.row_begin.push_back(0);
        return TGO_OK;
    }
    int rc = decode_staged_raw(ctx->staging, ctx->opts.partition_bits, ctx->opts.hard_query_limit, ctx->dec, ctx->stream,
                               err, false);
    ctx->dec.release();
    if (!rc) rc = staging_entries_to_host(ctx->staging, ctx->stream, err);
    st = std::move(ctx->staging);
    ctx->staging = RowStaging();
    if (rc) return rc;
    if (st.n_rep > 0 || std::any_of(st.vid.begin(), st.vid.end(), [](int64_t v) { return (v & 7) == 2; })) {
        err = "vertex cuts fold into their canonical vertex on a one-GPU load (VertexProgramScanJob.java:76-92)";
        return TGO_E_UNSUPPORTED;
    }
    if (st.opts.weight_key != 0 && st.plan.weight_dt != 0 && st.plan.weight_dt != TGO_DT_INTEGER) {
        err = "the partitioned programs read edge.<Integer>value(weight) (ShortestDistanceVertexProgram.java:53)";
        return TGO_E_UNSUPPORTED;
    }
    return TGO_OK;
}
void part_drop_staging(tgo_ctx* ctx) { ctx->staging = RowStaging(); ctx->dec.release(); }
int part_threads(const tgo_ctx* ctx) { return threads_of(ctx); }
void part_set_live(tgo_ctx* ctx, int64_t live) { ctx->st.num_vertices = live; }
int part_fail(tgo_ctx* ctx, int code, const std::string& msg) { return fail(ctx, code, msg); }
int64_t* part_dcounts_of(tgo_ctx* ctx) { return ctx->part_dcounts; }
// tgo_part_sssp_relax with the exchange header (sizes, 2 * nranks words) written on the device
int part_sssp_relax_dev(tgo_ctx* ctx, int64_t thr, int32_t nranks, int64_t* send, int64_t* sizes) {
    if (!sizes) return fail(ctx, TGO_E_INVALID, "null sizes");
    return part_sssp_relax_impl(ctx, thr, nranks, send, nullptr, sizes);
}
// The header fold after the driver's header all-to-all (delta.hip ds_header_fold).
int part_sssp_header_fold(tgo_ctx* ctx, const int64_t* own, const int64_t* recv, int nranks, int64_t* out) {
    HIP_TRY(k_ds_header_fold(own, recv, nranks, out, ctx->stream));
    return TGO_OK;
}
// ... and its 2 * nranks + 3 words to the host in the same launch (through the mapped counter
// page: part_read_words without its own publish kernel).
int part_sssp_header_read(tgo_ctx* ctx, const int64_t* own, const int64_t* recv, int nranks, int64_t* out,
                          int64_t* words) {
    Scratch& s = ctx->sc;
    const int count = 2 * nranks + 3;
    if (!s.hcnt || count > kCounterWords) return fail(ctx, TGO_E_STATE, "part_sssp_header_read");
    const unsigned long long seq = ++s.pub_seq;
    HIP_TRY(k_ds_header_fold(own, recv, nranks, out, ctx->stream, s.hcnt_dev, seq));
    if (int rc = wait_publish(ctx, seq)) return rc;
    const volatile unsigned long long* w = reinterpret_cast<volatile unsigned long long*>(s.hcnt);
    for (int i = 0; i < count; ++i) words[i] = static_cast<int64_t>(w[i]);
    return TGO_OK;
}
// Switch the run tgo_part_sssp_begin started onto the light/heavy split at bucket width delta
// (weighted loads; TGO_DS_SPLIT=0 keeps the plain form): the push view is split on the device
// (once per width), and the seed re-queued with its light degree.  Returns whether it did.
int part_sssp_split(tgo_ctx* ctx, int64_t delta, bool* on) {
    int rc = part_check(ctx);
    if (rc) return rc;
    DevGraph& g = ctx->g;
    Scratch& s = ctx->sc;
    *on = false;
    static const bool enabled = env_i64("TGO_DS_SPLIT", 1) != 0;
    if (!enabled || !g.has_weight || delta <= 0 || !s.ds_rbest) return TGO_OK;
    hipStream_t st = ctx->stream;
    const View push = push_view(g, g.scope);
    const int64_t n = g.n, words = (n + 63) / 64 + 1;
    if (!s.ds_light) {
        HIP_TRY(dev_alloc(ctx, s.ds_light, n + 1));
        HIP_TRY(dev_alloc(ctx, s.ds_member, words));
    }
    if (!s.ds_pws.off) {
        const int64_t nnz = (g.has_transpose ? g.push_t.nnz
                             : g.scope == TGO_SCOPE_IN_E ? g.in.nnz
                             : g.scope == TGO_SCOPE_OUT_E ? g.out.nnz : g.in.nnz + g.out.nnz);
        HIP_TRY(dev_alloc(ctx, s.ds_pws.off, n + 1));
        HIP_TRY(dev_alloc(ctx, s.ds_pws.adj, std::max<int64_t>(nnz, 1)));
        HIP_TRY(dev_alloc(ctx, s.ds_pws.w, std::max<int64_t>(nnz, 1)));
        s.ds_pws.nnz = nnz;
        s.ds_light_delta = -1;
        ctx->st.device_bytes = ctx->dev_bytes;
    }
    if (s.ds_light_delta != delta) {
        HIP_TRY(k_ds_split_rows(push, n, delta, s.ds_pws, s.ds_light, st));
        s.ds_light_delta = delta;
    }
    HIP_TRY(hipMemsetAsync(s.ds_member, 0, words * 8, st));
    if (ctx->part_seed >= 0) HIP_TRY(k_ds_seed_ws(s.ds_pws, s.ds_light, s.dist, s.q[0], s.qdeg, ctx->part_seed, st));
    ctx->part_split = true;
    *on = true;
    // the device-sized loop (TGO_DS_PART_DEVLOOP=0: the host-sized phases above) when the
    // packed queue counters hold a queue (2n + 2 takes, nnz entries), as on one GPU
    static const bool devloop = env_i64("TGO_DS_PART_DEVLOOP", 1) != 0;
    constexpr int64_t kDsMaxCount = int64_t(1) << (64 - kDsCountShift);
    if (devloop && 2 * n + 2 < kDsMaxCount && s.ds_pws.nnz < (int64_t(1) << kDsCountShift)) {
        if (!s.ds_loop) {
            for (int b = 0; b < 2; ++b) {
                HIP_TRY(dev_alloc(ctx, s.ds_q[b], 2 * n + 2));
                HIP_TRY(dev_alloc(ctx, s.ds_qp[b], 2 * n + 2));
            }
            HIP_TRY(dev_alloc(ctx, s.ds_loop, 1));
            ctx->st.device_bytes = ctx->dev_bytes;
        }
        HIP_TRY(k_ds_loop_seed(s.ds_pws, s.ds_light, s.dist, s.ds_q[0], s.ds_qp[0], s.ds_loop, ctx->part_seed, delta, st));
        ctx->part_devloop = true;
        ctx->part_cur = 0;
    }
    return part_done(ctx);
}
bool part_sssp_devloop(const tgo_ctx* ctx) { return ctx->part_devloop; }
// One phase of the device-sized loop, relax half: commit + relax of the current queue (remote
// targets marked), then the exchange header (sizes, 4 words per rank) and the pack.
// fold (one rank only, may be null): the header's fold (part_sssp_header_read's 5 words) read
// here — one rank's header all-to-all is the identity, so the header kernel publishes it.
int part_sssp_dev_relax(tgo_ctx* ctx, int32_t nranks, int64_t* send, int64_t* sizes, int64_t* fold) {
    DevGraph& g = ctx->g;
    Scratch& s = ctx->sc;
    hipStream_t st = ctx->stream;
    if (!ctx->part_devloop || nranks < 1 || nranks > kMaxRanks || g.n * nranks != g.n_global)
        return fail(ctx, TGO_E_STATE, "part_sssp_dev_relax");
    HIP_TRY(k_ds_part_relax(s.ds_pws, s.ds_light, s.vb, s.ds_member, s.dist, s.msg, s.ds_q, s.ds_qp, s.ds_loop,
                            ctx->part_cur, s.ds_light_delta, g.lo, g.n, s.ds_rbest, s.ds_rmark, st));
    unsigned long long* counts = s.ds_pack;
    unsigned long long* offs = counts + kMaxRanks;
    unsigned long long* cursor = offs + kMaxRanks;
    const int64_t words = g.n_global / 64, wpr = g.n / 64;
    if (nranks > 1) HIP_TRY(k_ds_mark_count(s.ds_rmark, words, wpr, counts, st));   // one rank marks nothing
    if (fold) {
        if (nranks != 1 || !s.hcnt) return fail(ctx, TGO_E_STATE, "part_sssp_dev_relax: fold");
        const unsigned long long seq = ++s.pub_seq;
        HIP_TRY(k_ds_part_header(counts, nranks, s.ds_loop, ctx->part_cur, offs, cursor, sizes, st, s.hcnt_dev, seq));
        if (int rc = wait_publish(ctx, seq)) return rc;
        const volatile unsigned long long* w = reinterpret_cast<volatile unsigned long long*>(s.hcnt);
        for (int i = 0; i < 5; ++i) fold[i] = static_cast<int64_t>(w[i]);
        return TGO_OK;
    }
    HIP_TRY(k_ds_part_header(counts, nranks, s.ds_loop, ctx->part_cur, offs, cursor, sizes, st));
    if (nranks > 1) HIP_TRY(k_ds_mark_pack(s.ds_rmark, words, wpr, g.n, s.ds_rbest, offs, cursor, send, st));
    return TGO_OK;
}
// ... apply half: the received pairs into the next queue, which becomes current
int part_sssp_dev_apply(tgo_ctx* ctx, const int64_t* recv, int64_t npairs) {
    Scratch& s = ctx->sc;
    if (!ctx->part_devloop) return fail(ctx, TGO_E_STATE, "part_sssp_dev_apply");
    HIP_TRY(k_ds_part_apply(recv, npairs, s.ds_pws, s.ds_light, s.dist, s.vb, s.ds_q, s.ds_qp, s.ds_loop, ctx->part_cur,
                            ctx->stream));
    ctx->part_cur ^= 1;
    return TGO_OK;
}
// ... after an empty global phase: the next near queue (and the members' heavy entries) below thr
int part_sssp_dev_extract(tgo_ctx* ctx, int64_t thr) {
    Scratch& s = ctx->sc;
    if (!ctx->part_devloop) return fail(ctx, TGO_E_STATE, "part_sssp_dev_extract");
    HIP_TRY(k_ds_part_extract(s.ds_pws, s.ds_light, s.vb, s.ds_member, ctx->g.n, s.dist, s.ds_q, s.ds_qp, s.ds_loop,
                              ctx->part_cur, thr, ctx->stream));
    return TGO_OK;
}
// `count` device words (on the ctx stream, after the work queued so far) to out, through the
// host-mapped counter page: one tiny kernel and a spin instead of a copy and a stream wait.
int part_read_words(tgo_ctx* ctx, const int64_t* dev, int count, int64_t* out) {
    Scratch& s = ctx->sc;
    if (!s.hcnt || count < 0 || count > kCounterWords) return fail(ctx, TGO_E_STATE, "part_read_words");
    const unsigned long long seq = ++s.pub_seq;
    HIP_TRY(k_publish_words(dev, count, s.hcnt_dev, seq, ctx->stream));
    if (int rc = wait_publish(ctx, seq)) return rc;
    const volatile unsigned long long* w = reinterpret_cast<volatile unsigned long long*>(s.hcnt);
    for (int i = 0; i < count; ++i) out[i] = static_cast<int64_t>(w[i]);
    return TGO_OK;
}
// The next multi-source settle also sums the new frontier's push entries per source into
// out (64 words, zeroed here on the ctx stream): the native driver's split after that level
// reads them instead of a tgo_part_ms_source_entries pass.  One-shot; nullptr cancels.
// count_only: that settle builds no frontier queue (the next level will likely pull;
// tgo_part_ms_push builds the queue if it runs after all).
int part_ms_settle_sums(tgo_ctx* ctx, int64_t* out, bool count_only) {
    ctx->part_srcent = nullptr;                                  // out == nullptr: cancel
    ctx->part_count_only = count_only;
    if (!out) return TGO_OK;
    HIP_TRY(hipMemsetAsync(out, 0, 64 * sizeof(int64_t), ctx->stream));
    ctx->part_srcent = reinterpret_cast<unsigned long long*>(out);
    return TGO_OK;
}
// The next tgo_part_ms_push writes its owned targets' candidates straight into next (with the
// bypass on); nullptr cancels.
void part_ms_own_next(tgo_ctx* ctx, uint64_t* next) {
    ctx->part_own_next = next;
    if (!next) ctx->part_own_direct = nullptr;
}
void part_ms_bypass(tgo_ctx* ctx, uint64_t* cand_global, int self) {
    ctx->part_ms_cand = cand_global;
    ctx->part_ms_self = cand_global ? self : -1;
}
std::shared_ptr<void>& part_state_of(tgo_ctx* ctx) { return ctx->part_state; }
int part_in_list(tgo_ctx* ctx, const int32_t** adj, int64_t* nnz) {
    if (int rc = part_check(ctx)) return rc;
    *adj = ctx->g.in.adj;
    *nnz = ctx->g.in.nnz;
    return TGO_OK;
}
int part_out_list(tgo_ctx* ctx, const int32_t** adj, int64_t* nnz) {
    if (int rc = part_check(ctx)) return rc;
    *adj = ctx->g.out.adj;
    *nnz = ctx->g.out.nnz;
    return TGO_OK;
}
// ghost exchange of the dense multi-source levels (tgo_set_tuning TGO_TUNE_MS_GHOST; default on)
bool ms_ghost_of(const tgo_ctx* ctx) { return ctx->ms_ghost != 0; }
// the blocked gathered layout of the last tgo_part_pr_blocked (world 0: plain layout)
int part_pr_layout_of(tgo_ctx* ctx, int32_t* world, int64_t* hot, int64_t* span) {
    if (int rc = part_check(ctx)) return rc;
    const bool blocked = part_pr_blocked_ready(ctx);
    *world = blocked ? ctx->part_pr_world : 0;
    *hot = blocked ? ctx->part_pr_hot : 0;
    *span = blocked ? ctx->part_pr_span : ctx->g.n;
    return TGO_OK;
}
int part_dims(tgo_ctx* ctx, int64_t* n_local, int64_t* lo, int64_t* n_global, int64_t* entries) {
    if (int rc = part_check(ctx)) return rc;
    *n_local = ctx->g.n;
    *lo = ctx->g.lo;
    *n_global = ctx->g.n_global;
    *entries = ctx->g.out.nnz + ctx->g.in.nnz;
    return TGO_OK;
}
int part_scratch(tgo_ctx* ctx, void** p, int64_t bytes, int slot) {
    Scratch& s = ctx->sc;
    if (slot < 0 || slot >= Scratch::kDrvSlots) return fail(ctx, TGO_E_INVALID, "driver scratch slot");
    if (s.drv_bytes[slot] < bytes) {                // fresh buffers start zero
        uint8_t* q = nullptr;
        HIP_TRY(dev_alloc(ctx, q, bytes));
        HIP_TRY(hipMemsetAsync(q, 0, static_cast<size_t>(bytes), ctx->stream));
        s.drv[slot] = q;
        s.drv_bytes[slot] = bytes;
    }
    *p = s.drv[slot];
    return TGO_OK;
}
// Push budget of the multi-source pull levels' sparse sources (the source split), as a
// fraction of the list entries: the ctx's tgo_set_tuning value, else TGO_MS_SPLIT, else 0.5 %.
double ms_split_of(const tgo_ctx* ctx) {
    static const double env = env_double("TGO_MS_SPLIT", 0.005);
    return ctx->ms_split >= 0.0 ? ctx->ms_split : env;
}

}  // namespace tgo

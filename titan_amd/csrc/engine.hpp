// engine.hpp — internal interfaces of the MI355X OLAP engine (not part of the C-ABI).
//
// Data layout in HBM (see DESIGN.md "Data layout"):
//   out-CSR : off_o[n+1] (int64), adj_o[E_o] (int32 dense ids), w_o[E_o] (int32, optional)
//             row v = the OUT entries of Titan row v, in column order
//   in-CSR  : off_i[n+1], adj_i[E_i], w_i[E_i]  — the IN entries of row v
// A message scope's reversed incident traversal (FulgoraUtil.java:57) is a "view":
//   scope inE  -> receiver pulls over out-CSR, sender pushes over in-CSR
//   scope outE -> receiver pulls over in-CSR,  sender pushes over out-CSR
//   scope bothE-> both lists (pull == push)
// When the per-row preload cap truncated a row (QueryContainer.java:28,122) the pull lists
// are no longer transposes of each other, and the push list is an explicit transpose
// of the pull list (t-CSR).
#pragma once
#include <algorithm>
#include <cstdint>
#include <string>
#include <vector>
#include <hip/hip_runtime_api.h>
#include "../../include/titan_gpu_olap.h"

namespace tgo {

// ---------------------------------------------------------------- host graph
// A device array built on the device (assemble.hip, pr_layout.hip) and handed to the upload,
// which adopts it instead of a host round trip.  Move-only; frees itself if never adopted.
template <class T>
struct DevArray {
    T* p = nullptr;
    int64_t n = -1;             // element count; < 0: no device array
    DevArray() = default;
    DevArray(const DevArray&) = delete;
    DevArray& operator=(const DevArray&) = delete;
    DevArray(DevArray&& o) noexcept : p(o.p), n(o.n) { o.p = nullptr; o.n = -1; }
    DevArray& operator=(DevArray&& o) noexcept {
        if (this != &o) { reset(); p = o.p; n = o.n; o.p = nullptr; o.n = -1; }
        return *this;
    }
    ~DevArray() { reset(); }
    void reset() { if (p) (void)hipFree(p); p = nullptr; n = -1; }
    void own(T* q, int64_t count) { reset(); p = q; n = count; }
    bool present() const { return n >= 0; }
};

struct HostCsr {
    std::vector<int64_t> off;   // n+1
    std::vector<int32_t> adj;
    std::vector<int32_t> w;     // empty when unweighted
    std::vector<uint32_t> col;  // TGO_LOAD_COLUMN_ORDER: each entry's position in its Titan row
                                // (column order across both directions); empty otherwise
    // device-resident lists of a device assembly; the host vectors above are then filled only
    // where a host consumer needs them (weights: weight_sorted_push)
    DevArray<int32_t> dadj, dw;
    DevArray<uint32_t> dcol;
    int64_t nnz() const { return dadj.present() ? dadj.n : static_cast<int64_t>(adj.size()); }
    bool has_col() const { return dcol.present() || !col.empty(); }
};

struct HostGraph {
    int64_t n = 0;
    // Long / Double weight keys: the value table the lists' weight column indexes (host or device)
    std::vector<int64_t> wval;
    DevArray<int64_t> d_wval;
    std::vector<int64_t> titan_id;   // row order (the API's dense ids)
    bool ids_sorted = false;         // titan_id known strictly increasing (no check needed)
    std::vector<int32_t> perm;       // row-order dense id -> internal id (degree-grouped)
    HostCsr out, in;
    HostCsr push_t;             // explicit transpose of the pull view (cap / asymmetric rows)
    bool has_transpose = false;
    bool has_weight = false;
    int32_t weight_dt = TGO_DT_INTEGER;   // datatype of the weight property (int32 bits; Float: IEEE bits)
    int32_t scope = TGO_SCOPE_BOTH_E;
    int64_t ghost = 0, truncated = 0, skipped = 0;
    int64_t partitioned = 0, partition_rows = 0, ghost_partition_rows = 0;
    // largest OUT / IN list of a vertex cut (PageRank has no combiner: >= 2 messages at a
    // cut make the reference throw, FulgoraUtil.java:80-91)
    int64_t pv_max_out = 0, pv_max_in = 0;
    std::vector<uint8_t> pv_flags;   // row-order dense id -> is a vertex cut (empty if none)
};

// Owner of a codec PlanView (codec.hpp) built from tgo_schema + tgo_load_opts.
// Long / Double weight keys: the weight column holds staged positions into a 64-bit value table
inline bool wide_weight_dt(int dt) { return dt == TGO_DT_LONG || dt == TGO_DT_DOUBLE; }

struct HostPlan {
    std::vector<uint8_t> label_bytes;   // LabelPlan records (opaque here; codec.hpp defines them)
    std::vector<int64_t> key_ids;
    std::vector<int8_t> key_dts;
    std::vector<int8_t> dts;
    int32_t n_labels = 0;
    int64_t weight_key = 0;
    int32_t weight_dt = 0;               // datatype of weight_key (0: no weight)
};
// Staging of decoded rows between tgo_load_rows batches (decoded on arrival).
struct RowStaging {
    std::vector<int64_t> vid;        // live vertices in row order
    std::vector<int64_t> row_begin;  // per live row, index into entries (size = vid+1)
    std::vector<int64_t> other;      // other vertex Titan id per kept entry
    std::vector<uint8_t> dir;        // 0 OUT, 1 IN
    std::vector<int32_t> w;          // weight (INT32_MIN = property missing)
    // the device decoder's kept entries stay on the device for the device assembly (the
    // host vectors other / dir / w are then empty; staging_entries_to_host fetches them)
    DevArray<int64_t> d_other;
    DevArray<uint8_t> d_dir;
    DevArray<int32_t> d_w;
    std::vector<int64_t> wv;         // wide weight keys: entry k's 64-bit value (w[k] = k)
    DevArray<int64_t> d_wv;
    int64_t entries() const { return d_other.present() ? d_other.n : static_cast<int64_t>(other.size()); }
    std::vector<uint8_t> rep;        // per row: 1 = non-canonical representative of a vertex cut
    int64_t ghost = 0, truncated = 0, skipped = 0;
    int64_t n_rep = 0;               // representative rows staged
    bool active = false;
    tgo_load_opts opts{};
    std::vector<int64_t> labels;
    // device decode: the scan's work blocks are concatenated here (offsets rebased) and
    // decoded in one device pass at tgo_finish_load
    // (entry bytes and limit/valuePos words go straight to the device: DecodeScratch)
    std::vector<int64_t> raw_keys, raw_eb{0}, raw_bb{0};
    std::vector<uint8_t> plan_bytes;  // HostPlan of the first raw batch, serialised for comparison
    HostPlan plan;
};

// Result write-back (results.hip): device arrays of the last finished program.
struct ResultSource { const void* v0 = nullptr; const void* v1 = nullptr; };
struct ResultRows {
    int64_t nrows = 0, nentries = 0, nbytes = 0;
    bool write = false;
    int64_t* row_src = nullptr;              // API row index of every output row
    int64_t* row_entry_begin = nullptr;
    int64_t* row_byte_begin = nullptr;
    uint8_t* entry_bytes = nullptr;
    int64_t* entry_limit_valpos = nullptr;
};
int encode_results(const ResultSource& src, const tgo_result_args* a, const int32_t* perm, int64_t n,
                   int64_t* const scratch[4], void*& cub_tmp, size_t& cub_bytes, ResultRows* out, hipStream_t st,
                   std::string& err);

// Weight value marking an edge whose weight property is absent: traversing it makes the
// reference throw inside execute() (edge.value() on a missing key), i.e. TGO_E_PROGRAM.
constexpr int32_t kMissingWeight = INT32_MIN;

int build_plan(const tgo_schema* schema, const tgo_load_opts* opts, HostPlan& hp, std::string& err);
// tgo_decode_edge_entry body (graph_build.cpp).
int decode_one_entry(const tgo_schema* schema, const tgo_load_opts* opts, const uint8_t* entry,
                     int64_t len, int64_t value_pos, tgo_edge_entry* out, std::string& err);

int staging_begin(RowStaging& st, const tgo_load_opts* opts, std::string& err);
// Grow-only device buffer (the device decoder reuses its buffers across row batches).
template <class T>
struct DBuf {
    T* p = nullptr;
    int64_t cap = 0;
    hipError_t grow(int64_t need) {
        if (need <= cap) return hipSuccess;
        if (p) (void)hipFree(p);
        p = nullptr;
        cap = 0;
        const int64_t c = std::max<int64_t>(need, 1) + need / 4;
        const hipError_t e = hipMalloc(&p, static_cast<size_t>(c) * sizeof(T));
        if (e == hipSuccess) cap = c;
        return e;
    }
    void release() { if (p) (void)hipFree(p); p = nullptr; cap = 0; }
    // host -> device append after the first `used` elements (a grow keeps them)
    hipError_t append(const T* h, int64_t n, int64_t used, hipStream_t s) {
        if (n <= 0) return hipSuccess;
        if (used + n > cap) {
            T* np = nullptr;
            const int64_t c = std::max<int64_t>(2 * cap, used + n);
            hipError_t e = hipMalloc(&np, static_cast<size_t>(c) * sizeof(T));
            if (e != hipSuccess) return e;
            if (used > 0) e = hipMemcpyAsync(np, p, static_cast<size_t>(used) * sizeof(T), hipMemcpyDeviceToDevice, s);
            if (e == hipSuccess) e = hipStreamSynchronize(s);
            if (e != hipSuccess) { (void)hipFree(np); return e; }
            if (p) (void)hipFree(p);
            p = np;
            cap = c;
        }
        return hipMemcpyAsync(p + used, h, static_cast<size_t>(n) * sizeof(T), hipMemcpyHostToDevice, s);
    }
};
struct DecodeScratch {
    DBuf<int64_t> keys, eb, bb, lv, vid, first, keep, koff, other, plan_keys, ks, c_other, wv, c_wv;
    DBuf<uint8_t> bytes, rep, dir, sel, plan_labels, c_dir;
    DBuf<int8_t> plan_kdts, plan_dts;
    DBuf<int32_t> status, w, err, c_w;
    int64_t bytes_used = 0, lv_used = 0;   // raw work blocks staged on the device so far
    DBuf<unsigned long long> trunc;
    void* cub_tmp = nullptr;
    size_t cub_bytes = 0;
    void release();
};
// The same decode as decode_rows, on the device (decode.hip): the batch is uploaded, one
// kernel classifies rows (key filter, ghost check, user-edge slice, cap) and one decodes
// every kept entry; the staging arrays come back to the host.
int stage_rows_raw(RowStaging& st, const tgo_rows* rows, const tgo_schema* schema, const tgo_load_opts* opts,
                   DecodeScratch& ds, hipStream_t stream, std::string& err);
int decode_staged_raw(RowStaging& st, int pb, int64_t hard_limit, DecodeScratch& ds, hipStream_t stream,
                      std::string& err,
                      bool device_entries = false);
// Device-resident staged entries (decode_staged_raw with device_entries) to the host vectors.
int staging_entries_to_host(RowStaging& st, hipStream_t stream, std::string& err);
int decode_rows(RowStaging& st, const tgo_rows* rows, const tgo_schema* schema,
                const tgo_load_opts* opts, int pb, int64_t hard_limit, int threads,
                std::string& err);
int assemble_from_rows(RowStaging& st, HostGraph& g, int threads, std::string& err);
int assemble_from_edges(const tgo_edges* e, const tgo_load_opts* opts, int64_t hard_limit,
                        HostGraph& g, int threads, std::string& err);
// hipMemcpy in pieces of at most 256 MiB: single pageable copies of several GiB (RMAT-27
// lists are 8.6 GB each) are split so no one staging transfer spans more than 2^32 bytes.
inline hipError_t copy_chunked(void* dst, const void* src, size_t bytes, hipMemcpyKind kind) {
    constexpr size_t kPiece = size_t(256) << 20;
    for (size_t o = 0; o < bytes; o += kPiece) {
        const hipError_t e = hipMemcpy(static_cast<char*>(dst) + o, static_cast<const char*>(src) + o,
                                       std::min(kPiece, bytes - o), kind);
        if (e != hipSuccess) return e;
    }
    return hipSuccess;
}
// Large device -> host copies (tmp_cache.cpp): through two pinned 64 MB buffers, each piece
// copied out by several host threads (a pageable hipMemcpy of GBs runs at a few GB/s); the
// device data must be complete (the producing stream synchronised).
hipError_t copy_d2h(void* dst, const void* src, size_t bytes);
// madvise(MADV_HUGEPAGE) over a large host buffer before its first touch (fewer page faults).
void advise_huge(void* p, size_t bytes);
// Resize a host vector for a large download: capacity reserved untouched, advised huge, then
// value-initialised (the zero fill faults 2 MB pages where the kernel allows them).
template <class T>
void host_resize(std::vector<T>& h, size_t count) {
    if (count * sizeof(T) >= (size_t(64) << 20) && h.capacity() < count) {
        std::vector<T>().swap(h);
        h.reserve(count);
        advise_huge(h.data(), count * sizeof(T));
    }
    h.resize(count);
}
// Large temporaries of the load-time device builds (tmp_cache.cpp): freed blocks >= 64 MB are
// reused by the next request they fit; tmp_trim releases them (every load entry point).
hipError_t tmp_alloc(void** p, size_t bytes);
void tmp_free(void* p, size_t bytes);
void tmp_disown(void* p);          // a tmp_alloc block taken over for good (freed with hipFree)
void tmp_trim();
// The same graph assembled on the device (assemble.hip): radix sorts instead of the host
// counting sorts; m < 2^32.
int assemble_edges_device(const tgo_edges* e, const tgo_load_opts* opts, int64_t hard_limit, HostGraph& g,
                          hipStream_t s, std::string& err);
// assemble_from_rows on the device (no vertex cuts: the caller keeps those on the host path)
int assemble_rows_device(RowStaging& st, HostGraph& g, hipStream_t s, std::string& err);
// tgo_load_csr: the caller's rows as device-resident staging (each row's OUT entries then its
// IN entries, neighbour Titan ids), for assemble_rows_device / assemble_from_rows.
struct CsrInput {
    int64_t n;
    const int64_t* titan_ids;
    const int64_t* off[2];
    const int32_t* idx[2];
    const int32_t* w[2];
};
int stage_csr_device(const CsrInput& in, bool weighted, RowStaging& st, hipStream_t s, std::string& err);
int partition_layout(const tgo_edges* e, int64_t n_global, int64_t lo, int64_t hi, int threads,
                     int32_t* layout_local, std::string& err);
int assemble_partition(const tgo_edges* e, int64_t n_global, int64_t lo, int64_t hi,
                       const tgo_load_opts* opts, int64_t hard_limit, const int32_t* layout, HostGraph& g,
                       int threads, std::string& err);
// 1-D partition from edgestore rows (tgo_load_partition_rows; graph_build.cpp): this rank's
// decoded rows over global slot ids r * S + i, its layout, and the push view's exchange pairs.
int assemble_partition_rows(RowStaging& st, const std::vector<int64_t>& slot_vid, int64_t S, int rank,
                            HostGraph& g, int threads, std::string& err);
void partition_rows_layout(const HostGraph& g, int64_t lo, int32_t* layout_local);
int apply_partition_layout(HostGraph& g, int64_t lo, const int32_t* layout, int threads, std::string& err);
void partition_pull_pairs(const HostGraph& g, int64_t lo, int64_t S, int world, std::vector<int64_t>& counts,
                          std::vector<int64_t>& pairs);
void partition_push_from_pairs(HostGraph& g, const int64_t* pairs, int64_t npairs);
// assemble_partition on the device (assemble.hip), array for array; m < 2^32.
int assemble_partition_device(const tgo_edges* e, int64_t n_global, int64_t lo, int64_t hi, const tgo_load_opts* opts,
                              int64_t hard_limit, const int32_t* layout, HostGraph& g, hipStream_t s, std::string& err);

// ---------------------------------------------------------------- device graph
struct DevCsr {
    int64_t* off = nullptr;
    int32_t* adj = nullptr;
    int32_t* w = nullptr;
    uint32_t* col = nullptr;    // column position of every entry (TGO_LOAD_COLUMN_ORDER loads)
    int64_t nnz = 0;
};

// A list view handed to kernels: up to two CSRs walked back to back per vertex.
struct View {
    const int64_t* off0; const int32_t* adj0; const int32_t* w0;
    const int64_t* off1; const int32_t* adj1; const int32_t* w1;
    int nlists;
};

// A multi-source pull level split at a neighbour id (msbfs.hip): the walk reads neighbours
// < hot_lim only; rows it leaves open get acc / need for the blocked cold pass (ms_cold).
struct MsColdSplit {
    int32_t hot_lim = 0x7FFFFFFF;   // INT32_MAX: no split
    uint64_t* acc = nullptr;        // n: the open rows' partial masks
    uint8_t* need = nullptr;        // n: 1 = the row waits for the cold pass (ms_finish resets)
};

// Row blocks for the CSR-adaptive gather (PageRank / walk counts), built on the host.
struct RowBlocks {
    int64_t nblocks = 0;        // short-row blocks
    int64_t* blk = nullptr;     // nblocks+1 row boundaries (device)
    int64_t nchunks = 0;        // chunks of long rows
    int64_t* chunk_row = nullptr;   // per chunk: row
    int64_t* chunk_beg = nullptr;   // per chunk: first entry
    int64_t* chunk_end = nullptr;
    int64_t nlong = 0;          // long rows
    int64_t* long_row = nullptr;    // per long row: row id
    int64_t* long_chunk = nullptr;  // nlong+1: chunk index range
    int64_t* bdesc = nullptr;   // 2*(nblocks+1): {first row, first entry} of every block — one
                                // load per bound instead of blk -> off (gather_hot_pf)
    std::vector<int64_t> h_blk;
};

// Cache-blocked PageRank gather.  The update is bound by L2 misses: every
// random 8-byte gather that misses the XCD's 4 MB L2 costs one 128-byte fabric request,
// served at ~55 G requests/s chip-wide whether the line sits in the Infinity Cache or in HBM
// (profiles/r02f_pmc_calibration.txt).  So the in-lists are split by source:
//   hot  : sources < hot (the hottest after the degree-grouped relabel; their messages fit
//          in L2) -> gathered row by row as before, in a compact hot CSR;
//   cold : sources >= hot, cut into segments of `seg` sources (a 2 MB slice of the message
//          vector).  Segment s belongs to XCD s % 8 and its workgroups are launched at
//          blockIdx % 8 == s % 8 in segment order, so each XCD's L2 holds the slice it is
//          working on and every cold gather hits L2.  Each (row, segment) run of entries is
//          a "piece" (split at kTile entries) whose sum is written to partial[piece] in piece
//          order (streaming writes; row-major slots measured slower: the scattered 8-byte
//          writes cost more than they save, profiles/r02n_pr_probe.log); cold_fold adds each
//          row's pieces (segment order) into csum[row], which the hot pass adds to its sum.
// Every sum has a fixed order: results are bitwise reproducible run to run.
struct XcdBase { int64_t b[9]; };
constexpr int kPackShift = 12;              // packed tile entry = source << 12 | slot (kTile <= 4096)           // XCD x owns cold blocks [b[x], b[x+1]) of xblk
struct ColdBlocks {
    int64_t hot = 0, seg = 0, npieces = 0, nblocks = 0, max_xcd_blocks = 0;
    DevCsr hcsr;                // hot CSR (n+1 offsets, hot entries)
    int64_t* poff = nullptr;    // npieces+1: piece -> entry range in cadj
    int32_t* cadj = nullptr;    // cold entries, segment-major, row order inside a segment
    uint32_t* cptr = nullptr;   // n+1: row -> its pieces in cpid
    int32_t* cpid = nullptr;    // pieces of each row, segment order
    int64_t* bbeg = nullptr;    // per cold block: first piece
    int64_t* bend = nullptr;    // per cold block: end piece
    int32_t* xblk = nullptr;    // cold blocks in XCD-major launch order
    int32_t* bsrc = nullptr;    // per cold block: first source of its segment (packed tiles)
    int64_t* cdesc = nullptr;   // 4 per launch slot j (xblk order): {first piece, end piece,
                                // first entry, bsrc << 16 | entries} — one load for the chain
                                // xblk -> bbeg/bend -> poff (cold_gather, prefetching form)
    bool cpacked = false;       // cold tiles source-sorted and packed relative to bsrc
    bool cfx = false;           // cold tiles for cold_fx (fixed-point piece sums, cfx_desc): up to
                                // 4096 pieces and TGO_PR_FX_CE entries, packed (source - bsrc) << 12 | piece - first
    int64_t* cfx_desc = nullptr;   // 4 per launch slot j (xblk order): first entry, end entry, first piece, bsrc << 16 | pieces
    int cfx_shift = 12;            // piece-id bits of a packed cold entry (13 for 8192-piece tiles)
    double* partial = nullptr;  // npieces, in piece order (streaming writes)
    double* csum = nullptr;     // n_rows: per-row cold sums (cold_fold; 0 for rows without pieces)
    int32_t* crow = nullptr;    // rows that own cold pieces (ascending)
    int64_t n_crows = 0;
    int64_t n_rows = 0;         // rows the hot pass updates: [0, n_active) — the rest have no entries
    XcdBase xbase{};
    RowBlocks rb_hot;           // CSR-adaptive blocks of the hot CSR
    bool packed = false;        // hot CSR tiles source-sorted and packed (pack_tiles)
    int hot_tile = 4096;        // entries per hot tile (TGO_PR_HOT_TILE: 4096, 8192 or 16384)
    int hot_shift = 12;         // packed hot entry = source << hot_shift | slot (log2 hot_tile)
    int hot_pipe = 0;           // hot pass as persistent workgroups that gather tile t+1 while
                                // reducing tile t (TGO_PR_HOT_PIPE; gather_hot_pipe)
    int num_cus = 256;          // persistent grid: workgroups per CU x CUs
    // LDS window pass (lds_window, spmv.hip): the rows' entries with source < win come from a
    // copy of contrib[0, win) in LDS instead of L2 gathers; the pass writes every row's window
    // sum into csum, which cold_fold then accumulates onto (win = 0: no window)
    int64_t win = 0;
    int64_t* woff = nullptr;    // n_rows+1
    uint16_t* widx = nullptr;   // window entries (source ids < win), row-major
    RowBlocks rb_win;           // CSR-adaptive blocks of the window CSR (bdesc used)
    // Fixed-point hot pass (gather_hot_fx, spmv.hip): super-tiles of <= 2^fx_rbits rows and <=
    // TGO_PR_FX_E entries (pack_supertiles_device), entries source-sorted and packed as
    // source << fx_rbits | row - first row; sums are 128-bit fixed-point integers (exact,
    // order-free), so a tile needs one LDS accumulator per row instead of one slot per entry
    bool fx = false;
    int fx_rbits = 12;
    int64_t fx_ntiles = 0;
    int64_t* fx_desc = nullptr;         // 4 per tile: first entry, end entry, first row, rows or -(long + 1)
    int64_t fx_nlong = 0;
    int32_t* fx_long_row = nullptr;     // rows longer than a tile
    unsigned long long* fx_long_acc = nullptr;   // 2 per long row (low, high word), zero between updates
    // source-split hot pass (TGO_PR_FX_SPLIT = S, off by default since round 6): S launches over S ranges of the hot sources, so
    // each launch's messages fit an XCD's L2; the row sums carried between them in fx_part
    int fx_split = 0;
    int64_t* fx_mid = nullptr;          // (S + 1) per tile: its entry bounds of the source ranges
    unsigned long long* fx_part = nullptr;       // 2 per hot row (low, high word)
    // exact range of the fixed-point passes (fx or cfx; spmv.hip FxGuard): nonzero messages with
    // a biased exponent outside [fx_elo, fx_ehi) set *fx_bad, and the program re-runs on the plain
    // fp64 gather (fx_ehi from the longest in-list: a row of D entries stays below 2^47)
    int fx_elo = 0, fx_ehi = 0x800;
    unsigned* fx_bad = nullptr;
};
struct HostColdBlocks {
    int64_t hot = 0, seg = 0;
    // LDS window (device build only): sources [0, win) of every row, as uint16, row-major —
    // woff (n+1) and the entries; the hot CSR then holds sources [win, hot)
    int64_t win = 0;
    std::vector<int64_t> woff;
    std::vector<uint16_t> widx;         // host build
    DevArray<uint16_t> d_widx;          // device build
    std::vector<int64_t> hoff, poff, bbeg, bend;
    std::vector<int32_t> hadj, cadj, cpid, xblk, crow, bsrc;
    DevArray<int32_t> d_hadj, d_cadj;   // the device build keeps hadj / cadj on the device
    bool cpacked = false;
    std::vector<uint32_t> cptr;
    XcdBase xbase{};
    int64_t max_xcd_blocks = 0;
    bool cfx = false;                   // cold tiles packed for cold_fx: (source - base) << cfx_shift | piece - first piece
    int cfx_shift = 12;
};
// Builds the split of a CSR (entries = source ids) at hot / seg (see ColdBlocks); returns
// false when nothing is cold (n <= hot) or the piece count overflows 32-bit indices.
bool build_cold_blocks(const std::vector<int64_t>& off, const std::vector<int32_t>& adj, int64_t n_src,
                       int64_t hot, int64_t seg, int64_t tile, int64_t max_pieces, int threads, bool pack,
                       HostColdBlocks& hc, int64_t win = 0);
// pr_layout.hip: build_cold_blocks / pack_tiles on the device (same arrays)
int pack_supertiles_device(int32_t* d_adj, const int64_t* d_off, const std::vector<int64_t>& off, int64_t n_rows,
                           int64_t max_e, int rbits, std::vector<int64_t>& tdesc, std::vector<int32_t>& long_rows,
                           std::vector<int64_t>& long_len, hipStream_t s, std::string& err);
int build_cold_blocks_device(const int64_t* d_off, const int32_t* d_adj, int64_t n, int64_t nnz, int64_t n_src,
                             int64_t hot, int64_t seg, int64_t tile, int64_t max_pieces, bool pack, HostColdBlocks& hc,
                             bool& built, hipStream_t s, std::string& err, int64_t win = 0, bool fx = false);
int pack_tiles_device(int32_t* d_adj, int64_t m, const std::vector<int64_t>& tstart, const std::vector<int32_t>* tbase,
                      int shift, hipStream_t s, std::string& err);
// part_ghost.hip: the partitioned PageRank ghost exchange
int ghost_needs(const int32_t* d_adj, int64_t nnz, const int32_t* d_adj2, int64_t nnz2, int64_t nl, int rank, int world,
                int32_t** need, std::vector<int64_t>& need_count, hipStream_t s, std::string& err);
hipError_t k_pack_u64(const uint64_t* src, const int32_t* row, int64_t m, uint64_t* out, hipStream_t s);
hipError_t k_unpack_u64(const uint64_t* in, const int32_t* pos, int64_t m, uint64_t* g, hipStream_t s);
hipError_t k_gathered_pos(const int32_t* u, int64_t m, int64_t nl, int64_t A, int64_t H, int64_t W, int32_t* pos,
                          hipStream_t s);
hipError_t k_sub_i32(int32_t* v, int64_t m, int32_t by, hipStream_t s);
hipError_t k_pack_f64(const double* src, const int32_t* row, int64_t m, double* out, hipStream_t s);
hipError_t k_unpack_f64(const double* in, const int32_t* pos, int64_t m, double* g, hipStream_t s);
int sort_rows_device(const int64_t* d_off, int64_t n, int32_t* d_vals, int64_t m, hipStream_t s, std::string& err);
hipError_t k_part_gathered_index(const int32_t* in, int64_t m, int64_t nl, int64_t A, int64_t H, int64_t W, int32_t* out,
                                 int* bad, hipStream_t s);

struct DevGraph {
    int64_t n = 0;
    int32_t* perm = nullptr;    // row-order dense id -> internal id (device)
    int64_t n_active = 0;       // internal ids >= n_active have no entries (never reachable)
    DevCsr out, in, push_t;
    bool has_transpose = false;
    bool has_weight = false;
    int32_t weight_dt = TGO_DT_INTEGER;
    bool has_col = false;       // out.col / in.col hold column positions
    int32_t min_weight = 0, max_weight = 0;
    double mean_weight = 1.0;   // over present weights (delta-stepping's default bucket width)
    int64_t* wval = nullptr;    // Long / Double weight keys: the value table the weight column indexes
    int32_t scope = TGO_SCOPE_BOTH_E;
    bool partitioned = false;   // 1-D vertex partition: rows [lo, lo+n) of an n_global graph
    int64_t lo = 0, n_global = 0;
    RowBlocks rb_out, rb_in;    // CSR-adaptive blocks per pull list
    bool rb_out_ready = false, rb_in_ready = false;
    DevCsr push_ws;             // weighted loads: push entries sorted by weight (light/heavy delta-stepping)
    bool push_ws_ready = false;
    ColdBlocks cold_in;         // cache-blocked in-lists (one-GPU PageRank)
    bool cold_in_ready = false;
    // split first pull level of the multi-source sweep (built on its first use, per scope)
    int32_t* msc_adj = nullptr;     // cold entries' neighbours, (segment, row) order
    int32_t* msc_row = nullptr;     // and rows
    int64_t msc_C = 0;
    int32_t msc_hot = 0;
    int32_t msc_scope = -1;         // scope the layout was built for (-1: none yet)
    int64_t msc_req = 0;            // and its hot head
};

// Multi-source BFS levels as bit planes: the level of (v, source r) is
// sum_k ((p[k * stride + v] >> r) & 1) << k; levels < 2^kLevelPlanes (uint16 range).
constexpr int kLevelPlanes = 16;
struct LevelPlanes {
    uint64_t* p;
    int64_t stride;
};

// Device scratch reused across programs (allocated on first use, sized for n).
struct Counters {               // device-side level counters (one cache line each)
    unsigned long long qlen;    // next-queue length
    unsigned long long pad0[7];
    unsigned long long mf;      // sum of push degrees of the next frontier
    unsigned long long pad1[7];
    unsigned long long err;     // program failure flag
    unsigned long long pad2[7];
    unsigned long long red[2];  // reductions (reached vertices, reached entries)
    unsigned long long red2;    // third reduction (delta-stepping: bucket members left)
    unsigned long long pad3[5];
};

// State of the device-driven delta-stepping loop (delta_loop.hip), in device memory.
constexpr int kDsCountShift = 35;   // queue counters: count << 35 | entries (one atomic reserves both):
                                    // counts < 2^29 (a queue holds <= 2n + 2 takes: n <= 2^28 - 1),
                                    // entries < 2^35 (RMAT-27 bothE: 2^32)
static_assert((int64_t(1) << (64 - kDsCountShift)) > 2 * (int64_t(1) << 27) + 2,
              "the device delta loop must hold a scale-27 queue (api.cpp run_delta_split guard)");
// Binned form (kDsMaxBins piles): a relaxation that improves a vertex to a distance of a later
// bucket appends it to that bucket's pile; the next bucket is extracted from its pile, not by
// a scan of the whole pending bitmap (delta_loop.hip).
constexpr int kDsMaxBins = 32;
struct DsLoop {
    unsigned long long qc[2];   // per queue buffer
    long long tm;               // smallest improvement since the last extraction that queued nothing
    long long lo;               // smallest distance the last extraction left pending
    long long thr;              // bucket threshold
    unsigned long long extract; // ds_decide -> extraction this step: 0 none, 1 bitmap scan, 2 piles
    unsigned long long members; // a bucket member was marked since the last extraction
    unsigned long long done, err;
    unsigned long long phases, relaxed, buckets, extractions;
    // binned loop
    long long bucket;           // current bucket: thr = (bucket + 1) * delta
    long long xbin;             // pile of the decided extraction (-1: members only)
    unsigned long long xcount;  // its entries
    unsigned long long xm;      // member-list entries of the decided extraction
    unsigned long long mcount;  // member list length
    unsigned long long overflow;          // bit b: pile b dropped entries (its bucket is scanned)
    unsigned long long spill;   // a candidate beyond the piles' reach (cannot happen when the
                                // piles cover the largest weight; the host then reruns unbinned)
    unsigned long long full_scans;        // extractions by the bitmap scan (large or overflowed piles)
    unsigned long long xfin;    // the decided extraction follows a finished single bucket (members final)
    long long mlo;              // lowest bucket of the current range: a jump over empty piles
                                // while the finished bucket's heavy entries are pushed lets
                                // them land in the skipped buckets, which merge into the range
                                // [mlo, bucket]; only a single-bucket range has final members
    // pull form of a large finished bucket's heavy entries (ds_pull_heavy)
    unsigned long long xpull;   // this step pulls instead of queueing the members' heavy entries
    unsigned long long pulls;   // pulls so far (pull j uses bitmap / list j & 1)
    long long pbucket;          // the finished bucket of the current pull
    unsigned long long pcount[2];         // members recorded per list
    unsigned long long xprev;   // entries of the previous pull's list the extraction clears
    unsigned long long bc[kDsMaxBins];    // pile counts
    // small-step mode (ds_small_steps): the queue buffer in use, kept on the device because
    // one launch runs a varying number of steps, and the step the launch left to the grid
    // kernels: 0 none, 1 extract + commit + relax, 2 relax only
    unsigned long long cur;
    unsigned long long big;
    unsigned long long small_steps;       // steps the single-block kernel ran
    // partitioned loop (ds_part_extract): the extraction's pending minimum, moved into lo by
    // the next header (after every block of the extraction has added to it)
    long long lo_next;
    unsigned long long xnew;    // an extraction ran since the last header
};

struct Scratch {
    static constexpr int kDrvSlots = 24;
    void* drv[kDrvSlots] = {};  // partitioned C++ driver buffers (part_driver.cpp), by slot:
    int64_t drv_bytes[kDrvSlots] = {};   // 0-7 multi-source sweep, 8-12 BFS, 13-17 SSSP, 18-23 PageRank
    int64_t n = 0;
    int32_t* level = nullptr;       // n
    int32_t* q[2] = {nullptr, nullptr};   // frontier queues
    int64_t* qdeg = nullptr;        // push degree of each queue entry
    int64_t* qpre = nullptr;        // exclusive scan of qdeg (+1)
    uint64_t* fb = nullptr;         // frontier bitmap
    uint64_t* nb = nullptr;         // next-frontier bitmap
    uint64_t* vb = nullptr;         // visited bitmap
    int64_t* dist = nullptr;        // n: int64 distances / messages
    int64_t* msg = nullptr;         // n: SSSP message snapshot
    double* vec[3] = {nullptr, nullptr, nullptr};  // PageRank vectors
    double* partial = nullptr;      // long-row partial sums
    int64_t partial_cap = 0;
    void* cub_tmp = nullptr;
    size_t cub_bytes = 0;
    Counters* cnt = nullptr;        // device
    Counters* hcnt = nullptr;       // host mirror: fine-grained (coherent) pinned memory, mapped
    unsigned long long* hcnt_dev = nullptr;   // its device address; word kCounterWords = seq
    unsigned long long pub_seq = 0; // last published sequence number
    // multi-source BFS (allocated on first use)
    uint64_t* ms_vis = nullptr;     // n: reached-by mask
    uint64_t* ms_fbm = nullptr;     // n/64: frontier bitmap of a pull level (fr != 0)
    unsigned long long* ms_srcent = nullptr;   // 64: per-source frontier sizes of a pull level
    int64_t* ms_rp[2] = {nullptr, nullptr};    // ranged push: list bounds per (entry, range), kMsRangePairs each
    uint64_t* ms_fr = nullptr;      // n: frontier mask
    uint64_t* ms_nx = nullptr;      // n: next-frontier mask
    uint64_t* ms_lvl = nullptr;     // kLevelPlanes x n: bit r of plane k = bit k of source r's level
    int32_t ms_nplanes = 0;         // planes zeroed (and valid) in the current sweep
    int64_t* ms_seeds = nullptr;    // 64
    unsigned long long* ms_stat = nullptr;   // 128: reached[64], entries[64]
    int32_t ms_nsrc = 0;
    int* pk_ovf = nullptr;          // fixed-capacity exchange overflow flag (checked at ms_end)
    uint8_t* pk_touch = nullptr;    // per pack chunk: written by this level's push (PackTouch)
    int64_t* pk_cnt = nullptr;      // partitioned sparse exchange: per-chunk pair counts
    int64_t* pk_off = nullptr;      // and their exclusive scan (n_global / kPackChunk + 1 each)
    // light/heavy delta-stepping (allocated on first use)
    int64_t* ds_light = nullptr;    // n: end of each vertex's light entries in push_ws
    int64_t ds_light_delta = -1;    // bucket width ds_light was computed for
    uint64_t* ds_member = nullptr;  // words: vertices relaxed in the current bucket
    int32_t* ds_q[2] = {nullptr, nullptr};    // device-driven loop: queues (2n + 2: light + heavy)
    int64_t* ds_qp[2] = {nullptr, nullptr};   // and their entry offsets
    DsLoop* ds_loop = nullptr;
    uint64_t* ms_cacc = nullptr;    // split pull: partial masks of the rows left to the cold pass
    uint8_t* ms_need = nullptr;     // and their flags (n, zero between levels)
    int32_t* ds_pile = nullptr;     // binned loop: kDsMaxBins piles of ds_pile_cap vertices
    int64_t ds_pile_cap = 0;
    int32_t* ds_mlist = nullptr;    // n: members of the current bucket
    uint64_t* ds_done = nullptr;    // words: members of finished buckets (final distances)
    uint64_t* ds_pm[2] = {nullptr, nullptr};   // pull form: member bitmaps (words) and lists (n)
    int32_t* ds_pl[2] = {nullptr, nullptr};
    // generic vertex programs (allocated on first use): row-order staging + internal-order vectors
    int64_t* gv[3] = {nullptr, nullptr, nullptr};
    uint8_t* gh[3] = {nullptr, nullptr, nullptr};
    void* sort_tmp = nullptr;
    size_t sort_bytes = 0;
    // partitioned delta-stepping (allocated on first use)
    int64_t* ds_rbest = nullptr;    // n_global: best distance sent to each remote vertex
    uint64_t* ds_rmark = nullptr;   // n_global bits: remote vertices improved this phase
    unsigned long long* ds_pack = nullptr;   // 3 x kMaxRanks: counts, offsets, cursors
    DevCsr ds_pws;                  // the push view split at ds_light_delta (k_ds_split_rows)
};

constexpr int kMaxRanks = 64;

// ---------------------------------------------------------------- kernel launchers (HIP)
hipError_t k_fill_i32(int32_t* p, int32_t v, int64_t n, hipStream_t s);
hipError_t k_fill_i64(int64_t* p, int64_t v, int64_t n, hipStream_t s);
hipError_t k_bfs_seed(const View& push, int32_t* level, uint64_t* vb, uint64_t* fb, int32_t* q,
                      int64_t* qdeg, int64_t seed, hipStream_t s);
hipError_t k_td_expand(const View& push, const int32_t* q, const int64_t* qpre, int64_t qlen,
                       int32_t* level, uint64_t* vb, uint64_t* nb, int32_t* qn, int64_t* qdeg_n,
                       Counters* cnt, int32_t next_level, hipStream_t s);
// bottom-up level: counts the next frontier (qlen, mf) without queueing it (k_bfs_queue)
hipError_t k_bu_step(const View& pull, const View& push, int64_t n, const uint64_t* fb, uint64_t* vb, uint64_t* nb,
                     int32_t* level, Counters* cnt, int32_t next_level, hipStream_t s);
hipError_t k_bfs_queue(const View& push, int64_t n, const uint64_t* fb, int32_t* qn, int64_t* qdeg, Counters* cnt,
                       hipStream_t s);
hipError_t k_level_to_dist(const int32_t* level, int64_t* dist, int64_t n, hipStream_t s);
hipError_t k_publish_counts(const Counters* c, int64_t* out, int64_t* slot, hipStream_t s);
// Level control without a copy + stream synchronisation: one wave stores the counters into the
// host-mapped mirror, then the sequence number after them (system scope); the host spins on it.
constexpr int kCounterWords = static_cast<int>(sizeof(Counters) / 8);
hipError_t k_publish_counters(const Counters* c, unsigned long long* host, unsigned long long seq, hipStream_t s);
// `count` (<= kCounterWords) device words published like the counters (partitioned drivers)
// The delta loop's done / err / spill flags to host-mapped words 0..2 and the sequence number.
hipError_t k_ds_publish(const DsLoop* L, unsigned long long* host, unsigned long long seq, hipStream_t s);
hipError_t k_publish_words(const int64_t* src, int count, unsigned long long* host, unsigned long long seq, hipStream_t s);
hipError_t k_level_turn(Counters* c, unsigned long long* host, unsigned long long seq, uint64_t* clear, int64_t words,
                        int64_t* qdeg, hipStream_t s);
// One launch instead of per-level memsets: zero the counters (cnt may be null), the next
// frontier bitmap (words, may be 0) and the scan tail slot (may be null).
hipError_t k_level_prep(Counters* cnt, uint64_t* nb, int64_t words, int64_t* tail, hipStream_t s);
hipError_t k_reach_stats(const View& both_or_pull, const int64_t* dist, int64_t n,
                         unsigned long long* out2, hipStream_t s);
hipError_t k_degree_i64(const View& v, const int32_t* q, int64_t qlen, int64_t* qdeg, hipStream_t s);

// SSSP (hop-bounded Jacobi, exact reference semantics)
hipError_t k_sssp_seed(const View& push, int64_t* dist, int64_t* msg, uint64_t* vb, int32_t* q,
                       int64_t* qdeg, int64_t seed, hipStream_t s);
hipError_t k_sssp_relax(const View& push, const int32_t* q, const int64_t* qpre, int64_t qlen,
                        const int64_t* msg, int64_t* dist, uint64_t* mark, int32_t* qn,
                        int64_t* qdeg_n, Counters* cnt, int weighted, hipStream_t s);
hipError_t k_sssp_commit(const int32_t* q, int64_t qlen, const int64_t* dist, int64_t* msg,
                         uint64_t* mark, hipStream_t s);
hipError_t k_dist_finalize(int64_t* dist, int64_t n, hipStream_t s);

// SSSP (delta-stepping, converged distances) — delta.hip
hipError_t k_ds_seed(const View& push, int64_t* dist, int32_t* q, int64_t* qdeg, int64_t seed, hipStream_t s);
hipError_t k_ds_commit(const int32_t* q, int64_t qlen, const int64_t* dist, int64_t* msg, uint64_t* pend, hipStream_t s);
hipError_t k_ds_relax(const View& push, const int32_t* q, const int64_t* qpre, int64_t qlen, const int64_t* msg,
                      int64_t* dist, uint64_t* pend, int32_t* qn, int64_t* qdeg_n, Counters* cnt, int weighted,
                      int64_t thr, hipStream_t s);
// light/heavy delta-stepping over the weight-sorted push lists (delta.hip)
hipError_t k_ds_light_end(const DevCsr& ws, int64_t delta, int64_t n, int64_t* light, hipStream_t s);
hipError_t k_ds_seed_ws(const DevCsr& ws, const int64_t* light, int64_t* dist, int32_t* q, int64_t* qdeg, int64_t seed,
                        hipStream_t s);
// track (partitioned, see ds_track_reset): pending-minimum / member state, nullptr on one GPU
hipError_t k_ds_commit_ws(const int32_t* q, int64_t qlen, const int64_t* dist, int64_t* msg, uint64_t* pend,
                          uint64_t* member, int64_t* qdeg, Counters* cnt, hipStream_t s, long long* track = nullptr);
hipError_t k_ds_relax_ws(const DevCsr& ws, const int64_t* light, const int32_t* q, const int64_t* qpre, int64_t qlen,
                         const int64_t* msg, int64_t* dist, uint64_t* pend, int32_t* qn, int64_t* qdeg_n, Counters* cnt,
                         int64_t thr, hipStream_t s);
// partitioned: remote targets to rbest / rmark (as k_ds_relax_part)
hipError_t k_ds_relax_ws_part(const DevCsr& ws, const int64_t* light, const int32_t* q, const int64_t* qpre, int64_t qlen,
                              const int64_t* msg, int64_t* dist, uint64_t* pend, int32_t* qn, int64_t* qdeg_n,
                              Counters* cnt, int64_t thr, int64_t lo, int64_t n_local, int64_t* rbest, uint64_t* rmark,
                              long long* track, hipStream_t s);
// partitioned loads: ws (off n+1, adj / w push-view nnz) = the push view with every row stably
// partitioned at delta (light entries first); light[v] = end of v's light run
hipError_t k_ds_split_rows(const View& push, int64_t n, int64_t delta, DevCsr& ws, int64_t* light, hipStream_t s);
hipError_t k_ds_extract_ws(const DevCsr& ws, const int64_t* light, uint64_t* pend, uint64_t* member, int64_t n,
                           const int64_t* dist, int64_t thr, int32_t* qn, int64_t* qdeg, Counters* cnt, hipStream_t s,
                           long long* track = nullptr);
hipError_t k_ds_pending_min_ws(const uint64_t* pend, const uint64_t* member, int64_t words, const int64_t* dist,
                               Counters* cnt, hipStream_t s);
// device-driven light/heavy loop (delta_loop.hip)
hipError_t k_ds_loop_seed(const DevCsr& ws, const int64_t* light, int64_t* dist, int32_t* q, int64_t* qpre, DsLoop* L,
                          int64_t seed, int64_t delta, hipStream_t s);
hipError_t k_ds_loop_step(const DevCsr& ws, const int64_t* light, uint64_t* pend, uint64_t* member, int64_t n,
                          int64_t* dist, int64_t* msg, int32_t* const q[2], int64_t* const qpre[2], DsLoop* L, int cur,
                          int64_t delta, hipStream_t s);
// the partitioned device loop (delta_loop.hip, 1-D partition section): commit + relax of queue
// cur (remote targets to rbest / rmark), the exchange header, the owner-side apply into queue
// cur ^ 1, and the extraction below thr after an empty global phase
hipError_t k_ds_part_relax(const DevCsr& ws, const int64_t* light, uint64_t* pend, uint64_t* member, int64_t* dist,
                           int64_t* msg, int32_t* const q[2], int64_t* const qpre[2], DsLoop* L, int cur, int64_t delta,
                           int64_t lo, int64_t n_local, int64_t* rbest, uint64_t* rmark, hipStream_t s);
hipError_t k_ds_part_header(unsigned long long* counts, int nranks, DsLoop* L, int cur, unsigned long long* offs,
                            unsigned long long* cursor, int64_t* sizes, hipStream_t s, unsigned long long* host = nullptr,
                            unsigned long long seq = 0);
hipError_t k_ds_part_apply(const int64_t* recv, int64_t npairs, const DevCsr& ws, const int64_t* light, int64_t* dist,
                           uint64_t* pend, int32_t* const q[2], int64_t* const qpre[2], DsLoop* L, int cur, hipStream_t s);
hipError_t k_ds_part_extract(const DevCsr& ws, const int64_t* light, uint64_t* pend, uint64_t* member, int64_t n,
                             int64_t* dist, int32_t* const q[2], int64_t* const qpre[2], DsLoop* L, int cur, int64_t thr,
                             hipStream_t s);
// Pull form of the heavy entries of a finished bucket with >= min_members members: every
// vertex that can still improve reads its pull list (view) for heavy entries from those members
// (bitmap pm[j & 1], list pl[j & 1]) instead of the members pushing them.  min_members <= 0: off.
struct DsPull {
    View view{};
    int64_t n_active = 0;
    int64_t min_members = 0;
    uint64_t* pm[2] = {nullptr, nullptr};
    int32_t* pl[2] = {nullptr, nullptr};
};
// the binned form: nbins piles of cap entries (pile), member list mlist (n), done bitmap (words,
// zeroed by the caller: members of finished buckets)
hipError_t k_ds_loop_step_bins(const DevCsr& ws, const int64_t* light, uint64_t* pend, uint64_t* member, int64_t n,
                               int64_t* dist, int64_t* msg, int32_t* const q[2], int64_t* const qpre[2], DsLoop* L,
                               int cur, int64_t delta, int nbins, int32_t* pile, int64_t cap, int32_t* mlist,
                               uint64_t* done, bool done_filter, int64_t scan_above, const DsPull& pull,
                               hipStream_t s);
// the binned form with small steps (delta_loop.hip ds_small_steps): one launch runs the tiny
// steps in one block, then the grid kernels the step it stopped at; queue buffer on the device
// (DsLoop::cur).  Without the done filter and the pull form.
hipError_t k_ds_loop_step_small(const DevCsr& ws, const int64_t* light, uint64_t* pend, uint64_t* member, int64_t n,
                                int64_t* dist, int64_t* msg, int32_t* const q[2], int64_t* const qpre[2], DsLoop* L,
                                int64_t delta, int nbins, int32_t* pile, int64_t cap, int32_t* mlist, uint64_t* done,
                                int64_t scan_above, hipStream_t s);
hipError_t k_ds_pending_min(const uint64_t* pend, int64_t words, const int64_t* dist, Counters* cnt, hipStream_t s);
// partitioned loop state (delta.hip ds_track_reset): reset before an extraction; the header
// all-to-all's result folded into {sent W, received W, global queue, pending min, -members}
hipError_t k_ds_track_reset(long long* track, hipStream_t s);
hipError_t k_ds_header_fold(const int64_t* own, const int64_t* recv, int nranks, int64_t* out, hipStream_t s,
                            unsigned long long* host = nullptr, unsigned long long seq = 0);
hipError_t k_ds_extract(const View& push, uint64_t* pend, int64_t n, const int64_t* dist, int64_t thr, int32_t* qn,
                        int64_t* qdeg, Counters* cnt, hipStream_t s, long long* track = nullptr);
hipError_t k_ds_relax_part(const View& push, const int32_t* q, const int64_t* qpre, int64_t qlen, const int64_t* msg,
                           int64_t* dist, uint64_t* pend, int32_t* qn, int64_t* qdeg_n, Counters* cnt, int weighted,
                           int64_t thr, int64_t lo, int64_t n_local, int64_t* rbest, uint64_t* rmark, long long* track,
                           hipStream_t s);
hipError_t k_ds_mark_count(const uint64_t* rmark, int64_t words, int64_t wpr, unsigned long long* counts, hipStream_t s);
hipError_t k_ds_mark_pack(uint64_t* rmark, int64_t words, int64_t wpr, int64_t n_local, const int64_t* rbest,
                          const unsigned long long* offs, unsigned long long* cursor, int64_t* send, hipStream_t s);
// also zeroes counts and cursor (the next phase's count / this phase's pack start from 0)
hipError_t k_ds_mark_sizes(unsigned long long* counts, int nranks, int64_t qlen, unsigned long long* offs,
                           unsigned long long* cursor, const long long* track, int64_t* sizes, hipStream_t s);
hipError_t k_ds_apply(const View& push, const int64_t* recv, int64_t npairs, int64_t* dist, uint64_t* pend, int32_t* qn,
                      int64_t* qdeg_n, Counters* cnt, int64_t thr, const int64_t* ws_off, const int64_t* light,
                      long long* track, hipStream_t s);
hipError_t k_unpermute_i64(const int64_t* in, const int32_t* perm, int64_t* out, int64_t n, hipStream_t s);
hipError_t k_ms_seed(const int64_t* seeds, int nseeds, uint64_t* vis, uint64_t* fr, int64_t fr_rows, hipStream_t s);
hipError_t k_ms_diag_take(unsigned long long* out10, hipStream_t s);   // 10 diagnostic words
hipError_t k_ms_pull(const View& pull, const View& push, int64_t n_active, uint64_t full, const uint64_t* fr,
                     const uint64_t* fbm, uint64_t* vis, uint64_t* nx, LevelPlanes lvl, Counters* cnt,
                     int32_t next_level, hipStream_t s, int32_t filter_from, uint64_t dense = ~0ULL,
                     const uint64_t* cand = nullptr, MsColdSplit cs = MsColdSplit());
// the blocked cold pass and the settle of the rows it completed (msbfs.hip)
hipError_t k_ms_cold(const int32_t* cadj, const int32_t* crow, int64_t C, const uint64_t* fr, const uint8_t* need,
                     uint64_t* acc, hipStream_t s);
hipError_t k_ms_finish(const View& push, int64_t n_active, uint64_t full, uint64_t* vis, uint64_t* nx,
                       const uint64_t* cand, LevelPlanes lvl, Counters* cnt, int32_t next_level, uint8_t* need,
                       const uint64_t* acc, hipStream_t s);
hipError_t k_cold_flags(const int32_t* adj, int64_t m, int32_t hot, uint32_t* flag, hipStream_t s);
hipError_t k_cold_emit(const int64_t* off, int64_t n, const int32_t* adj, int64_t m, const uint32_t* flag,
                       const uint64_t* pos, int64_t base, int32_t hot, int64_t seg, uint64_t* key, int32_t* val,
                       hipStream_t s);
hipError_t k_low_rows(const uint64_t* key, int64_t m, int32_t* row, hipStream_t s);
// pr_layout.hip: the cold layout of a split pull (entries >= hot of both lists of v, sorted by
// (segment, row)); C = 0 when nothing is cold
int build_ms_cold(const View& v, int64_t n, int32_t hot, int64_t seg, DevArray<int32_t>& cadj, DevArray<int32_t>& crow,
                  int64_t& C, hipStream_t s, std::string& err);
// per-source frontier sizes of fr (out64[s], zeroed first) — the pull level's split
hipError_t k_ms_source_counts(const uint64_t* fr, int64_t n_active, unsigned long long* out64, hipStream_t s);
// exact push entries of the frontiers of the sources in `cand` (out64[s], zeroed first)
hipError_t k_ms_source_entries(const View& push, const uint64_t* fr, int64_t n_active, uint64_t cand,
                               unsigned long long* out64, hipStream_t s);
hipError_t k_ms_fbitmap(const uint64_t* fr, int64_t n, uint64_t* fbm, hipStream_t s);
hipError_t k_ms_queue(const View& push, int64_t n_active, const uint64_t* fr, int32_t* qn, int64_t* qdeg, Counters* cnt,
                      hipStream_t s, uint64_t mask = ~0ULL);
// Partitioned push: per-pack-chunk "written" flags (chunk of global word v: owner v / n_local,
// chunk (v % n_local) / kPackChunk of the owner's cps) so the pack skips untouched chunks.
struct PackTouch { uint8_t* flag = nullptr; int64_t n_local = 1; int64_t cps = 1; };
hipError_t k_ms_push(const View& push, const int32_t* q, const int64_t* qpre, int64_t qlen, const uint64_t* fr,
                     const uint64_t* vis, uint64_t* nx, hipStream_t s, PackTouch touch = {}, uint64_t mask = ~0ULL,
                     bool probe = true, uint64_t* own_nx = nullptr, int64_t own_lo = 0);
constexpr int64_t kMsRangePairs = int64_t(1) << 22;   // ranged push: (entry, range) bounds per list
// Target-ranged push of a small frontier (msbfs.hip): pairs (range of S targets, entry) in
// range-major order, XCD x on the x-th eighth; P0 / P1 hold qlen * (R + 1), cnt / pre R * qlen + 1.
hipError_t k_ms_push_ranged(const View& push, const int32_t* q, int64_t qlen, int64_t n_active, int64_t S,
                            int64_t* P0, int64_t* P1, int64_t* cnt, int64_t* pre, void*& tmp, size_t& tmp_bytes,
                            const uint64_t* fr, const uint64_t* vis, uint64_t* nx, hipStream_t s, uint64_t mask = ~0ULL);
// ms_settle without the queue (the next level pulls; counts only)
hipError_t k_ms_settle_count(const View& push, int64_t n_active, uint64_t* vis, uint64_t* nx, LevelPlanes lvl,
                            Counters* cnt, int32_t next_level, hipStream_t s, unsigned long long* srcent = nullptr);
hipError_t k_ms_settle(const View& push, int64_t n_active, uint64_t* vis, uint64_t* nx, LevelPlanes lvl, int32_t* qn,
                       int64_t* qdeg, Counters* cnt, int32_t next_level, hipStream_t s,
                       unsigned long long* srcent = nullptr);
hipError_t k_ms_reach(const View& v, const uint64_t* vis, int64_t n_active, int nsrc, unsigned long long* reached,
                      unsigned long long* entries, hipStream_t s);
hipError_t k_ms_extract(LevelPlanes lvl, int nplanes, const uint64_t* vis, const int32_t* perm, int r, int64_t* dist,
                        int64_t n, hipStream_t s);
hipError_t k_or_slices(const uint64_t* recv, int nslices, int64_t n_local, uint64_t* out, hipStream_t s);
constexpr int64_t kPackChunk = 2048;   // candidate words per wave in the sparse-exchange pack
hipError_t k_ms_pack(bool write, uint64_t* cand, int64_t n_local, int64_t cps, int64_t nchunks, int64_t* cnt,
                     const int64_t* offs, int64_t* send, hipStream_t s, uint8_t* touched = nullptr, int self = -1);
// the own slice left by a pack with self: OR into nx, cleared (touched chunks only)
hipError_t k_ms_or_local(uint64_t* cand_own, int64_t n_local, int64_t cps, uint8_t* touched_own, uint64_t* nx,
                         hipStream_t s);
hipError_t k_slice_elems(const int64_t* off, int64_t cps, int nranks, int64_t* out, hipStream_t s);
hipError_t k_ms_or_pairs(const int64_t* pairs, int64_t npairs, uint64_t* nx, hipStream_t s);
hipError_t k_ms_pack_fixed(uint64_t* cand, int64_t n_local, int64_t cps, int64_t nchunks, const int64_t* offs,
                           int nranks, int64_t cap, int64_t* send, int* ovf, uint8_t* touched, hipStream_t s,
                           int self = -1);
hipError_t k_ms_or_fixed(const int64_t* recv, int nslices, int64_t cap, uint64_t* nx, hipStream_t s);
hipError_t k_part_td_mark(const View& push, const int32_t* q, const int64_t* qpre, int64_t qlen,
                          uint64_t* disc, const uint64_t* vb_local, int64_t lo, int64_t n_local, hipStream_t s);
hipError_t k_part_claim(const View& push, const uint64_t* recv, int nslices, int64_t words, int64_t n_local,
                        uint64_t* vb, uint64_t* nb, int32_t* level, int32_t* qn, int64_t* qdeg_n,
                        Counters* cnt, int32_t next_level, hipStream_t s, bool or_into_nb = false);
hipError_t k_part_td_claim(const View& push, const int32_t* q, const int64_t* qpre, int64_t qlen, uint64_t* disc,
                           uint64_t* vb, uint64_t* nb, int32_t* level, int32_t* qn, int64_t* qdeg_n, Counters* cnt,
                           int32_t next_level, int64_t lo, int64_t n_local, hipStream_t s);
// tgo_part_bfs_run's top-down level (api.cpp): owned targets claimed during the expansion, remote
// ones marked in disc (world > 1) and claimed from the received slices into the same queue.
int part_bfs_td_fused(tgo_ctx* ctx, int32_t level, uint64_t* disc, uint64_t* nb_local);
int part_bfs_claim_remote(tgo_ctx* ctx, int32_t level, const uint64_t* recv, int32_t nslices, uint64_t* nb_local);
int part_bfs_level_done(tgo_ctx* ctx);
hipError_t k_unpermute_i32(const int32_t* in, const int32_t* perm, int32_t* out, int64_t n, hipStream_t s);

// PageRank gather diagnostics: [diag_lo, diag_hi) = only sources in this range are gathered
// (the others read as 0; results invalid) — attributes the update's time to source ranges.
struct PrTuning {
    int32_t diag_lo = 0, diag_hi = 0;
};

// CSR-adaptive gather
hipError_t k_pr_init(const DevCsr& out, double* edge_count, double* contrib, double* pr,
                     double inv_n, int64_t n, hipStream_t s);
hipError_t k_pr_iter(const DevCsr& in, const RowBlocks& rb, const double* contrib,
                     const double* edge_count, double* pr, double* contrib_next, double* partial,
                     double alpha, double base, int64_t n, const PrTuning& t, hipStream_t s);
hipError_t k_fill_f64(double* p, double v, int64_t n, hipStream_t s);
// guard_entries (the first rank update of a program): every gathered message is checked against
// the fixed-point passes' exact range (FxGuard); later updates check only the emitted
// contributions, one per row (PrFinal)
hipError_t k_pr_cold_phase(const ColdBlocks& cb, const double* contrib, hipStream_t s, bool guard_entries);
// per fixed-point hot tile (desc, packed source << rbits | row): the first entry with source >= hs
// first > 0: the first range is [0, first) (TGO_PR_FX_SPLIT_AT), else S even ranges
hipError_t k_fx_split_points(const uint32_t* padj, const int64_t* desc, int64_t ntiles, int rbits, int64_t hot,
                             int nsplit, int64_t first, int64_t* bnd, hipStream_t s);
hipError_t k_pr_hot_phase(const ColdBlocks& cb, const double* contrib, const double* edge_count, double* pr,
                          double* contrib_next, double* partial_long, double alpha, double base, hipStream_t s,
                          bool guard_entries);
hipError_t k_walk_iter(const DevCsr& out, const RowBlocks& rb, const int32_t* prev, int32_t* next,
                       int32_t* partial, int64_t n, hipStream_t s);

// Generic vertex programs (generic.hip)
// The weight column of a generic edge function: 32-bit integers (kind 0), a Float's IEEE bits
// (1), or indices into the Long (2) / Double (3, IEEE bits) value table `wide`.
struct WeightCol {
    int kind = 0;
    const int64_t* wide = nullptr;
};
// An edge-function program (tgo_set_edge_program, validated on the host), handed to the gather
// kernels by value: uniform across every lane, read through the kernel arguments.
struct EdgeProg {
    int32_t n = 0;                  // ops; 0 = none set
    int32_t uses_w = 0;             // pushes e.value(weight)
    int32_t has_i = 0, has_f = 0;   // long / double constants given
    int32_t ops[TGO_EDGE_PROGRAM_MAX_OPS] = {};
    int64_t ic[TGO_EDGE_PROGRAM_MAX_CONSTS] = {};
    double fc[TGO_EDGE_PROGRAM_MAX_CONSTS] = {};
};
hipError_t k_local_gather(const View& pull, int64_t n, int value_type, const void* msg_int, const uint8_t* has_int,
                          int comb, int fn, WeightCol wc, const EdgeProg& pg, void* out_int, uint8_t* out_has_int,
                          unsigned long long* err, hipStream_t s);
hipError_t k_list_count(const View& pull, const int32_t* perm, int64_t n, const uint8_t* has_int, bool needs_w,
                        int64_t* cnt, unsigned long long* err, hipStream_t s);
hipError_t k_list_fill_sort(const View& pull, const uint32_t* col0, const uint32_t* col1, const int32_t* perm,
                            int32_t* inv, int64_t n, int value_type, const void* msg_int, const uint8_t* has_int,
                            int fn, WeightCol wc, const EdgeProg& pg, const int64_t* off_out, int64_t total,
                            uint32_t* key_in, uint32_t* key_out, void* val_in, void* val_out, void*& tmp,
                            size_t& tmp_bytes, unsigned long long* err, hipStream_t s);
hipError_t k_to_internal(const void* row8, const uint8_t* row1, const int32_t* perm, void* int8, uint8_t* int1,
                         int64_t n, hipStream_t s);
hipError_t k_to_rows(const void* int8, const uint8_t* int1, const int32_t* perm, void* row8, uint8_t* row1, int64_t n,
                     hipStream_t s);
hipError_t k_global_combine(void*& tmp, size_t& tmp_bytes, const int64_t* targets, int64_t m, int64_t n,
                            int value_type, const void* values, int comb, int64_t* scratch3m, void* out,
                            uint8_t* out_has, hipStream_t s);

hipError_t scan_exclusive_i64(void*& tmp, size_t& tmp_bytes, const int64_t* in, int64_t* out,
                              int64_t n, hipStream_t s);

// Push entries of the loaded scope in one list per vertex sorted by (weight, target).
void weight_sorted_push(const HostGraph& g, HostCsr& ws, int threads);
// Source-sorted, packed tiles of a CSR (see graph_build.cpp); false if sources need > 19 bits.
// shift = log2 of the slot space (tile <= 1 << shift); sources must fit 32 - shift bits (the
// packed word is read as uint32 by kernels whose shift exceeds 12).
bool pack_tiles(const std::vector<int64_t>& off, std::vector<int32_t>& adj, const std::vector<int64_t>& blk,
                const std::vector<int64_t>& cbeg, const std::vector<int64_t>& cend, int64_t tile, int threads,
                int shift = kPackShift);
// Row-block construction (host) for a CSR.
void build_row_blocks(const std::vector<int64_t>& off, int64_t tile, int64_t max_rows,
                      std::vector<int64_t>& blk, std::vector<int64_t>& chunk_row,
                      std::vector<int64_t>& chunk_beg, std::vector<int64_t>& chunk_end,
                      std::vector<int64_t>& long_row, std::vector<int64_t>& long_chunk);
#ifndef TGO_KTILE
#define TGO_KTILE 4096
#endif
// entries per CSR-adaptive block (32 KB of fp64 in LDS; round 1: 2048 1.84, 8192 1.87 ms/update;
// TGO_KTILE builds a probe library with another size, scripts/gpu_ktile.sh)
constexpr int64_t kTile = TGO_KTILE;
constexpr int64_t kMaxRows = 1024;   // rows per CSR-adaptive block

}  // namespace tgo

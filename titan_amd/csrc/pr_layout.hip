// pr_layout.hip — the cache-blocked PageRank layout (engine.hpp ColdBlocks) built on the device.
//
// graph_build.cpp build_cold_blocks / pack_tiles restated as sorts over the device in-lists,
// array for array (TGO_HOST_ASSEMBLY=1 keeps the host build):
//   hot CSR     : each row's entries with source < hot (a prefix: rows are sorted by source)
//   cold pieces : the other entries grouped segment-major, rows in order inside a segment,
//                 list order inside a row ((segment, row) stable radix sort), cut into runs of
//                 one (row, segment) and at `tile` entries (a flag + scan);
//   cpid / cptr : every row's pieces in segment order (stable sort of the pieces by row);
//   blocks      : the greedy per-segment packing of pieces (<= tile entries, <= max_pieces
//                 pieces) — sequential, on the host from the piece offsets;
//   packing     : every cold block's and hot tile's entries sorted by source and packed as
//                 (source << 12 | slot) — one radix sort over (tile << 32 | packed) keys.
// The reference's update this layout feeds: PageRankVertexProgram.java:84-89.
#include <algorithm>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstdint>
#include <cstring>
#include <string>
#include <vector>

#include <hip/hip_runtime.h>
#include <rocprim/rocprim.hpp>

#include "engine.hpp"
#include "trace.hpp"

namespace tgo {
namespace {

constexpr int kB = 256;
inline unsigned grid(int64_t work) {
    const int64_t g = (work + kB - 1) / kB;
    return static_cast<unsigned>(std::max<int64_t>(1, std::min<int64_t>(g, 65536)));
}

template <class T>
struct Buf {                            // large ones recycled (tmp_cache.cpp)
    T* p = nullptr;
    size_t bytes = 0;
    hipError_t alloc(int64_t count) {
        release();
        bytes = static_cast<size_t>(std::max<int64_t>(count, 1)) * sizeof(T);
        void* q = nullptr;
        const hipError_t e = tmp_alloc(&q, bytes);
        p = static_cast<T*>(q);
        return e;
    }
    void release() { if (p) tmp_free(p, bytes); p = nullptr; }
    T* take() { T* q = p; tmp_disown(q); p = nullptr; return q; }     // hand over (DevArray::own)
    ~Buf() { release(); }
};

#define PL_TRY(x)                                                                  \
    do {                                                                           \
        hipError_t e_ = (x);                                                       \
        if (e_ != hipSuccess) { err = std::string("pr layout: ") + hipGetErrorString(e_); return TGO_E_HIP; } \
    } while (0)

// row of entry k: last r with off[r] <= k (rows may be empty)
__device__ __forceinline__ int64_t row_of(const int64_t* __restrict__ off, int64_t n, int64_t k) {
    int64_t lo = 0, hi = n;
    while (hi - lo > 1) { const int64_t mid = (lo + hi) >> 1; if (off[mid] <= k) lo = mid; else hi = mid; }
    return lo;
}

__global__ void unsorted_rows(const int64_t* __restrict__ off, const int32_t* __restrict__ adj, int64_t n, int64_t nnz,
                              int* bad) {
    for (int64_t k = blockIdx.x * (int64_t)blockDim.x + threadIdx.x + 1; k < nnz; k += (int64_t)gridDim.x * blockDim.x)
        if (adj[k] < adj[k - 1] && off[row_of(off, n, k)] != k) atomicOr(bad, 1);
}
__global__ void hot_counts(const int64_t* __restrict__ off, const int32_t* __restrict__ adj, int64_t n, int32_t hot,
                           int64_t* __restrict__ hcount) {
    for (int64_t r = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; r < n; r += (int64_t)gridDim.x * blockDim.x) {
        int64_t lo = off[r], hi = off[r + 1];
        while (lo < hi) { const int64_t mid = (lo + hi) >> 1; if (adj[mid] < hot) lo = mid + 1; else hi = mid; }
        hcount[r] = lo - off[r];
    }
}
// window prefix (sources < win) -> widx; the rest of the hot prefix -> hadj; cold entry ->
// (segment << 32 | row, source) at its cold position.  wcount == nullptr: no window.
__global__ void split_entries(const int64_t* __restrict__ off, const int32_t* __restrict__ adj, int64_t n, int64_t nnz,
                              const int64_t* __restrict__ hcount, const int64_t* __restrict__ hoff, int32_t hot,
                              int64_t seg, int32_t* __restrict__ hadj, uint64_t* __restrict__ ckey,
                              int32_t* __restrict__ cval, const int64_t* __restrict__ wcount,
                              const int64_t* __restrict__ woff, uint16_t* __restrict__ widx) {
    for (int64_t k = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; k < nnz; k += (int64_t)gridDim.x * blockDim.x) {
        const int64_t r = row_of(off, n, k);
        const int64_t j = k - off[r];
        const int32_t u = adj[k];
        const int64_t wc = wcount ? wcount[r] : 0;
        if (j < wc) {
            widx[woff[r] + j] = static_cast<uint16_t>(u);
        } else if (j < hcount[r]) {
            hadj[hoff[r] + (j - wc)] = u;
        } else {
            // cold entries before this one: the row's earlier entries minus the hot and window ones
            const int64_t c = (off[r] - hoff[r] - (wcount ? woff[r] : 0)) + (j - hcount[r]);
            ckey[c] = (static_cast<uint64_t>((u - hot) / seg) << 32) | static_cast<uint64_t>(r);
            cval[c] = u;
        }
    }
}
__global__ void sub_counts(const int64_t* __restrict__ a, const int64_t* __restrict__ b, int64_t m, int64_t* __restrict__ out) {
    for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < m; i += (int64_t)gridDim.x * blockDim.x)
        out[i] = a[i] - b[i];
}
// run starts (a new (segment, row)) and piece starts (a run start or every tile-th entry of a run)
__global__ void run_marks(const uint64_t* __restrict__ key, int64_t m, int64_t* __restrict__ rs) {
    for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < m; i += (int64_t)gridDim.x * blockDim.x)
        rs[i] = (i == 0 || key[i] != key[i - 1]) ? i : 0;
}
__global__ void piece_marks(const uint64_t* __restrict__ key, const int64_t* __restrict__ runstart, int64_t m, int64_t tile,
                            uint32_t* __restrict__ start) {
    for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < m; i += (int64_t)gridDim.x * blockDim.x)
        start[i] = ((i - runstart[i]) % tile == 0) ? 1u : 0u;
}
__global__ void piece_fill(const uint32_t* __restrict__ start, const uint64_t* __restrict__ pid, const uint64_t* __restrict__ key,
                           int64_t m, int64_t* __restrict__ poff, uint32_t* __restrict__ prow, uint32_t* __restrict__ pseg,
                           uint32_t* __restrict__ pix) {
    for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < m; i += (int64_t)gridDim.x * blockDim.x) {
        if (!start[i]) continue;
        const uint64_t p = pid[i];
        poff[p] = i;
        prow[p] = static_cast<uint32_t>(key[i]);
        pseg[p] = static_cast<uint32_t>(key[i] >> 32);
        pix[p] = static_cast<uint32_t>(p);
    }
}
// cptr[r] = first position of row r among the pieces sorted by row (n+1 entries)
__global__ void row_starts_u32(const uint32_t* __restrict__ prow_sorted, int64_t np, int64_t n, uint32_t* __restrict__ cptr) {
    for (int64_t r = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; r <= n; r += (int64_t)gridDim.x * blockDim.x) {
        int64_t lo = 0, hi = np;
        while (lo < hi) { const int64_t mid = (lo + hi) >> 1; if (prow_sorted[mid] < r) lo = mid + 1; else hi = mid; }
        cptr[r] = static_cast<uint32_t>(lo);
    }
}
// tile packing: entry k of the tile starting at tstart[t] (tiles cover their entries in order)
__global__ void pack_keys(const int32_t* __restrict__ adj, int64_t m, const int64_t* __restrict__ tstart, int64_t ntiles,
                          const int32_t* __restrict__ tbase, int shift, uint64_t* __restrict__ key) {
    for (int64_t k = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; k < m; k += (int64_t)gridDim.x * blockDim.x) {
        int64_t lo = 0, hi = ntiles;                 // last tile with tstart <= k
        while (hi - lo > 1) { const int64_t mid = (lo + hi) >> 1; if (tstart[mid] <= k) lo = mid; else hi = mid; }
        const uint32_t packed = (static_cast<uint32_t>(adj[k] - (tbase ? tbase[lo] : 0)) << shift) |
                                static_cast<uint32_t>(k - tstart[lo]);
        key[k] = (static_cast<uint64_t>(lo) << 32) | packed;
    }
}
// super-tile packing (gather_hot_fx / cold_fx): entry k of tile t (desc: first entry, end, first
// row, rows or a long row's -(index + 1); rows = pieces and off = piece offsets for cold tiles)
// -> t << 32 | (source - tbase[t]) << rbits | row - first row
__global__ void pack_rowlocal_keys(const int32_t* __restrict__ adj, int64_t m, const int64_t* __restrict__ td,
                                   int64_t ntiles, const int64_t* __restrict__ off, int rbits, uint64_t* __restrict__ key,
                                   const int32_t* __restrict__ tbase = nullptr) {
    for (int64_t k = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; k < m; k += (int64_t)gridDim.x * blockDim.x) {
        int64_t lo = 0, hi = ntiles;                 // last tile whose first entry is <= k (empty tiles skipped by ties)
        while (hi - lo > 1) { const int64_t mid = (lo + hi) >> 1; if (td[4 * mid] <= k) lo = mid; else hi = mid; }
        const int64_t r0 = td[4 * lo + 2], nr = td[4 * lo + 3];
        int64_t rl = 0;
        if (nr > 1) {                                // the row of entry k: last r in [r0, r0 + nr) with off[r] <= k
            int64_t a = r0, b = r0 + nr;
            while (b - a > 1) { const int64_t mid = (a + b) >> 1; if (off[mid] <= k) a = mid; else b = mid; }
            rl = a - r0;
        }
        const uint32_t src = static_cast<uint32_t>(adj[k] - (tbase ? tbase[lo] : 0));
        key[k] = (static_cast<uint64_t>(lo) << 32) | (static_cast<uint64_t>(src << rbits) | static_cast<uint64_t>(rl));
    }
}
__global__ void unpack_keys(const uint64_t* __restrict__ key, int64_t m, int32_t* __restrict__ adj) {
    for (int64_t k = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; k < m; k += (int64_t)gridDim.x * blockDim.x)
        adj[k] = static_cast<int32_t>(static_cast<uint32_t>(key[k]));
}

struct Sort {
    Buf<uint8_t> tmp;
    size_t have = 0;
    hipStream_t s;
    hipError_t grow(size_t need) {
        if (need <= have) return hipSuccess;
        have = need;
        return tmp.alloc(static_cast<int64_t>(need));
    }
    template <class V>
    hipError_t pairs(const uint64_t* ki, uint64_t* ko, const V* vi, V* vo, int64_t m, int bits) {
        size_t need = 0;
        hipError_t e = rocprim::radix_sort_pairs(nullptr, need, ki, ko, vi, vo, static_cast<size_t>(m), 0, bits, s);
        if (e != hipSuccess || (e = grow(need)) != hipSuccess) return e;
        return rocprim::radix_sort_pairs(tmp.p, need, ki, ko, vi, vo, static_cast<size_t>(m), 0, bits, s);
    }
    hipError_t pairs32(const uint32_t* ki, uint32_t* ko, const uint32_t* vi, uint32_t* vo, int64_t m) {
        size_t need = 0;
        hipError_t e = rocprim::radix_sort_pairs(nullptr, need, ki, ko, vi, vo, static_cast<size_t>(m), 0, 32, s);
        if (e != hipSuccess || (e = grow(need)) != hipSuccess) return e;
        return rocprim::radix_sort_pairs(tmp.p, need, ki, ko, vi, vo, static_cast<size_t>(m), 0, 32, s);
    }
    hipError_t keys(const uint64_t* ki, uint64_t* ko, int64_t m, int bits) {
        size_t need = 0;
        hipError_t e = rocprim::radix_sort_keys(nullptr, need, ki, ko, static_cast<size_t>(m), 0, bits, s);
        if (e != hipSuccess || (e = grow(need)) != hipSuccess) return e;
        return rocprim::radix_sort_keys(tmp.p, need, ki, ko, static_cast<size_t>(m), 0, bits, s);
    }
    template <class In, class Out>
    hipError_t excl(const In* in, Out* out, int64_t m) {
        size_t need = 0;
        hipError_t e = rocprim::exclusive_scan(nullptr, need, in, out, Out(0), static_cast<size_t>(m), rocprim::plus<Out>(), s);
        if (e != hipSuccess || (e = grow(need)) != hipSuccess) return e;
        return rocprim::exclusive_scan(tmp.p, need, in, out, Out(0), static_cast<size_t>(m), rocprim::plus<Out>(), s);
    }
    hipError_t incl_max(const int64_t* in, int64_t* out, int64_t m) {
        size_t need = 0;
        hipError_t e = rocprim::inclusive_scan(nullptr, need, in, out, static_cast<size_t>(m), rocprim::maximum<int64_t>(), s);
        if (e != hipSuccess || (e = grow(need)) != hipSuccess) return e;
        return rocprim::inclusive_scan(tmp.p, need, in, out, static_cast<size_t>(m), rocprim::maximum<int64_t>(), s);
    }
};

// device -> host vector (pinned double-buffered copy, huge-page-advised vector); D may differ
// from T in signedness only (same size)
template <class T, class D>
hipError_t fetch(std::vector<T>& h, const D* d, int64_t count, hipStream_t s) {
    static_assert(sizeof(T) == sizeof(D), "fetch: element sizes differ");
    host_resize(h, static_cast<size_t>(count));
    if (count <= 0) return hipSuccess;
    hipError_t e = hipStreamSynchronize(s);
    if (e != hipSuccess) return e;
    return copy_d2h(h.data(), d, static_cast<size_t>(count) * sizeof(T));
}

int bits_for(int64_t x) {
    int b = 1;
    while ((int64_t(1) << b) <= x) ++b;
    return b;
}

}  // namespace

// Sort every tile's entries by (source - base) and pack them as (source - base) << shift | slot,
// in place on the device: tiles are the ranges [tstart[t], tstart[t+1]) covering [0, m).
int pack_tiles_device(int32_t* d_adj, int64_t m, const std::vector<int64_t>& tstart, const std::vector<int32_t>* tbase,
                      int shift, hipStream_t s, std::string& err) {
    if (m == 0) return TGO_OK;
    const int64_t nt = static_cast<int64_t>(tstart.size());
    Buf<int64_t> ts;
    Buf<int32_t> tb;
    Buf<uint64_t> k0, k1;
    PL_TRY(ts.alloc(nt));
    PL_TRY(copy_chunked(ts.p, tstart.data(), nt * 8, hipMemcpyHostToDevice));
    if (tbase) {
        PL_TRY(tb.alloc(nt));
        PL_TRY(copy_chunked(tb.p, tbase->data(), nt * 4, hipMemcpyHostToDevice));
    }
    PL_TRY(k0.alloc(m));
    PL_TRY(k1.alloc(m));
    pack_keys<<<grid(m), kB, 0, s>>>(d_adj, m, ts.p, nt, tbase ? tb.p : nullptr, shift, k0.p);
    Sort so{{}, 0, s};
    PL_TRY(so.keys(k0.p, k1.p, m, 32 + bits_for(nt)));
    unpack_keys<<<grid(m), kB, 0, s>>>(k1.p, m, d_adj);
    PL_TRY(hipStreamSynchronize(s));
    return TGO_OK;
}

// Super-tiles of the hot CSR (rows [0, n_rows), entries [0, off[n_rows]) on the device, sources
// < 2^(32 - rbits)) for the fixed-point hot pass (gather_hot_fx, spmv.hip): greedy row ranges of
// at most 2^rbits rows and max_e entries; a row with more than max_e entries forms tiles of its
// own (max_e-entry chunks, rows field -(long index + 1), long_rows[index] = the row).  Every
// tile's entries are then sorted by source and packed in place as source << rbits | row - r0.
// tdesc: 4 per tile {first entry, end entry, first row, rows or -(long index + 1)}.
int pack_supertiles_device(int32_t* d_adj, const int64_t* d_off, const std::vector<int64_t>& off, int64_t n_rows,
                           int64_t max_e, int rbits, std::vector<int64_t>& tdesc, std::vector<int32_t>& long_rows,
                           std::vector<int64_t>& long_len, hipStream_t s, std::string& err) {
    tdesc.clear();
    long_rows.clear();
    long_len.clear();
    const int64_t R = int64_t(1) << rbits;
    if (max_e < 1 || static_cast<int64_t>(off.size()) < n_rows + 1) { err = "pr layout: super-tile arguments"; return TGO_E_INVALID; }
    for (int64_t r = 0; r < n_rows;) {
        const int64_t e0 = off[r];
        if (off[r + 1] - e0 > max_e) {               // a long row: chunks of its own
            const int64_t li = static_cast<int64_t>(long_rows.size());
            long_rows.push_back(static_cast<int32_t>(r));
            long_len.push_back(off[r + 1] - e0);
            for (int64_t c = e0; c < off[r + 1]; c += max_e)
                tdesc.insert(tdesc.end(), {c, std::min(c + max_e, off[r + 1]), r, -(li + 1)});
            ++r;
            continue;
        }
        const int64_t rmax = std::min(n_rows, r + R);
        // the last r2 in (r, rmax] with off[r2] - e0 <= max_e
        int64_t r2 = std::upper_bound(off.begin() + r + 1, off.begin() + rmax + 1, e0 + max_e) - off.begin() - 1;
        r2 = std::max(r2, r + 1);
        tdesc.insert(tdesc.end(), {e0, off[r2], r, r2 - r});
        r = r2;
    }
    const int64_t nt = static_cast<int64_t>(tdesc.size() / 4), m = off[n_rows];
    if (m == 0 || nt == 0) return TGO_OK;
    Buf<int64_t> td;
    Buf<uint64_t> k0, k1;
    PL_TRY(td.alloc(4 * nt));
    PL_TRY(copy_chunked(td.p, tdesc.data(), 4 * nt * 8, hipMemcpyHostToDevice));
    PL_TRY(k0.alloc(m));
    PL_TRY(k1.alloc(m));
    pack_rowlocal_keys<<<grid(m), kB, 0, s>>>(d_adj, m, td.p, nt, d_off, rbits, k0.p);
    Sort so{{}, 0, s};
    PL_TRY(so.keys(k0.p, k1.p, m, 32 + bits_for(nt)));
    unpack_keys<<<grid(m), kB, 0, s>>>(k1.p, m, d_adj);
    PL_TRY(hipStreamSynchronize(s));
    return TGO_OK;
}

// The ColdBlocks host structure (graph_build.cpp build_cold_blocks, same arrays) from device
// in-lists.  built = false when the layout does not apply (nothing cold, too many pieces) or
// a row is not sorted by source (then the caller keeps the host build).
int build_cold_blocks_device(const int64_t* d_off, const int32_t* d_adj, int64_t n, int64_t nnz, int64_t n_src,
                             int64_t hot, int64_t seg, int64_t tile, int64_t max_pieces, bool pack, HostColdBlocks& hc,
                             bool& built, hipStream_t s, std::string& err, int64_t win, bool fx) {
    built = false;
    hc = HostColdBlocks();
    if (hot <= 0 || seg <= 0 || n_src <= hot || n <= 0 || hot >= INT32_MAX) return TGO_OK;
    if (win < 0 || win > 65536 || win > hot) win = 0;       // uint16 window entries inside the hot range
    const int64_t nseg = (n_src - hot + seg - 1) / seg;
    Sort so{{}, 0, s};
    static const bool trace = std::getenv("TGO_TRACE") && std::atoi(std::getenv("TGO_TRACE")) != 0;
    auto t_last = std::chrono::steady_clock::now();
    auto lap = [&](const char* what) {
        if (!trace && !tracing()) return;
        (void)hipStreamSynchronize(s);
        const auto now = std::chrono::steady_clock::now();
        const double ms = std::chrono::duration<double, std::milli>(now - t_last).count();
        if (trace) std::fprintf(stderr, "[tgo]     cold build %-18s %8.1f ms\n", what, ms);
        trace_complete(std::string("pagerank_layout.build.") + what, ms * 1e3);
        t_last = now;
    };
    {
        Buf<int> bad;
        PL_TRY(bad.alloc(1));
        PL_TRY(hipMemsetAsync(bad.p, 0, sizeof(int), s));
        if (nnz > 1) unsorted_rows<<<grid(nnz), kB, 0, s>>>(d_off, d_adj, n, nnz, bad.p);
        int hb = 0;
        PL_TRY(hipMemcpyAsync(&hb, bad.p, sizeof(int), hipMemcpyDeviceToHost, s));
        PL_TRY(hipStreamSynchronize(s));
        if (hb) return TGO_OK;
    }
    hc.hot = hot;
    hc.seg = seg;
    // hot prefix per row, its CSR
    Buf<int64_t> hcount, hoff;
    PL_TRY(hcount.alloc(n + 1));
    PL_TRY(hoff.alloc(n + 1));
    hot_counts<<<grid(n), kB, 0, s>>>(d_off, d_adj, n, static_cast<int32_t>(hot), hcount.p);
    PL_TRY(hipMemsetAsync(hcount.p + n, 0, sizeof(int64_t), s));
    PL_TRY(so.excl(hcount.p, hoff.p, n + 1));
    int64_t nhot = 0;
    PL_TRY(hipMemcpyAsync(&nhot, hoff.p + n, 8, hipMemcpyDeviceToHost, s));
    PL_TRY(hipStreamSynchronize(s));
    const int64_t C = nnz - nhot;
    // LDS window: each row's sources < win leave the hot CSR for the window CSR
    Buf<int64_t> wcount, woff;
    Buf<uint16_t> widx;
    int64_t nwin = 0;
    if (win > 0) {
        PL_TRY(wcount.alloc(n + 1));
        PL_TRY(woff.alloc(n + 1));
        hot_counts<<<grid(n), kB, 0, s>>>(d_off, d_adj, n, static_cast<int32_t>(win), wcount.p);
        PL_TRY(hipMemsetAsync(wcount.p + n, 0, sizeof(int64_t), s));
        PL_TRY(so.excl(wcount.p, woff.p, n + 1));
        PL_TRY(hipMemcpyAsync(&nwin, woff.p + n, 8, hipMemcpyDeviceToHost, s));
        PL_TRY(hipStreamSynchronize(s));
        // the hot CSR keeps [wcount, hcount) of every row
        Buf<int64_t> hc2;
        PL_TRY(hc2.alloc(n + 1));
        sub_counts<<<grid(n + 1), kB, 0, s>>>(hcount.p, wcount.p, n + 1, hc2.p);
        PL_TRY(so.excl(hc2.p, hoff.p, n + 1));
        PL_TRY(hipStreamSynchronize(s));
        nhot -= nwin;
        PL_TRY(widx.alloc(nwin));
    }
    Buf<int32_t> hadj, cval, cadj;
    Buf<uint64_t> ckey, skey;
    PL_TRY(hadj.alloc(nhot));
    PL_TRY(cval.alloc(C));
    PL_TRY(cadj.alloc(C));
    PL_TRY(ckey.alloc(C));
    PL_TRY(skey.alloc(C));
    if (nnz) split_entries<<<grid(nnz), kB, 0, s>>>(d_off, d_adj, n, nnz, hcount.p, hoff.p, static_cast<int32_t>(hot), seg,
                                                   hadj.p, ckey.p, cval.p, win > 0 ? wcount.p : nullptr, woff.p, widx.p);
    if (win > 0) {
        PL_TRY(fetch(hc.woff, woff.p, n + 1, s));
        hc.win = win;
        PL_TRY(hipStreamSynchronize(s));
        hc.d_widx.own(widx.take(), nwin);
    }
    lap("split");
    if (C) PL_TRY(so.pairs(ckey.p, skey.p, cval.p, cadj.p, C, 32 + bits_for(nseg)));
    lap("cold sort");
    ckey.release();
    cval.release();
    // pieces
    Buf<int64_t> rs, runstart, poff;
    Buf<uint32_t> start, prow, pseg, pix, prow_s, pix_s, cptr;
    Buf<uint64_t> pid;
    PL_TRY(rs.alloc(C));
    PL_TRY(runstart.alloc(C));
    PL_TRY(start.alloc(C + 1));
    PL_TRY(pid.alloc(C + 1));
    if (C) {
        run_marks<<<grid(C), kB, 0, s>>>(skey.p, C, rs.p);
        PL_TRY(so.incl_max(rs.p, runstart.p, C));
        piece_marks<<<grid(C), kB, 0, s>>>(skey.p, runstart.p, C, tile, start.p);
    }
    PL_TRY(hipMemsetAsync(start.p + C, 0, sizeof(uint32_t), s));
    PL_TRY(so.excl(start.p, pid.p, C + 1));
    uint64_t np64 = 0;
    PL_TRY(hipMemcpyAsync(&np64, pid.p + C, 8, hipMemcpyDeviceToHost, s));
    PL_TRY(hipStreamSynchronize(s));
    const int64_t np = static_cast<int64_t>(np64);
    if (np >= (int64_t(1) << 31)) return TGO_OK;                  // the host rule: 32-bit piece ids
    rs.release();
    runstart.release();
    PL_TRY(poff.alloc(np + 1));
    PL_TRY(prow.alloc(np)); PL_TRY(pseg.alloc(np)); PL_TRY(pix.alloc(np));
    PL_TRY(prow_s.alloc(np)); PL_TRY(pix_s.alloc(np)); PL_TRY(cptr.alloc(n + 1));
    if (C) piece_fill<<<grid(C), kB, 0, s>>>(start.p, pid.p, skey.p, C, poff.p, prow.p, pseg.p, pix.p);
    PL_TRY(hipMemcpyAsync(poff.p + np, &C, 8, hipMemcpyHostToDevice, s));
    if (np) PL_TRY(so.pairs32(prow.p, prow_s.p, pix.p, pix_s.p, np));
    row_starts_u32<<<grid(n + 1), kB, 0, s>>>(prow_s.p, np, n, cptr.p);
    start.release();
    pid.release();
    skey.release();
    lap("pieces");
    // to the host: the piece structure, the hot CSR and the cold entries
    std::vector<uint32_t> h_pseg;
    PL_TRY(fetch(hc.poff, poff.p, np + 1, s));
    PL_TRY(fetch(h_pseg, pseg.p, np, s));
    PL_TRY(fetch(hc.cptr, cptr.p, n + 1, s));
    PL_TRY(fetch(hc.cpid, pix_s.p, np, s));             // piece ids < 2^31 (checked above)
    PL_TRY(fetch(hc.hoff, hoff.p, n + 1, s));
    hc.crow.clear();
    for (int64_t r = 0; r < n; ++r)
        if (hc.cptr[r + 1] > hc.cptr[r]) hc.crow.push_back(static_cast<int32_t>(r));
    lap("fetch");
    // blocks: greedy per segment (<= tile entries, <= max_pieces pieces), segment-major
    std::vector<int64_t> seg_pbase(nseg + 1, np);
    for (int64_t p = np - 1; p >= 0; --p) seg_pbase[h_pseg[p]] = p;
    for (int64_t sg = nseg - 1; sg >= 0; --sg) seg_pbase[sg] = std::min(seg_pbase[sg], seg_pbase[sg + 1]);
    for (int64_t sg = 0; sg < nseg; ++sg) {
        int64_t p = seg_pbase[sg];
        while (p < seg_pbase[sg + 1]) {
            int64_t e = p;
            while (e < seg_pbase[sg + 1] && e - p < max_pieces && hc.poff[e + 1] - hc.poff[p] <= tile) ++e;
            hc.bbeg.push_back(p);
            hc.bend.push_back(e);
            hc.bsrc.push_back(static_cast<int32_t>(hot + sg * seg));
            p = e;
        }
    }
    const int64_t nb = static_cast<int64_t>(hc.bbeg.size());
    lap("blocks (host)");
    const int cshift = max_pieces > (int64_t(1) << kPackShift) ? kPackShift + 1 : kPackShift;
    if (fx && pack && max_pieces <= (int64_t(1) << cshift) && seg <= (int64_t(1) << (32 - cshift))) {
        // fixed-point cold tiles (cold_fx): (source - segment base) << cshift | piece - first piece
        std::vector<int64_t> td(4 * nb);
        for (int64_t b = 0; b < nb; ++b) {
            td[4 * b] = hc.poff[hc.bbeg[b]];
            td[4 * b + 1] = hc.poff[hc.bend[b]];
            td[4 * b + 2] = hc.bbeg[b];
            td[4 * b + 3] = hc.bend[b] - hc.bbeg[b];
        }
        if (nb > 0 && C > 0) {
            Buf<int64_t> dtd;
            Buf<int32_t> dtb;
            Buf<uint64_t> k0, k1;
            PL_TRY(dtd.alloc(4 * nb));
            PL_TRY(copy_chunked(dtd.p, td.data(), 4 * nb * 8, hipMemcpyHostToDevice));
            PL_TRY(dtb.alloc(nb));
            PL_TRY(copy_chunked(dtb.p, hc.bsrc.data(), nb * 4, hipMemcpyHostToDevice));
            PL_TRY(k0.alloc(C));
            PL_TRY(k1.alloc(C));
            pack_rowlocal_keys<<<grid(C), kB, 0, s>>>(cadj.p, C, dtd.p, nb, poff.p, cshift, k0.p, dtb.p);
            PL_TRY(so.keys(k0.p, k1.p, C, 32 + bits_for(nb)));
            unpack_keys<<<grid(C), kB, 0, s>>>(k1.p, C, cadj.p);
        }
        hc.cpacked = true;
        hc.cfx = true;
        hc.cfx_shift = cshift;
    } else if (pack && seg <= (int64_t(1) << (31 - kPackShift)) && tile <= (int64_t(1) << kPackShift)) {
        std::vector<int64_t> tstart(nb);
        for (int64_t b = 0; b < nb; ++b) tstart[b] = hc.poff[hc.bbeg[b]];
        if (nb > 0)
            if (int rc = pack_tiles_device(cadj.p, C, tstart, &hc.bsrc, kPackShift, s, err)) return rc;
        hc.cpacked = true;
    }
    PL_TRY(hipStreamSynchronize(s));
    hc.d_cadj.own(cadj.take(), C);                   // both stay on the device (upload_cold_blocks)
    hc.d_hadj.own(hadj.take(), nhot);
    hc.xblk.resize(nb);
    for (int64_t b = 0; b < nb; ++b) hc.xblk[b] = static_cast<int32_t>(b);
    const int64_t total = hc.poff[np];
    hc.max_xcd_blocks = 0;
    int64_t b = 0;
    for (int x = 0; x < 8; ++x) {
        hc.xbase.b[x] = b;
        const int64_t target = total * (x + 1) / 8;
        while (b < nb && (x == 7 || hc.poff[hc.bend[b]] <= target)) ++b;
        hc.max_xcd_blocks = std::max<int64_t>(hc.max_xcd_blocks, b - hc.xbase.b[x]);
    }
    hc.xbase.b[8] = nb;
    built = true;
    return TGO_OK;
}

// Partitioned PageRank (tgo_part_pr_blocked): every in-list source u (global slot id, rank
// r = u / nl, offset o = u % nl) to its position in the blocked gathered vector — rank-major
// hot slices [0, H) first, then the cold slices [H, A); a source past A sets *bad.
__global__ void part_gathered_index(const int32_t* __restrict__ in, int64_t m, int64_t nl, int64_t A, int64_t H,
                                    int64_t W, int32_t* __restrict__ out, int* __restrict__ bad) {
    for (int64_t k = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; k < m; k += (int64_t)gridDim.x * blockDim.x) {
        const int64_t u = in[k], r = u / nl, o = u % nl;
        if (o >= A) { *bad = 1; out[k] = 0; continue; }
        out[k] = static_cast<int32_t>(o < H ? r * H + o : W * H + r * (A - H) + (o - H));
    }
}
hipError_t k_part_gathered_index(const int32_t* in, int64_t m, int64_t nl, int64_t A, int64_t H, int64_t W, int32_t* out,
                                 int* bad, hipStream_t s) {
    if (m > 0) {
        const unsigned g = static_cast<unsigned>(std::min<int64_t>((m + 255) / 256, 65536));
        part_gathered_index<<<g, 256, 0, s>>>(in, m, nl, A, H, W, out, bad);
    }
    return hipGetLastError();
}

namespace {
__global__ void row_value_keys(const int64_t* __restrict__ off, int64_t n, const int32_t* __restrict__ v, int64_t m,
                               uint64_t* __restrict__ key) {
    for (int64_t k = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; k < m; k += (int64_t)gridDim.x * blockDim.x)
        key[k] = (static_cast<uint64_t>(row_of(off, n, k)) << 32) | static_cast<uint32_t>(v[k]);
}
__global__ void low_words(const uint64_t* __restrict__ key, int64_t m, int32_t* __restrict__ v) {
    for (int64_t k = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; k < m; k += (int64_t)gridDim.x * blockDim.x)
        v[k] = static_cast<int32_t>(static_cast<uint32_t>(key[k]));
}
}  // namespace

// The cold layout of a split multi-source pull (msbfs.hip ms_cold): every pull-list entry whose
// neighbour is >= hot, from both lists of the view, sorted by (segment of the neighbour, row) —
// crow / cadj per entry.  C = 0 when nothing is cold.
int build_ms_cold(const View& v, int64_t n, int32_t hot, int64_t seg, DevArray<int32_t>& cadj, DevArray<int32_t>& crow,
                  int64_t& C, hipStream_t s, std::string& err) {
    C = 0;
    if (n <= hot || seg <= 0) return TGO_OK;
    const int64_t* off[2] = {v.off0, v.off1};
    const int32_t* adj[2] = {v.adj0, v.adj1};
    int64_t m[2] = {0, 0}, cnt[2] = {0, 0};
    Sort so{{}, 0, s};
    Buf<uint32_t> flag[2];
    Buf<uint64_t> pos[2];
    for (int l = 0; l < v.nlists; ++l) {
        PL_TRY(hipMemcpyAsync(&m[l], off[l] + n, sizeof(int64_t), hipMemcpyDeviceToHost, s));
        PL_TRY(hipStreamSynchronize(s));
        PL_TRY(flag[l].alloc(m[l] + 1));
        PL_TRY(pos[l].alloc(m[l] + 1));
        PL_TRY(k_cold_flags(adj[l], m[l], hot, flag[l].p, s));
        PL_TRY(hipMemsetAsync(flag[l].p + m[l], 0, sizeof(uint32_t), s));
        PL_TRY(so.excl(flag[l].p, pos[l].p, m[l] + 1));
        PL_TRY(hipMemcpyAsync(&cnt[l], pos[l].p + m[l], sizeof(int64_t), hipMemcpyDeviceToHost, s));
        PL_TRY(hipStreamSynchronize(s));
    }
    const int64_t total = cnt[0] + cnt[1];
    if (total == 0) return TGO_OK;
    Buf<uint64_t> k0, k1;
    Buf<int32_t> v0, v1, rows;
    PL_TRY(k0.alloc(total));
    PL_TRY(k1.alloc(total));
    PL_TRY(v0.alloc(total));
    PL_TRY(v1.alloc(total));
    for (int l = 0; l < v.nlists; ++l)
        PL_TRY(k_cold_emit(off[l], n, adj[l], m[l], flag[l].p, pos[l].p, l == 0 ? 0 : cnt[0], hot, seg, k0.p, v0.p, s));
    const int64_t nseg = (n - hot + seg - 1) / seg;
    PL_TRY(so.pairs(k0.p, k1.p, v0.p, v1.p, total, 32 + bits_for(nseg)));
    PL_TRY(rows.alloc(total));
    PL_TRY(k_low_rows(k1.p, total, rows.p, s));
    PL_TRY(hipStreamSynchronize(s));
    cadj.own(v1.take(), total);
    crow.own(rows.take(), total);
    C = total;
    return TGO_OK;
}

// Sort every row's (non-negative) values ascending in place: one radix sort of (row, value)
// keys.  The partitioned PageRank maps its sources into the blocked gathered vector, which is
// not monotone in the global id, so the rows are re-sorted before the device cold build.
int sort_rows_device(const int64_t* d_off, int64_t n, int32_t* d_vals, int64_t m, hipStream_t s, std::string& err) {
    if (m <= 1) return TGO_OK;
    Buf<uint64_t> k0, k1;
    PL_TRY(k0.alloc(m));
    PL_TRY(k1.alloc(m));
    row_value_keys<<<grid(m), kB, 0, s>>>(d_off, n, d_vals, m, k0.p);
    Sort so{{}, 0, s};
    PL_TRY(so.keys(k0.p, k1.p, m, 32 + bits_for(n)));
    low_words<<<grid(m), kB, 0, s>>>(k1.p, m, d_vals);
    PL_TRY(hipStreamSynchronize(s));
    return TGO_OK;
}

}  // namespace tgo

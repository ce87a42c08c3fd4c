// assemble.hip — CSR assembly of an edge-list load on the device (tgo_load_edges).
//
// The same graph as the host path (graph_build.cpp assemble_from_edges), array for array:
// every directed edge u->v is an OUT entry of row u and an IN entry of row v
// (StandardTitanGraph.java:564-591); a row's entries are in column order (direction, other
// Titan id, relation id — IDHandler / EdgeSerializer.java:255-259), which for dense ids in
// row order is (neighbour, edge index); the untyped single-direction scopes cut each row at
// the QueryContainer limit in that order (QueryContainer.java:28,122 and
// BasicVertexCentricQueryBuilder.java:418-431); then the degree-grouped relabel (DBG) and,
// when the cut made the lists asymmetric, the explicit push transpose.  Each of those steps
// is one stable LSD radix sort over 64-bit (row << b | neighbour) keys, which keeps the edge
// order among equal keys — exactly the host path's (neighbour, edge index) tie order:
//   [cap or column order]  sort 1 by (row, neighbour) from edge order; row offsets by
//                          binary search; keep flags + scan = the cut; column positions
//   relabel                degrees -> half-octave buckets -> order (sort of n keys)
//   final lists            sort 2 by (perm[row], perm[neighbour]) from the sort-1 order
//                          (or edge order): = the host's stable per-row re-sort by the new ids
//   transpose              sort by (target, source) from row order
// Weights / column positions ride along as a 32-bit payload (an index into the previous
// order) and are gathered once at the end.
#include <algorithm>
#include <chrono>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>

#include <thread>

#include <hip/hip_runtime.h>
#include <rocprim/rocprim.hpp>

#include "engine.hpp"
#include "trace.hpp"

namespace tgo {
namespace {

constexpr int kB = 256;

inline unsigned grid(int64_t work) {
    int64_t g = (work + kB - 1) / kB;
    return static_cast<unsigned>(std::max<int64_t>(1, std::min<int64_t>(g, 65536)));
}

template <class T>
struct ScopedBuf {                      // scoped device buffer (large ones recycled: tmp_cache.cpp)
    T* p = nullptr;
    size_t n = 0;
    hipError_t alloc(size_t count) {
        release();
        n = count;
        void* q = nullptr;
        const hipError_t e = tmp_alloc(&q, std::max<size_t>(count, 1) * sizeof(T));
        p = static_cast<T*>(q);
        return e;
    }
    void release() {
        if (p) tmp_free(p, std::max<size_t>(n, 1) * sizeof(T));
        p = nullptr;
        n = 0;
    }
    T* take() {                         // hand the allocation over (DevArray::own)
        T* q = p;
        tmp_disown(q);
        p = nullptr;
        n = 0;
        return q;
    }
    ~ScopedBuf() { release(); }
};

#define AS_TRY(x)                                            \
    do {                                                     \
        hipError_t e_ = (x);                                 \
        if (e_ != hipSuccess) {                              \
            err = std::string("device assembly: ") + hipGetErrorString(e_); \
            return TGO_E_HIP;                                \
        }                                                    \
    } while (0)

__global__ void range_check(const int32_t* __restrict__ src, const int32_t* __restrict__ dst, int64_t m, int64_t n,
                            int* bad) {
    for (int64_t k = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; k < m; k += (int64_t)gridDim.x * blockDim.x)
        if (src[k] < 0 || src[k] >= n || dst[k] < 0 || dst[k] >= n) atomicOr(bad, 1);
}

// key = own << b | nbr (or through perm), val = edge index
__global__ void edge_keys(const int32_t* __restrict__ own, const int32_t* __restrict__ nbr, int64_t m, int b,
                          const int32_t* __restrict__ perm, uint64_t* __restrict__ key, uint32_t* __restrict__ val) {
    for (int64_t k = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; k < m; k += (int64_t)gridDim.x * blockDim.x) {
        uint64_t o = static_cast<uint32_t>(own[k]), x = static_cast<uint32_t>(nbr[k]);
        if (perm) { o = static_cast<uint32_t>(perm[o]); x = static_cast<uint32_t>(perm[x]); }
        key[k] = (o << b) | x;
        if (val) val[k] = static_cast<uint32_t>(k);
    }
}

// off[v] = first position of row v in keys sorted by row (binary search), v in [0, n]
__global__ void row_offsets(const uint64_t* __restrict__ key, int64_t m, int b, int64_t n, int64_t* __restrict__ off) {
    for (int64_t v = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; v <= n; v += (int64_t)gridDim.x * blockDim.x) {
        int64_t lo = 0, hi = m;
        const uint64_t t = static_cast<uint64_t>(v) << b;
        while (lo < hi) {
            const int64_t mid = (lo + hi) >> 1;
            if (key[mid] < t) lo = mid + 1; else hi = mid;
        }
        off[v] = lo;
    }
}

// Degrees of an uncut load: one atomic per entry end (hub contention is bounded by degree).
__global__ void degree_count(const int32_t* __restrict__ src, const int32_t* __restrict__ dst, int64_t m,
                             uint32_t* __restrict__ deg) {
    for (int64_t k = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; k < m; k += (int64_t)gridDim.x * blockDim.x) {
        atomicAdd(&deg[src[k]], 1u);
        atomicAdd(&deg[dst[k]], 1u);
    }
}

// Per row: kept OUT / IN counts under the limit (the first `limit` entries of [OUT... | IN...]),
// truncated rows counted (a + b >= limit: the slice came back full, VertexJobConverter.java:125).
__global__ void cap_rows(const int64_t* __restrict__ oo, const int64_t* __restrict__ oi, int64_t n, int64_t limit,
                         int64_t* __restrict__ ko, int64_t* __restrict__ ki, uint32_t* __restrict__ deg,
                         unsigned long long* __restrict__ truncated) {
    unsigned long long t = 0;
    for (int64_t v = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; v < n; v += (int64_t)gridDim.x * blockDim.x) {
        const int64_t a = oo[v + 1] - oo[v], b = oi[v + 1] - oi[v];
        if (a + b >= limit) ++t;
        const int64_t ka = min(a, limit);
        const int64_t kb = min(b, limit - ka);
        ko[v] = ka;
        ki[v] = kb;
        deg[v] = static_cast<uint32_t>(ka + kb);
    }
    if (t) atomicAdd(truncated, t);
}

// Keep flag of every sorted entry (position j < kept count of its row) and its column
// position in the Titan row (OUT entries first: col = j; IN entries: col = kept OUT + j).
__global__ void keep_flags(const uint64_t* __restrict__ key, int64_t m, int b, const int64_t* __restrict__ off,
                           const int64_t* __restrict__ kept, const int64_t* __restrict__ col_base,
                           uint32_t* __restrict__ flag, uint32_t* __restrict__ col) {
    for (int64_t k = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; k < m; k += (int64_t)gridDim.x * blockDim.x) {
        const int64_t v = static_cast<int64_t>(key[k] >> b);
        const int64_t j = k - off[v];
        flag[k] = j < kept[v] ? 1u : 0u;
        if (col) col[k] = static_cast<uint32_t>((col_base ? col_base[v] : 0) + j);
    }
}

// Compact the kept entries: key through perm, payload = kept index's sort-1 position.
__global__ void compact_kept(const uint64_t* __restrict__ key, const uint32_t* __restrict__ flag,
                             const uint64_t* __restrict__ pos, int64_t m, int b, const int32_t* __restrict__ perm,
                             uint64_t* __restrict__ okey, uint32_t* __restrict__ oval) {
    const uint64_t mask = (uint64_t(1) << b) - 1;
    for (int64_t k = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; k < m; k += (int64_t)gridDim.x * blockDim.x) {
        if (!flag[k]) continue;
        const uint64_t p = pos[k];
        uint64_t o = key[k] >> b, x = key[k] & mask;
        if (perm) { o = static_cast<uint32_t>(perm[o]); x = static_cast<uint32_t>(perm[x]); }
        okey[p] = (o << b) | x;
        oval[p] = static_cast<uint32_t>(k);
    }
}

// Re-key through perm (sort 2 input), payload = the entry's index.
__global__ void rekey(const uint64_t* __restrict__ key, int64_t m, int b, const int32_t* __restrict__ perm,
                      uint64_t* __restrict__ okey, uint32_t* __restrict__ oval) {
    const uint64_t mask = (uint64_t(1) << b) - 1;
    for (int64_t k = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; k < m; k += (int64_t)gridDim.x * blockDim.x) {
        const uint64_t o = static_cast<uint32_t>(perm[key[k] >> b]), x = static_cast<uint32_t>(perm[key[k] & mask]);
        okey[k] = (o << b) | x;
        if (oval) oval[k] = static_cast<uint32_t>(k);
    }
}

// Half-octave bucket of a degree (graph_build.cpp degree_group_order: 1 + floor(2 log2 d),
// 0 for d = 0) in integer arithmetic: floor(log2(d^2)).  Sort key: hottest bucket first,
// row order inside a bucket.
__global__ void bucket_keys(const uint32_t* __restrict__ deg, int64_t n, uint64_t* __restrict__ key) {
    for (int64_t v = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; v < n; v += (int64_t)gridDim.x * blockDim.x) {
        const uint64_t d = deg[v];
        const int bk = d == 0 ? 0 : 1 + (63 - __clzll(static_cast<long long>(d * d)));
        key[v] = (static_cast<uint64_t>(127 - bk) << 32) | static_cast<uint64_t>(v);
    }
}
__global__ void order_to_perm(const uint64_t* __restrict__ sorted, int64_t n, int32_t* __restrict__ perm) {
    for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x)
        perm[static_cast<uint32_t>(sorted[i])] = static_cast<int32_t>(i);
}

// Final list: neighbour ids, weights / column positions gathered through the payload chain.
__global__ void emit_list(const uint64_t* __restrict__ key, const uint32_t* __restrict__ val, int64_t m, int b,
                          const uint32_t* __restrict__ edge_of, const int32_t* __restrict__ weight,
                          const uint32_t* __restrict__ col_in, int32_t* __restrict__ adj, int32_t* __restrict__ w,
                          uint32_t* __restrict__ col) {
    const uint64_t mask = (uint64_t(1) << b) - 1;
    for (int64_t k = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; k < m; k += (int64_t)gridDim.x * blockDim.x) {
        adj[k] = static_cast<int32_t>(key[k] & mask);
        if (val) {
            const uint32_t p = val[k];
            if (w) w[k] = weight[edge_of ? edge_of[p] : p];
            if (col) col[k] = col_in[p];
        }
    }
}

// Transpose keys: entry k of row v (key = v << b | t) -> t << b | v, payload k.
__global__ void transpose_keys(const uint64_t* __restrict__ key, int64_t m, int b, uint64_t* __restrict__ tkey,
                               uint32_t* __restrict__ tval) {
    const uint64_t mask = (uint64_t(1) << b) - 1;
    for (int64_t k = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; k < m; k += (int64_t)gridDim.x * blockDim.x) {
        tkey[k] = ((key[k] & mask) << b) | (key[k] >> b);
        if (tval) tval[k] = static_cast<uint32_t>(k);
    }
}
__global__ void shift_u32(uint32_t* __restrict__ v, int64_t m, uint32_t by) {
    for (int64_t k = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; k < m; k += (int64_t)gridDim.x * blockDim.x) v[k] += by;
}
__global__ void gather_i32(const uint32_t* __restrict__ idx, const int32_t* __restrict__ in, int64_t m,
                           int32_t* __restrict__ out) {
    for (int64_t k = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; k < m; k += (int64_t)gridDim.x * blockDim.x)
        out[k] = in[idx[k]];
}


// ---- rows (tgo_load_rows after the decode): Titan ids -> dense ids by binary search over the
// sorted vertex ids; the staged entries are already grouped by row in column order
__global__ void id_keys(const int64_t* __restrict__ vid, int64_t n, uint64_t* __restrict__ key, uint32_t* __restrict__ val) {
    for (int64_t v = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; v < n; v += (int64_t)gridDim.x * blockDim.x) {
        key[v] = static_cast<uint64_t>(vid[v]) ^ 0x8000000000000000ULL;     // signed order
        val[v] = static_cast<uint32_t>(v);
    }
}
// Per staged entry: its row (binary search over row_begin), its neighbour's dense id (-1: the
// neighbour never executes -> dropped, VertexState.java:103-137) and the direction flags.
__global__ void entry_dense(const int64_t* __restrict__ other, const uint8_t* __restrict__ dir, int64_t E,
                            const int64_t* __restrict__ row_begin, int64_t n, const uint64_t* __restrict__ skey,
                            const uint32_t* __restrict__ sval, int32_t* __restrict__ row, int32_t* __restrict__ dense,
                            uint32_t* __restrict__ fout, uint32_t* __restrict__ fin) {
    for (int64_t k = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; k < E; k += (int64_t)gridDim.x * blockDim.x) {
        int64_t lo = 0, hi = n;                          // last row with row_begin <= k
        while (hi - lo > 1) { const int64_t mid = (lo + hi) >> 1; if (row_begin[mid] <= k) lo = mid; else hi = mid; }
        const uint64_t t = static_cast<uint64_t>(other[k]) ^ 0x8000000000000000ULL;
        int64_t a = 0, b = n;
        while (a < b) { const int64_t mid = (a + b) >> 1; if (skey[mid] < t) a = mid + 1; else b = mid; }
        const int32_t d = (a < n && skey[a] == t) ? static_cast<int32_t>(sval[a]) : -1;
        row[k] = static_cast<int32_t>(lo);
        dense[k] = d;
        fout[k] = (d >= 0 && dir[k] == 0) ? 1u : 0u;
        fin[k] = (d >= 0 && dir[k] != 0) ? 1u : 0u;
    }
}
// Compact one direction's entries (staged order) into keys row << b | dense, payload = the
// staged entry index (weights, column positions gathered at the end).
__global__ void compact_dir(const uint32_t* __restrict__ flag, const uint64_t* __restrict__ pos, int64_t E, int b,
                            const int32_t* __restrict__ row, const int32_t* __restrict__ dense,
                            uint64_t* __restrict__ okey, uint32_t* __restrict__ oval) {
    for (int64_t k = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; k < E; k += (int64_t)gridDim.x * blockDim.x) {
        if (!flag[k]) continue;
        const uint64_t p = pos[k];
        okey[p] = (static_cast<uint64_t>(static_cast<uint32_t>(row[k])) << b) | static_cast<uint32_t>(dense[k]);
        oval[p] = static_cast<uint32_t>(k);
    }
}
__global__ void col_of(const int32_t* __restrict__ row, const int64_t* __restrict__ row_begin, int64_t E,
                       uint32_t* __restrict__ col) {
    for (int64_t k = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; k < E; k += (int64_t)gridDim.x * blockDim.x)
        col[k] = static_cast<uint32_t>(k - row_begin[row[k]]);
}
__global__ void degree_rows(const int64_t* __restrict__ oo, const int64_t* __restrict__ oi, int64_t n,
                            uint32_t* __restrict__ deg) {
    for (int64_t v = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; v < n; v += (int64_t)gridDim.x * blockDim.x)
        deg[v] = static_cast<uint32_t>((oo[v + 1] - oo[v]) + (oi[v + 1] - oi[v]));
}
// Views check (graph_build.cpp finish_views): every OUT entry u->v has an IN entry at v.
__global__ void count_targets(const int32_t* __restrict__ adj, int64_t m, uint32_t* __restrict__ cnt) {
    for (int64_t k = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; k < m; k += (int64_t)gridDim.x * blockDim.x)
        atomicAdd(&cnt[adj[k]], 1u);
}
__global__ void count_mismatch(const uint32_t* __restrict__ cnt, const int64_t* __restrict__ off, int64_t n, int* bad) {
    for (int64_t v = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; v < n; v += (int64_t)gridDim.x * blockDim.x)
        if (static_cast<int64_t>(cnt[v]) != off[v + 1] - off[v]) atomicOr(bad, 1);
}

// ---- partitions (tgo_load_partition): the rows of the owned range [lo, lo + n) only
// Entries of direction d whose row (own) is owned: flag for the compaction scan.
__global__ void owned_flags(const int32_t* __restrict__ own, int64_t m, int64_t lo, int64_t hi, uint32_t* __restrict__ flag) {
    for (int64_t k = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; k < m; k += (int64_t)gridDim.x * blockDim.x)
        flag[k] = (own[k] >= lo && own[k] < hi) ? 1u : 0u;
}
// Owned entries compacted in edge order: key = (own - lo) << b | nbr (global id), payload = edge index.
__global__ void owned_keys(const int32_t* __restrict__ own, const int32_t* __restrict__ nbr, const uint32_t* __restrict__ flag,
                           const uint64_t* __restrict__ pos, int64_t m, int64_t lo, int b, uint64_t* __restrict__ key,
                           uint32_t* __restrict__ val) {
    for (int64_t k = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; k < m; k += (int64_t)gridDim.x * blockDim.x) {
        if (!flag[k]) continue;
        const uint64_t p = pos[k];
        key[p] = (static_cast<uint64_t>(own[k] - lo) << b) | static_cast<uint32_t>(nbr[k]);
        val[p] = static_cast<uint32_t>(k);
    }
}
// Re-key through the global layout: row -> layout[lo + row] - lo, neighbour -> layout[nbr].
__global__ void part_rekey(const uint64_t* __restrict__ key, int64_t m, int b, const int32_t* __restrict__ layout,
                           int64_t lo, uint64_t* __restrict__ okey, uint32_t* __restrict__ oval) {
    const uint64_t mask = (uint64_t(1) << b) - 1;
    for (int64_t k = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; k < m; k += (int64_t)gridDim.x * blockDim.x) {
        const int64_t r = static_cast<int64_t>(key[k] >> b);
        const uint64_t o = static_cast<uint64_t>(layout[lo + r] - lo), x = static_cast<uint32_t>(layout[key[k] & mask]);
        okey[k] = (o << b) | x;
        if (oval) oval[k] = static_cast<uint32_t>(k);
    }
}

// Global degrees of a partition load's edge list (every row, owned or not).
__global__ void degree_both(const int32_t* __restrict__ src, const int32_t* __restrict__ dst, int64_t m,
                            uint32_t* __restrict__ dout, uint32_t* __restrict__ din) {
    for (int64_t k = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; k < m; k += (int64_t)gridDim.x * blockDim.x) {
        atomicAdd(&dout[src[k]], 1u);
        atomicAdd(&din[dst[k]], 1u);
    }
}
// Kept entries of every global pull row under the cut (OUT entries first, QueryContainer
// limit): pull = OUT (inE scope) keeps min(out, limit); pull = IN (outE) keeps
// min(in, limit - min(out, limit)).  drops[0] = 1 when some row loses entries.
__global__ void pull_kept(const uint32_t* __restrict__ dout, const uint32_t* __restrict__ din, int64_t n, int64_t limit,
                          int pull_out, uint32_t* __restrict__ kept, int* __restrict__ drops) {
    for (int64_t v = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; v < n; v += (int64_t)gridDim.x * blockDim.x) {
        const int64_t a = dout[v], b = din[v];
        if (a + b > limit) *drops = 1;
        const int64_t ka = a < limit ? a : limit;
        const int64_t kb = b < limit - ka ? b : limit - ka;
        kept[v] = static_cast<uint32_t>(pull_out ? ka : kb);
    }
}
// Edges of the pull rows that lose entries (kept < row length): flag for the compaction.
__global__ void cut_row_flags(const int32_t* __restrict__ prow, int64_t m, const uint32_t* __restrict__ kept,
                              const uint32_t* __restrict__ dlen, uint32_t* __restrict__ flag) {
    for (int64_t k = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; k < m; k += (int64_t)gridDim.x * blockDim.x) {
        const int32_t v = prow[k];
        flag[k] = kept[v] < dlen[v] ? 1u : 0u;
    }
}
// Sorted (pull row, neighbour) entries of the cut rows: entry j of row v is dropped when
// j >= kept[v]; mark its edge.
__global__ void mark_dropped(const uint64_t* __restrict__ key, const uint32_t* __restrict__ eidx, int64_t c, int b,
                             const uint32_t* __restrict__ kept, uint8_t* __restrict__ dropped) {
    for (int64_t k = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; k < c; k += (int64_t)gridDim.x * blockDim.x) {
        const uint64_t v = key[k] >> b;
        // first entry of the row: binary search for the first key >= v << b
        int64_t lo = 0, hi = k;
        const uint64_t t = v << b;
        while (lo < hi) {
            const int64_t mid = (lo + hi) >> 1;
            if (key[mid] < t) lo = mid + 1; else hi = mid;
        }
        if (k - lo >= static_cast<int64_t>(kept[v])) dropped[eidx[k]] = 1;
    }
}
// Push entries of the owned push rows (the pull neighbour in [lo, hi)), kept edges only.
__global__ void push_flags(const int32_t* __restrict__ pn, int64_t m, int64_t lo, int64_t hi,
                           const uint8_t* __restrict__ dropped, uint32_t* __restrict__ flag) {
    for (int64_t k = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; k < m; k += (int64_t)gridDim.x * blockDim.x)
        flag[k] = (pn[k] >= lo && pn[k] < hi && !dropped[k]) ? 1u : 0u;
}
// key = (push row, through the layout) << b | (pull row, through the layout), payload = edge.
__global__ void push_keys(const int32_t* __restrict__ pn, const int32_t* __restrict__ pr, const uint32_t* __restrict__ flag,
                          const uint64_t* __restrict__ pos, int64_t m, int64_t lo, int b, const int32_t* __restrict__ layout,
                          uint64_t* __restrict__ key, uint32_t* __restrict__ val) {
    for (int64_t k = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; k < m; k += (int64_t)gridDim.x * blockDim.x) {
        if (!flag[k]) continue;
        const uint64_t p = pos[k];
        const int64_t row = layout ? static_cast<int64_t>(layout[pn[k]]) - lo : static_cast<int64_t>(pn[k]) - lo;
        const uint32_t t = static_cast<uint32_t>(layout ? layout[pr[k]] : pr[k]);
        key[p] = (static_cast<uint64_t>(row) << b) | t;
        val[p] = static_cast<uint32_t>(k);
    }
}

struct Sorter {
    ScopedBuf<uint8_t> tmp;
    hipStream_t s;
    hipError_t pairs(const uint64_t* ki, uint64_t* ko, const uint32_t* vi, uint32_t* vo, int64_t m, int bits) {
        size_t need = 0;
        hipError_t e = rocprim::radix_sort_pairs(nullptr, need, ki, ko, vi, vo, static_cast<size_t>(m), 0, bits, s);
        if (e != hipSuccess) return e;
        if (need > tmp.n && (e = tmp.alloc(need)) != hipSuccess) return e;
        return rocprim::radix_sort_pairs(tmp.p, need, ki, ko, vi, vo, static_cast<size_t>(m), 0, bits, s);
    }
    hipError_t keys(const uint64_t* ki, uint64_t* ko, int64_t m, int bits) {
        size_t need = 0;
        hipError_t e = rocprim::radix_sort_keys(nullptr, need, ki, ko, static_cast<size_t>(m), 0, bits, s);
        if (e != hipSuccess) return e;
        if (need > tmp.n && (e = tmp.alloc(need)) != hipSuccess) return e;
        return rocprim::radix_sort_keys(tmp.p, need, ki, ko, static_cast<size_t>(m), 0, bits, s);
    }
    hipError_t excl_scan(const uint32_t* in, uint64_t* out, int64_t m) {
        size_t need = 0;
        hipError_t e = rocprim::exclusive_scan(nullptr, need, in, out, uint64_t(0), static_cast<size_t>(m),
                                               rocprim::plus<uint64_t>(), s);
        if (e != hipSuccess) return e;
        if (need > tmp.n && (e = tmp.alloc(need)) != hipSuccess) return e;
        return rocprim::exclusive_scan(tmp.p, need, in, out, uint64_t(0), static_cast<size_t>(m),
                                       rocprim::plus<uint64_t>(), s);
    }
};

// tgo_load_csr staging: entry k of direction d's list (row v by binary search over off)
// goes to its row's slot rb[v] + (OUT: k - off[v]; IN: out degree + k - off[v]); the other
// endpoint as its Titan id, bad indices flagged.
__global__ void csr_stage(const int64_t* __restrict__ off, const int32_t* __restrict__ idx,
                          const int32_t* __restrict__ w, const int64_t* __restrict__ other_off, int dir, int64_t n,
                          int64_t m, const int64_t* __restrict__ rb, const int64_t* __restrict__ tid,
                          int64_t* __restrict__ other, uint8_t* __restrict__ odir, int32_t* __restrict__ ow, int* bad) {
    for (int64_t k = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; k < m; k += (int64_t)gridDim.x * blockDim.x) {
        int64_t a = 0, b = n;                          // last v with off[v] <= k
        while (b - a > 1) { const int64_t c = (a + b) >> 1; if (off[c] <= k) a = c; else b = c; }
        const int64_t base = dir == 0 ? 0 : other_off[a + 1] - other_off[a];   // IN entries after OUT
        const int64_t pos = rb[a] + base + (k - off[a]);
        const int32_t u = idx[k];
        if (u < 0 || u >= n) { *bad = 1; continue; }
        other[pos] = tid[u];
        odir[pos] = static_cast<uint8_t>(dir);
        if (ow) ow[pos] = w[k];
    }
}

template <class T>
hipError_t download(std::vector<T>& h, const T* d, int64_t count, hipStream_t s) {
    host_resize(h, static_cast<size_t>(count));
    if (count == 0) return hipSuccess;
    const hipError_t e = hipStreamSynchronize(s);
    if (e != hipSuccess) return e;
    return copy_d2h(h.data(), d, static_cast<size_t>(count) * sizeof(T));
}

}  // namespace

int assemble_edges_device(const tgo_edges* e, const tgo_load_opts* opts, int64_t hard_limit, HostGraph& g,
                          hipStream_t s, std::string& err) {
    g = HostGraph();
    const int64_t n = e->n, m = e->m;
    if (n <= 0 || n >= INT32_MAX) { err = "vertex count out of range"; return TGO_E_INVALID; }
    if (m >= (int64_t(1) << 32)) { err = "more than 2^32 edges per load"; return TGO_E_UNSUPPORTED; }
    g.n = n;
    g.scope = opts->scope;
    g.has_weight = opts->weight_key != 0 && e->weight != nullptr;
    g.weight_dt = TGO_DT_INTEGER;
    const bool keep_col = (opts->flags & TGO_LOAD_COLUMN_ORDER) != 0;
    // ids: copied or synthesised by 8 host threads into huge-page-advised memory (n = 2^27 is
    // 1 GB), strictly increasing (checked for caller ids)
    host_resize(g.titan_id, static_cast<size_t>(n));
    {
        constexpr int kT = 8;
        bool bad[kT] = {};
        std::thread th[kT];
        const int64_t per = (n + kT - 1) / kT;
        for (int t = 0; t < kT; ++t)
            th[t] = std::thread([&, t] {
                const int64_t a = std::min(n, t * per), b = std::min(n, a + per);
                for (int64_t v = a; v < b; ++v) {
                    g.titan_id[v] = e->titan_ids ? e->titan_ids[v] : ((v + 1) << 3);
                    if (e->titan_ids && v > 0 && e->titan_ids[v] <= e->titan_ids[v - 1]) bad[t] = true;
                }
            });
        for (auto& x : th) x.join();
        for (bool x : bad)
            if (x) { err = "titan_ids must be strictly increasing"; return TGO_E_INVALID; }
    }
    g.ids_sorted = true;
    const bool cap = opts->apply_cap && opts->n_labels == 0 && opts->scope != TGO_SCOPE_BOTH_E;
    const int64_t limit = cap ? hard_limit : INT64_MAX;
    const bool sort1 = cap || keep_col;          // the cut / column positions need column order first
    int b = 1;
    while ((int64_t(1) << b) < n) ++b;
    const int bits = 2 * b;

    // TGO_TRACE=1: per-phase times on stderr (synchronising the stream at each phase end)
    static const bool trace = std::getenv("TGO_TRACE") && std::atoi(std::getenv("TGO_TRACE")) != 0;
    auto t_last = std::chrono::steady_clock::now();
    auto lap = [&](const char* what) {
        if (!trace && !tracing()) return;
        (void)hipStreamSynchronize(s);
        const auto now = std::chrono::steady_clock::now();
        const double ms = std::chrono::duration<double, std::milli>(now - t_last).count();
        if (trace) std::fprintf(stderr, "[tgo]   assemble %-16s %8.1f ms\n", what, ms);
        trace_complete(std::string("assemble.") + what, ms * 1e3);
        t_last = now;
    };
    ScopedBuf<int32_t> d_src, d_dst, d_w;
    AS_TRY(d_src.alloc(m));
    AS_TRY(d_dst.alloc(m));
    if (m) {
        AS_TRY(copy_chunked(d_src.p, e->src, m * sizeof(int32_t), hipMemcpyHostToDevice));
        AS_TRY(copy_chunked(d_dst.p, e->dst, m * sizeof(int32_t), hipMemcpyHostToDevice));
    }
    if (g.has_weight) {
        AS_TRY(d_w.alloc(m));
        if (m) AS_TRY(copy_chunked(d_w.p, e->weight, m * sizeof(int32_t), hipMemcpyHostToDevice));
    }
    {
        ScopedBuf<int> bad;
        AS_TRY(bad.alloc(1));
        AS_TRY(hipMemsetAsync(bad.p, 0, sizeof(int), s));
        if (m) range_check<<<grid(m), kB, 0, s>>>(d_src.p, d_dst.p, m, n, bad.p);
        int hb = 0;
        AS_TRY(hipMemcpyAsync(&hb, bad.p, sizeof(int), hipMemcpyDeviceToHost, s));
        AS_TRY(hipStreamSynchronize(s));
        if (hb) { err = "edge endpoint out of range"; return TGO_E_INVALID; }
    }
    lap("upload + check");
    Sorter so{{}, s};
    ScopedBuf<uint32_t> deg;
    AS_TRY(deg.alloc(n));
    // ---- sort 1 (column order) + cut, per direction: kept entries' sort-1 keys and payloads
    struct Dir { ScopedBuf<uint64_t> key; ScopedBuf<uint32_t> edge, col; int64_t count = 0; };
    Dir dir[2];                 // [0] OUT (rows = src), [1] IN (rows = dst)
    unsigned long long truncated = 0;
    if (sort1) {
        ScopedBuf<uint64_t> k1[2];
        ScopedBuf<uint32_t> v1[2];
        ScopedBuf<int64_t> off[2], kept[2];
        for (int d = 0; d < 2; ++d) {
            ScopedBuf<uint64_t> kt;
            ScopedBuf<uint32_t> vt;
            AS_TRY(kt.alloc(m));
            AS_TRY(vt.alloc(m));
            AS_TRY(k1[d].alloc(m));
            AS_TRY(v1[d].alloc(m));
            lap(d == 0 ? "sort 1 OUT allocs" : "sort 1 IN allocs");
            if (m) edge_keys<<<grid(m), kB, 0, s>>>(d == 0 ? d_src.p : d_dst.p, d == 0 ? d_dst.p : d_src.p, m, b, nullptr,
                                                    kt.p, vt.p);
            lap(d == 0 ? "sort 1 OUT keys" : "sort 1 IN keys");
            if (m) AS_TRY(so.pairs(kt.p, k1[d].p, vt.p, v1[d].p, m, bits));
            lap(d == 0 ? "sort 1 OUT sort" : "sort 1 IN sort");
            AS_TRY(off[d].alloc(n + 1));
            row_offsets<<<grid(n + 1), kB, 0, s>>>(k1[d].p, m, b, n, off[d].p);
            AS_TRY(kept[d].alloc(n));
        }
        lap("sort 1 scoped frees");
        ScopedBuf<unsigned long long> tr;
        AS_TRY(tr.alloc(1));
        AS_TRY(hipMemsetAsync(tr.p, 0, sizeof(unsigned long long), s));
        cap_rows<<<grid(n), kB, 0, s>>>(off[0].p, off[1].p, n, limit, kept[0].p, kept[1].p, deg.p, tr.p);
        AS_TRY(hipMemcpyAsync(&truncated, tr.p, sizeof(truncated), hipMemcpyDeviceToHost, s));
        for (int d = 0; d < 2; ++d) {
            ScopedBuf<uint32_t> flag, colfull;
            ScopedBuf<uint64_t> pos;
            AS_TRY(flag.alloc(m));
            AS_TRY(pos.alloc(m + 1));
            if (keep_col) AS_TRY(colfull.alloc(m));
            lap(d == 0 ? "cut OUT allocs" : "cut IN allocs");
            if (m) keep_flags<<<grid(m), kB, 0, s>>>(k1[d].p, m, b, off[d].p, kept[d].p, d == 1 ? kept[0].p : nullptr,
                                                     flag.p, keep_col ? colfull.p : nullptr);
            AS_TRY(so.excl_scan(flag.p, pos.p, m));
            uint64_t cnt = 0;
            uint32_t lastf = 0;
            if (m) {
                AS_TRY(hipMemcpyAsync(&cnt, pos.p + m - 1, sizeof(uint64_t), hipMemcpyDeviceToHost, s));
                AS_TRY(hipMemcpyAsync(&lastf, flag.p + m - 1, sizeof(uint32_t), hipMemcpyDeviceToHost, s));
            }
            AS_TRY(hipStreamSynchronize(s));
            lap(d == 0 ? "cut OUT flags + scan" : "cut IN flags + scan");
            const int64_t kc = static_cast<int64_t>(cnt + lastf);
            dir[d].count = kc;
            // kept entries: sort-1 keys (original ids), edge index, column position
            AS_TRY(dir[d].key.alloc(kc));
            AS_TRY(dir[d].edge.alloc(kc));
            if (keep_col) AS_TRY(dir[d].col.alloc(kc));
            ScopedBuf<uint32_t> sel;                           // sort-1 position of each kept entry
            AS_TRY(sel.alloc(kc));
            lap(d == 0 ? "cut OUT kept allocs" : "cut IN kept allocs");
            if (m) compact_kept<<<grid(m), kB, 0, s>>>(k1[d].p, flag.p, pos.p, m, b, nullptr, dir[d].key.p, sel.p);
            if (kc) {
                gather_i32<<<grid(kc), kB, 0, s>>>(sel.p, reinterpret_cast<const int32_t*>(v1[d].p), kc,
                                                   reinterpret_cast<int32_t*>(dir[d].edge.p));
                if (keep_col)
                    gather_i32<<<grid(kc), kB, 0, s>>>(sel.p, reinterpret_cast<const int32_t*>(colfull.p), kc,
                                                       reinterpret_cast<int32_t*>(dir[d].col.p));
            }
            AS_TRY(hipStreamSynchronize(s));             // the scoped buffers are freed next
            lap(d == 0 ? "cut OUT" : "cut IN");
        }
    } else {
        AS_TRY(hipMemsetAsync(deg.p, 0, n * sizeof(uint32_t), s));
        if (m) degree_count<<<grid(m), kB, 0, s>>>(d_src.p, d_dst.p, m, deg.p);
        for (int d = 0; d < 2; ++d) dir[d].count = m;
    }
    g.truncated = static_cast<int64_t>(truncated);
    lap(sort1 ? "sort 1 + cut" : "degrees");
    // ---- degree-grouped relabel: perm[v] = position of v (hottest half-octave first)
    ScopedBuf<int32_t> perm;
    AS_TRY(perm.alloc(n));
    {
        ScopedBuf<uint64_t> bk, bs;
        AS_TRY(bk.alloc(n));
        AS_TRY(bs.alloc(n));
        bucket_keys<<<grid(n), kB, 0, s>>>(deg.p, n, bk.p);
        AS_TRY(so.keys(bk.p, bs.p, n, 32 + 7));
        order_to_perm<<<grid(n), kB, 0, s>>>(bs.p, n, perm.p);
    }
    deg.release();
    lap("relabel");
    // ---- sort 2: final lists in (perm[row], perm[neighbour]) order
    HostCsr* outc[2] = {&g.out, &g.in};
    ScopedBuf<uint64_t> fkey[2];                    // final keys (kept for the transpose)
    ScopedBuf<int32_t> fadj[2], fw[2];
    for (int d = 0; d < 2; ++d) {
        const int64_t c = dir[d].count;
        ScopedBuf<uint64_t> kt;
        ScopedBuf<uint32_t> vt, vs;
        AS_TRY(kt.alloc(c));
        AS_TRY(fkey[d].alloc(c));
        const bool payload = g.has_weight || keep_col;
        if (sort1) {
            // re-key the kept sort-1 entries through perm, payload = their kept index
            AS_TRY(vt.alloc(payload ? c : 0));
            if (c) rekey<<<grid(c), kB, 0, s>>>(dir[d].key.p, c, b, perm.p, kt.p, payload ? vt.p : nullptr);
            lap(d == 0 ? "OUT rekey" : "IN rekey");
            dir[d].key.release();
            lap(d == 0 ? "OUT free sort-1 keys" : "IN free sort-1 keys");
        } else {
            AS_TRY(vt.alloc(payload ? c : 0));
            if (c) edge_keys<<<grid(c), kB, 0, s>>>(d == 0 ? d_src.p : d_dst.p, d == 0 ? d_dst.p : d_src.p, c, b, perm.p,
                                                    kt.p, payload ? vt.p : nullptr);
        }
        if (payload) {
            AS_TRY(vs.alloc(c));
            if (c) AS_TRY(so.pairs(kt.p, fkey[d].p, vt.p, vs.p, c, bits));
        } else if (c) {
            AS_TRY(so.keys(kt.p, fkey[d].p, c, bits));
        }
        lap(d == 0 ? "OUT sort 2" : "IN sort 2");
        kt.release();
        HostCsr& hc = *outc[d];
        ScopedBuf<int64_t> off;
        AS_TRY(off.alloc(n + 1));
        row_offsets<<<grid(n + 1), kB, 0, s>>>(fkey[d].p, c, b, n, off.p);
        AS_TRY(fadj[d].alloc(c));
        ScopedBuf<uint32_t> col;
        if (g.has_weight) AS_TRY(fw[d].alloc(c));
        if (keep_col) AS_TRY(col.alloc(c));
        if (c)
            emit_list<<<grid(c), kB, 0, s>>>(fkey[d].p, payload ? vs.p : nullptr, c, b,
                                             sort1 ? dir[d].edge.p : nullptr, d_w.p, sort1 ? dir[d].col.p : nullptr,
                                             fadj[d].p, g.has_weight ? fw[d].p : nullptr, keep_col ? col.p : nullptr);
        lap(d == 0 ? "OUT offsets + emit" : "IN offsets + emit");
        AS_TRY(download(hc.off, off.p, n + 1, s));
        if (g.has_weight) {                          // weight_sorted_push reads the host lists
            AS_TRY(download(hc.adj, fadj[d].p, c, s));
            AS_TRY(download(hc.w, fw[d].p, c, s));
        }
        AS_TRY(hipStreamSynchronize(s));
        lap(d == 0 ? "OUT download" : "IN download");
        if (keep_col) hc.dcol.own(col.take(), c);
        dir[d].edge.release();
        dir[d].col.release();
        lap(d == 0 ? "OUT frees" : "IN frees");
    }
    AS_TRY(download(g.perm, perm.p, n, s));
    // ---- push view: equal to the stored opposite list unless the cut made rows asymmetric
    g.has_transpose = g.truncated != 0;
    if (g.has_transpose && g.scope != TGO_SCOPE_BOTH_E) {
        const int d = g.scope == TGO_SCOPE_IN_E ? 0 : 1;      // pull list of inE = OUT rows, outE = IN rows
        const int64_t c = dir[d].count;
        ScopedBuf<uint64_t> tk, ts;
        ScopedBuf<uint32_t> tv, tvs;
        AS_TRY(tk.alloc(c));
        AS_TRY(ts.alloc(c));
        AS_TRY(tv.alloc(g.has_weight ? c : 0));
        lap("transpose allocs");
        if (c) transpose_keys<<<grid(c), kB, 0, s>>>(fkey[d].p, c, b, tk.p, g.has_weight ? tv.p : nullptr);
        lap("transpose keys");
        if (g.has_weight) {
            AS_TRY(tvs.alloc(c));
            if (c) AS_TRY(so.pairs(tk.p, ts.p, tv.p, tvs.p, c, bits));
        } else if (c) {
            AS_TRY(so.keys(tk.p, ts.p, c, bits));
        }
        lap("transpose sort");
        ScopedBuf<int64_t> off;
        AS_TRY(off.alloc(n + 1));
        row_offsets<<<grid(n + 1), kB, 0, s>>>(ts.p, c, b, n, off.p);
        ScopedBuf<int32_t> adj, w;
        AS_TRY(adj.alloc(c));
        if (g.has_weight) AS_TRY(w.alloc(c));
        if (c) emit_list<<<grid(c), kB, 0, s>>>(ts.p, g.has_weight ? tvs.p : nullptr, c, b, nullptr, fw[d].p, nullptr,
                                                adj.p, g.has_weight ? w.p : nullptr, nullptr);
        AS_TRY(download(g.push_t.off, off.p, n + 1, s));
        if (g.has_weight) {
            AS_TRY(download(g.push_t.adj, adj.p, c, s));
            AS_TRY(download(g.push_t.w, w.p, c, s));
        }
        AS_TRY(hipStreamSynchronize(s));
        g.push_t.dadj.own(adj.take(), c);
        if (g.has_weight) g.push_t.dw.own(w.take(), c);
        lap("transpose");
    }
    AS_TRY(hipStreamSynchronize(s));
    // the final lists stay on the device: upload_graph adopts them
    for (int d = 0; d < 2; ++d) {
        outc[d]->dadj.own(fadj[d].take(), dir[d].count);
        if (g.has_weight) outc[d]->dw.own(fw[d].take(), dir[d].count);
    }
    return TGO_OK;
}


// tgo_load_partition on the device: the rows of the owned range [lo, hi) of a global edge
// list (graph_build.cpp assemble_partition, array for array).  Row v (local) has the OUT
// entries of the edges with src = lo + v and the IN entries of those with dst = lo + v, each
// in column order (global neighbour, edge index) — the owned entries compacted in edge order,
// then one stable sort by (row, neighbour); the untyped single-direction scopes cut each row
// at the limit (OUT first); with a layout, rows and neighbours move to their layout ids and a
// second stable sort restores (row, neighbour) order, equal entries keeping the cut order.
int assemble_partition_device(const tgo_edges* e, int64_t n_global, int64_t lo, int64_t hi, const tgo_load_opts* opts,
                              int64_t hard_limit, const int32_t* layout, HostGraph& g, hipStream_t s, std::string& err) {
    g = HostGraph();
    const int64_t n = hi - lo, m = e->m;
    if (lo < 0 || hi > n_global || n <= 0 || n_global >= INT32_MAX) { err = "invalid partition range"; return TGO_E_INVALID; }
    if (m >= (int64_t(1) << 32)) { err = "more than 2^32 edges per load"; return TGO_E_UNSUPPORTED; }
    g.n = n;
    g.scope = opts->scope;
    g.has_weight = opts->weight_key != 0 && e->weight != nullptr;
    g.weight_dt = TGO_DT_INTEGER;
    g.titan_id.resize(n);
    for (int64_t v = 0; v < n; ++v) g.titan_id[v] = (lo + v + 1) << 3;
    if (layout) {                 // owned rows move inside [lo, hi); neighbours take their owners' layout
        g.perm.resize(n);
        std::vector<uint8_t> seen(n, 0);
        for (int64_t v = 0; v < n; ++v) {
            const int64_t p = static_cast<int64_t>(layout[lo + v]) - lo;
            if (p < 0 || p >= n || seen[p]) { err = "layout is not a permutation of the owned range"; return TGO_E_INVALID; }
            seen[p] = 1;
            g.perm[v] = static_cast<int32_t>(p);
        }
    }
    const bool cap = opts->apply_cap && opts->n_labels == 0 && opts->scope != TGO_SCOPE_BOTH_E;
    const int64_t limit = cap ? hard_limit : INT64_MAX;
    int b = 1;                    // neighbour bits (global ids)
    while ((int64_t(1) << b) < n_global) ++b;
    int br = 1;                   // row bits (local ids)
    while ((int64_t(1) << br) < n) ++br;
    const int bits = b + br;
    static const bool trace = std::getenv("TGO_TRACE") && std::atoi(std::getenv("TGO_TRACE")) != 0;
    auto t_last = std::chrono::steady_clock::now();
    auto lap = [&](const char* what) {
        if (!trace && !tracing()) return;
        (void)hipStreamSynchronize(s);
        const auto now = std::chrono::steady_clock::now();
        const double ms = std::chrono::duration<double, std::milli>(now - t_last).count();
        if (trace) std::fprintf(stderr, "[tgo]   partition %-14s %8.1f ms\n", what, ms);
        trace_complete(std::string("partition.") + what, ms * 1e3);
        t_last = now;
    };
    ScopedBuf<int32_t> d_src, d_dst, d_w, d_lay;
    AS_TRY(d_src.alloc(m));
    AS_TRY(d_dst.alloc(m));
    if (m) {
        AS_TRY(copy_chunked(d_src.p, e->src, m * sizeof(int32_t), hipMemcpyHostToDevice));
        AS_TRY(copy_chunked(d_dst.p, e->dst, m * sizeof(int32_t), hipMemcpyHostToDevice));
    }
    if (g.has_weight) {
        AS_TRY(d_w.alloc(m));
        if (m) AS_TRY(copy_chunked(d_w.p, e->weight, m * sizeof(int32_t), hipMemcpyHostToDevice));
    }
    if (layout) {
        AS_TRY(d_lay.alloc(n_global));
        AS_TRY(copy_chunked(d_lay.p, layout, n_global * sizeof(int32_t), hipMemcpyHostToDevice));
    }
    {
        ScopedBuf<int> bad;
        AS_TRY(bad.alloc(1));
        AS_TRY(hipMemsetAsync(bad.p, 0, sizeof(int), s));
        if (m) range_check<<<grid(m), kB, 0, s>>>(d_src.p, d_dst.p, m, n_global, bad.p);
        int hb = 0;
        AS_TRY(hipMemcpyAsync(&hb, bad.p, sizeof(int), hipMemcpyDeviceToHost, s));
        AS_TRY(hipStreamSynchronize(s));
        if (hb) { err = "edge endpoint out of range"; return TGO_E_INVALID; }
    }
    lap("upload + check");
    Sorter so{{}, s};
    auto count_of = [&](const uint32_t* flag, const uint64_t* pos, int64_t len, int64_t& out) -> hipError_t {
        uint64_t cnt = 0;
        uint32_t lastf = 0;
        out = 0;
        if (!len) return hipSuccess;
        hipError_t x = hipMemcpyAsync(&cnt, pos + len - 1, sizeof(uint64_t), hipMemcpyDeviceToHost, s);
        if (x == hipSuccess) x = hipMemcpyAsync(&lastf, flag + len - 1, sizeof(uint32_t), hipMemcpyDeviceToHost, s);
        if (x == hipSuccess) x = hipStreamSynchronize(s);
        out = static_cast<int64_t>(cnt + lastf);
        return x;
    };
    // ---- owned entries of each direction, sorted by (row, neighbour) from edge order
    ScopedBuf<uint64_t> k1[2];
    ScopedBuf<uint32_t> v1[2];
    ScopedBuf<int64_t> off[2], kept[2];
    int64_t cnt[2] = {0, 0};
    for (int d = 0; d < 2; ++d) {
        const int32_t* own = d == 0 ? d_src.p : d_dst.p;
        const int32_t* nbr = d == 0 ? d_dst.p : d_src.p;
        ScopedBuf<uint32_t> flag;
        ScopedBuf<uint64_t> pos;
        AS_TRY(flag.alloc(m));
        AS_TRY(pos.alloc(m + 1));
        if (m) owned_flags<<<grid(m), kB, 0, s>>>(own, m, lo, hi, flag.p);
        AS_TRY(so.excl_scan(flag.p, pos.p, m));
        AS_TRY(count_of(flag.p, pos.p, m, cnt[d]));
        ScopedBuf<uint64_t> kt;
        ScopedBuf<uint32_t> vt;
        AS_TRY(kt.alloc(cnt[d]));
        AS_TRY(vt.alloc(cnt[d]));
        if (m) owned_keys<<<grid(m), kB, 0, s>>>(own, nbr, flag.p, pos.p, m, lo, b, kt.p, vt.p);
        AS_TRY(k1[d].alloc(cnt[d]));
        AS_TRY(v1[d].alloc(cnt[d]));
        if (cnt[d]) AS_TRY(so.pairs(kt.p, k1[d].p, vt.p, v1[d].p, cnt[d], bits));
        AS_TRY(off[d].alloc(n + 1));
        row_offsets<<<grid(n + 1), kB, 0, s>>>(k1[d].p, cnt[d], b, n, off[d].p);
        AS_TRY(kept[d].alloc(n));
        AS_TRY(hipStreamSynchronize(s));            // the scoped buffers are freed next
    }
    lap("owned + sort 1");
    // ---- the cut (OUT entries first, then IN, up to the limit per row)
    unsigned long long truncated = 0;
    {
        ScopedBuf<unsigned long long> tr;
        ScopedBuf<uint32_t> deg;
        AS_TRY(tr.alloc(1));
        AS_TRY(deg.alloc(n));
        AS_TRY(hipMemsetAsync(tr.p, 0, sizeof(unsigned long long), s));
        cap_rows<<<grid(n), kB, 0, s>>>(off[0].p, off[1].p, n, limit, kept[0].p, kept[1].p, deg.p, tr.p);
        AS_TRY(hipMemcpyAsync(&truncated, tr.p, sizeof(truncated), hipMemcpyDeviceToHost, s));
        AS_TRY(hipStreamSynchronize(s));
    }
    g.truncated = static_cast<int64_t>(truncated);
    HostCsr* outc[2] = {&g.out, &g.in};
    ScopedBuf<int32_t> fadj[2], fw[2];
    int64_t fc[2] = {0, 0};
    for (int d = 0; d < 2; ++d) {
        // kept entries: keys in cut order, payload = edge index
        ScopedBuf<uint64_t> kk;
        ScopedBuf<uint32_t> ke;
        if (truncated) {
            ScopedBuf<uint32_t> flag, sel;
            ScopedBuf<uint64_t> pos;
            AS_TRY(flag.alloc(cnt[d]));
            AS_TRY(pos.alloc(cnt[d] + 1));
            if (cnt[d]) keep_flags<<<grid(cnt[d]), kB, 0, s>>>(k1[d].p, cnt[d], b, off[d].p, kept[d].p, nullptr, flag.p, nullptr);
            AS_TRY(so.excl_scan(flag.p, pos.p, cnt[d]));
            AS_TRY(count_of(flag.p, pos.p, cnt[d], fc[d]));
            AS_TRY(kk.alloc(fc[d]));
            AS_TRY(ke.alloc(fc[d]));
            AS_TRY(sel.alloc(fc[d]));
            if (cnt[d]) compact_kept<<<grid(cnt[d]), kB, 0, s>>>(k1[d].p, flag.p, pos.p, cnt[d], b, nullptr, kk.p, sel.p);
            if (fc[d]) gather_i32<<<grid(fc[d]), kB, 0, s>>>(sel.p, reinterpret_cast<const int32_t*>(v1[d].p), fc[d],
                                                          reinterpret_cast<int32_t*>(ke.p));
            AS_TRY(hipStreamSynchronize(s));
            k1[d].release();
            v1[d].release();
        } else {
            fc[d] = cnt[d];
            kk.p = k1[d].take();
            kk.n = static_cast<size_t>(cnt[d]);
            ke.p = v1[d].take();
            ke.n = static_cast<size_t>(cnt[d]);
        }
        const int64_t c = fc[d];
        // ---- layout: (layout row, layout neighbour), stable from the cut order
        ScopedBuf<uint64_t> fkey;
        ScopedBuf<uint32_t> fval;                    // payload: index into the cut order
        if (layout) {
            ScopedBuf<uint64_t> kt;
            ScopedBuf<uint32_t> vt;
            AS_TRY(kt.alloc(c));
            AS_TRY(vt.alloc(c));
            if (c) part_rekey<<<grid(c), kB, 0, s>>>(kk.p, c, b, d_lay.p, lo, kt.p, vt.p);
            AS_TRY(fkey.alloc(c));
            AS_TRY(fval.alloc(c));
            if (c) AS_TRY(so.pairs(kt.p, fkey.p, vt.p, fval.p, c, bits));
            AS_TRY(hipStreamSynchronize(s));
            kk.release();
        } else {
            fkey.p = kk.take();
            fkey.n = static_cast<size_t>(c);
        }
        ScopedBuf<int64_t> foff;
        AS_TRY(foff.alloc(n + 1));
        row_offsets<<<grid(n + 1), kB, 0, s>>>(fkey.p, c, b, n, foff.p);
        AS_TRY(fadj[d].alloc(c));
        if (g.has_weight) AS_TRY(fw[d].alloc(c));
        if (c)
            emit_list<<<grid(c), kB, 0, s>>>(fkey.p, layout ? fval.p : nullptr, c, b, layout ? ke.p : nullptr, d_w.p,
                                             nullptr, fadj[d].p, nullptr, nullptr);
        if (c && g.has_weight) {
            // weights through the payload chain: entry -> cut index (fval, with a layout) -> edge index
            ScopedBuf<uint32_t> eidx;
            AS_TRY(eidx.alloc(c));
            if (layout) gather_i32<<<grid(c), kB, 0, s>>>(fval.p, reinterpret_cast<const int32_t*>(ke.p), c,
                                                          reinterpret_cast<int32_t*>(eidx.p));
            gather_i32<<<grid(c), kB, 0, s>>>(layout ? eidx.p : ke.p, d_w.p, c, fw[d].p);
            AS_TRY(hipStreamSynchronize(s));
        }
        HostCsr& hc = *outc[d];
        AS_TRY(download(hc.off, foff.p, n + 1, s));
        if (g.has_weight) {                          // weight_sorted_push reads the host lists
            AS_TRY(download(hc.adj, fadj[d].p, c, s));
            AS_TRY(download(hc.w, fw[d].p, c, s));
        }
        AS_TRY(hipStreamSynchronize(s));
        lap(d == 0 ? "OUT" : "IN");
    }
    g.has_transpose = false;
    // ---- push view of a cut single-direction scope: the pull lists of EVERY rank decide which
    // entries a vertex pushes along (u pushes to v iff u survived in v's cut pull list), so the
    // owned push rows come from the global cut, not from the owned rows' own cut opposite lists
    // (the one-GPU load's explicit transpose, partitioned)
    if (cap && m) {
        const bool pull_out = opts->scope == TGO_SCOPE_IN_E;        // inE pulls over OUT entries
        const int32_t* prow = pull_out ? d_src.p : d_dst.p;          // pull row (receiver)
        const int32_t* pnbr = pull_out ? d_dst.p : d_src.p;          // pull neighbour (pusher)
        ScopedBuf<uint32_t> dout, din, kept_g;
        ScopedBuf<int> drops;
        AS_TRY(dout.alloc(n_global));
        AS_TRY(din.alloc(n_global));
        AS_TRY(kept_g.alloc(n_global));
        AS_TRY(drops.alloc(1));
        AS_TRY(hipMemsetAsync(dout.p, 0, n_global * 4, s));
        AS_TRY(hipMemsetAsync(din.p, 0, n_global * 4, s));
        AS_TRY(hipMemsetAsync(drops.p, 0, sizeof(int), s));
        degree_both<<<grid(m), kB, 0, s>>>(d_src.p, d_dst.p, m, dout.p, din.p);
        pull_kept<<<grid(n_global), kB, 0, s>>>(dout.p, din.p, n_global, limit, pull_out ? 1 : 0, kept_g.p, drops.p);
        int any = 0;
        AS_TRY(hipMemcpyAsync(&any, drops.p, sizeof(int), hipMemcpyDeviceToHost, s));
        AS_TRY(hipStreamSynchronize(s));
        if (any) {
            ScopedBuf<uint8_t> dropped;
            AS_TRY(dropped.alloc(m));
            AS_TRY(hipMemsetAsync(dropped.p, 0, m, s));
            {   // rank of every entry of the cut rows in its row's column order (neighbour, edge)
                ScopedBuf<uint32_t> flag;
                ScopedBuf<uint64_t> pos;
                AS_TRY(flag.alloc(m));
                AS_TRY(pos.alloc(m + 1));
                cut_row_flags<<<grid(m), kB, 0, s>>>(prow, m, kept_g.p, pull_out ? dout.p : din.p, flag.p);
                AS_TRY(so.excl_scan(flag.p, pos.p, m));
                int64_t c = 0;
                AS_TRY(count_of(flag.p, pos.p, m, c));
                ScopedBuf<uint64_t> kt, ks;
                ScopedBuf<uint32_t> vt, vs;
                AS_TRY(kt.alloc(c)); AS_TRY(vt.alloc(c)); AS_TRY(ks.alloc(c)); AS_TRY(vs.alloc(c));
                // the cut rows' entries: key = row << b | neighbour (the owned_keys layout, lo = 0)
                owned_keys<<<grid(m), kB, 0, s>>>(prow, pnbr, flag.p, pos.p, m, 0, b, kt.p, vt.p);
                int bg = 1;
                while ((int64_t(1) << bg) < n_global) ++bg;
                if (c) AS_TRY(so.pairs(kt.p, ks.p, vt.p, vs.p, c, b + bg));
                if (c) mark_dropped<<<grid(c), kB, 0, s>>>(ks.p, vs.p, c, b, kept_g.p, dropped.p);
                AS_TRY(hipStreamSynchronize(s));
            }
            ScopedBuf<uint32_t> flag;
            ScopedBuf<uint64_t> pos;
            AS_TRY(flag.alloc(m));
            AS_TRY(pos.alloc(m + 1));
            push_flags<<<grid(m), kB, 0, s>>>(pnbr, m, lo, hi, dropped.p, flag.p);
            AS_TRY(so.excl_scan(flag.p, pos.p, m));
            int64_t c = 0;
            AS_TRY(count_of(flag.p, pos.p, m, c));
            ScopedBuf<uint64_t> kt, ks;
            ScopedBuf<uint32_t> vt, vs;
            AS_TRY(kt.alloc(c)); AS_TRY(vt.alloc(c)); AS_TRY(ks.alloc(c)); AS_TRY(vs.alloc(c));
            push_keys<<<grid(m), kB, 0, s>>>(pnbr, prow, flag.p, pos.p, m, lo, b, layout ? d_lay.p : nullptr, kt.p, vt.p);
            if (c) AS_TRY(so.pairs(kt.p, ks.p, vt.p, vs.p, c, bits));
            ScopedBuf<int64_t> poff;
            AS_TRY(poff.alloc(n + 1));
            row_offsets<<<grid(n + 1), kB, 0, s>>>(ks.p, c, b, n, poff.p);
            ScopedBuf<int32_t> padj, pw;
            AS_TRY(padj.alloc(c));
            if (g.has_weight) AS_TRY(pw.alloc(c));
            if (c) emit_list<<<grid(c), kB, 0, s>>>(ks.p, vs.p, c, b, nullptr, d_w.p, nullptr, padj.p,
                                                    g.has_weight ? pw.p : nullptr, nullptr);
            AS_TRY(download(g.push_t.off, poff.p, n + 1, s));
            if (g.has_weight) {
                AS_TRY(download(g.push_t.adj, padj.p, c, s));
                AS_TRY(download(g.push_t.w, pw.p, c, s));
            }
            AS_TRY(hipStreamSynchronize(s));
            g.push_t.dadj.own(padj.take(), c);
            if (g.has_weight) g.push_t.dw.own(pw.take(), c);
            g.has_transpose = true;
            lap("push transpose");
        }
    }
    for (int d = 0; d < 2; ++d) {
        outc[d]->dadj.own(fadj[d].take(), fc[d]);
        if (g.has_weight) outc[d]->dw.own(fw[d].take(), fc[d]);
    }
    return TGO_OK;
}

int stage_csr_device(const CsrInput& in, bool weighted, RowStaging& st, hipStream_t s, std::string& err) {
    const int64_t n = in.n;
    if (n < 0 || n >= INT32_MAX) { err = "vertex count out of range"; return TGO_E_INVALID; }
    int64_t m[2];
    for (int d = 0; d < 2; ++d) {
        if (!in.off[d] || (n > 0 && in.off[d][0] != 0)) { err = "offsets must start at 0"; return TGO_E_INVALID; }
        for (int64_t v = 0; v < n; ++v)
            if (in.off[d][v + 1] < in.off[d][v]) { err = "row offsets decrease"; return TGO_E_INVALID; }
        m[d] = n > 0 ? in.off[d][n] : 0;
        if (m[d] > 0 && !in.idx[d]) { err = "null index array"; return TGO_E_INVALID; }
        if (weighted && m[d] > 0 && !in.w[d]) { err = "a weight array is missing"; return TGO_E_INVALID; }
    }
    const int64_t E = m[0] + m[1];
    if (E >= (int64_t(1) << 32)) { err = "more than 2^32 entries per load"; return TGO_E_UNSUPPORTED; }
    st.vid.resize(n);
    for (int64_t v = 0; v < n; ++v) st.vid[v] = in.titan_ids ? in.titan_ids[v] : ((v + 1) << 3);
    for (int64_t v = 1; in.titan_ids && v < n; ++v)
        if (in.titan_ids[v] <= in.titan_ids[v - 1]) { err = "titan_ids must be strictly increasing"; return TGO_E_INVALID; }
    st.rep.assign(n, 0);
    st.row_begin.resize(n + 1);
    st.row_begin[0] = 0;
    for (int64_t v = 0; v < n; ++v)
        st.row_begin[v + 1] = st.row_begin[v] + (in.off[0][v + 1] - in.off[0][v]) + (in.off[1][v + 1] - in.off[1][v]);
    int64_t* d_other = nullptr;
    uint8_t* d_dir = nullptr;
    int32_t* d_w = nullptr;
    AS_TRY(hipMalloc(&d_other, std::max<int64_t>(E, 1) * 8));
    st.d_other.own(d_other, E);
    AS_TRY(hipMalloc(&d_dir, std::max<int64_t>(E, 1)));
    st.d_dir.own(d_dir, E);
    if (weighted) {
        AS_TRY(hipMalloc(&d_w, std::max<int64_t>(E, 1) * 4));
        st.d_w.own(d_w, E);
    }
    if (n == 0 || E == 0) return TGO_OK;
    ScopedBuf<int64_t> tid, rb, off[2];
    ScopedBuf<int32_t> idx, w;
    ScopedBuf<int> bad;
    AS_TRY(tid.alloc(n)); AS_TRY(rb.alloc(n + 1)); AS_TRY(bad.alloc(1));
    AS_TRY(copy_chunked(tid.p, st.vid.data(), n * 8, hipMemcpyHostToDevice));
    AS_TRY(copy_chunked(rb.p, st.row_begin.data(), (n + 1) * 8, hipMemcpyHostToDevice));
    for (int d = 0; d < 2; ++d) {
        AS_TRY(off[d].alloc(n + 1));
        AS_TRY(copy_chunked(off[d].p, in.off[d], (n + 1) * 8, hipMemcpyHostToDevice));
    }
    AS_TRY(hipMemsetAsync(bad.p, 0, sizeof(int), s));
    for (int d = 0; d < 2; ++d) {
        if (m[d] == 0) continue;
        AS_TRY(idx.alloc(m[d]));
        AS_TRY(copy_chunked(idx.p, in.idx[d], m[d] * 4, hipMemcpyHostToDevice));
        if (weighted) {
            AS_TRY(w.alloc(m[d]));
            AS_TRY(copy_chunked(w.p, in.w[d], m[d] * 4, hipMemcpyHostToDevice));
        }
        csr_stage<<<grid(m[d]), kB, 0, s>>>(off[d].p, idx.p, weighted ? w.p : nullptr, off[0].p, d, n, m[d], rb.p, tid.p,
                                            d_other, d_dir, weighted ? d_w : nullptr, bad.p);
        AS_TRY(hipStreamSynchronize(s));                 // idx / w are reused by the next direction
    }
    int hb = 0;
    AS_TRY(hipMemcpyAsync(&hb, bad.p, sizeof(int), hipMemcpyDeviceToHost, s));
    AS_TRY(hipStreamSynchronize(s));
    if (hb) { err = "neighbour index out of range"; return TGO_E_INVALID; }
    return TGO_OK;
}

// Row loads (tgo_load_rows + tgo_finish_load): the host assemble_from_rows, on the device.
// Vertex cuts (representative rows, PartitionedVertex ids) keep the host path (the caller
// checks); the staging is the decoder's, in row order with each row in column order.
int assemble_rows_device(RowStaging& st, HostGraph& g, hipStream_t s, std::string& err) {
    g = HostGraph();
    const int64_t n = static_cast<int64_t>(st.vid.size());
    if (n >= INT32_MAX) { err = "more than 2^31-1 vertices per device"; return TGO_E_UNSUPPORTED; }
    const int64_t E = st.entries();
    if (E >= (int64_t(1) << 32)) { err = "more than 2^32 staged entries"; return TGO_E_UNSUPPORTED; }
    g.n = n;
    g.titan_id = st.vid;
    g.scope = st.opts.scope;
    g.has_weight = st.opts.weight_key != 0;
    g.weight_dt = st.plan.weight_dt ? st.plan.weight_dt : TGO_DT_INTEGER;
    g.ghost = st.ghost; g.truncated = st.truncated; g.skipped = st.skipped;
    const bool keep_col = (st.opts.flags & TGO_LOAD_COLUMN_ORDER) != 0;
    const bool weighted = g.has_weight && (st.d_other.present() ? st.d_w.n == E : static_cast<int64_t>(st.w.size()) == E);
    if (g.has_weight && !weighted) { err = "staged weights out of step"; return TGO_E_STATE; }
    if (n == 0) {
        g.out.off.assign(1, 0); g.in.off.assign(1, 0);
        st = RowStaging();
        return TGO_OK;
    }
    int b = 1;
    while ((int64_t(1) << b) < n) ++b;
    const int bits = 2 * b;
    Sorter so{{}, s};
    ScopedBuf<int64_t> d_vid, d_other, d_rb;
    ScopedBuf<uint8_t> d_dir;
    ScopedBuf<int32_t> d_w;
    AS_TRY(d_vid.alloc(n));
    AS_TRY(d_rb.alloc(n + 1));
    AS_TRY(copy_chunked(d_vid.p, st.vid.data(), n * 8, hipMemcpyHostToDevice));
    AS_TRY(copy_chunked(d_rb.p, st.row_begin.data(), (n + 1) * 8, hipMemcpyHostToDevice));
    // staged entries: in place when the device decoder left them on the device
    const bool dev_staged = st.d_other.present();
    const int64_t* p_other = st.d_other.p;
    const uint8_t* p_dir = st.d_dir.p;
    const int32_t* p_w = st.d_w.p;
    if (!dev_staged) {
        AS_TRY(d_other.alloc(E));
        AS_TRY(d_dir.alloc(E));
        if (E) {
            AS_TRY(copy_chunked(d_other.p, st.other.data(), E * 8, hipMemcpyHostToDevice));
            AS_TRY(copy_chunked(d_dir.p, st.dir.data(), E, hipMemcpyHostToDevice));
        }
        if (weighted) {
            AS_TRY(d_w.alloc(E));
            if (E) AS_TRY(copy_chunked(d_w.p, st.w.data(), E * 4, hipMemcpyHostToDevice));
        }
        p_other = d_other.p;
        p_dir = d_dir.p;
        p_w = d_w.p;
    }
    if (!weighted) p_w = nullptr;
    // id map: vertex ids sorted (signed order), their dense index alongside
    ScopedBuf<uint64_t> ik, sk;
    ScopedBuf<uint32_t> iv, sv;
    AS_TRY(ik.alloc(n)); AS_TRY(sk.alloc(n)); AS_TRY(iv.alloc(n)); AS_TRY(sv.alloc(n));
    id_keys<<<grid(n), kB, 0, s>>>(d_vid.p, n, ik.p, iv.p);
    AS_TRY(so.pairs(ik.p, sk.p, iv.p, sv.p, n, 64));
    ik.release(); iv.release();
    ScopedBuf<int32_t> row, dense;
    ScopedBuf<uint32_t> fl[2], col;
    AS_TRY(row.alloc(E)); AS_TRY(dense.alloc(E)); AS_TRY(fl[0].alloc(E)); AS_TRY(fl[1].alloc(E));
    if (E) entry_dense<<<grid(E), kB, 0, s>>>(p_other, p_dir, E, d_rb.p, n, sk.p, sv.p, row.p, dense.p, fl[0].p, fl[1].p);
    if (keep_col) {
        AS_TRY(col.alloc(E));
        if (E) col_of<<<grid(E), kB, 0, s>>>(row.p, d_rb.p, E, col.p);
    }
    AS_TRY(hipStreamSynchronize(s));
    d_other.release(); d_dir.release(); sk.release(); sv.release();
    st.d_other.reset(); st.d_dir.reset();
    // per direction: kept entries in staged order, keys row << b | dense
    ScopedBuf<uint64_t> k1[2];
    ScopedBuf<uint32_t> v1[2];
    ScopedBuf<int64_t> off1[2];
    int64_t cnt[2] = {0, 0};
    for (int d = 0; d < 2; ++d) {
        ScopedBuf<uint64_t> pos;
        AS_TRY(pos.alloc(E + 1));
        AS_TRY(so.excl_scan(fl[d].p, pos.p, E + 0));
        uint64_t last = 0;
        uint32_t lf = 0;
        if (E) {
            AS_TRY(hipMemcpyAsync(&last, pos.p + E - 1, 8, hipMemcpyDeviceToHost, s));
            AS_TRY(hipMemcpyAsync(&lf, fl[d].p + E - 1, 4, hipMemcpyDeviceToHost, s));
        }
        AS_TRY(hipStreamSynchronize(s));
        cnt[d] = static_cast<int64_t>(last + lf);
        AS_TRY(k1[d].alloc(cnt[d])); AS_TRY(v1[d].alloc(cnt[d])); AS_TRY(off1[d].alloc(n + 1));
        if (E) compact_dir<<<grid(E), kB, 0, s>>>(fl[d].p, pos.p, E, b, row.p, dense.p, k1[d].p, v1[d].p);
        row_offsets<<<grid(n + 1), kB, 0, s>>>(k1[d].p, cnt[d], b, n, off1[d].p);
        AS_TRY(hipStreamSynchronize(s));
    }
    row.release(); dense.release(); fl[0].release(); fl[1].release();
    // degree-grouped relabel over the kept lists
    ScopedBuf<int32_t> perm;
    AS_TRY(perm.alloc(n));
    {
        ScopedBuf<uint32_t> deg;
        ScopedBuf<uint64_t> bk, bs;
        AS_TRY(deg.alloc(n)); AS_TRY(bk.alloc(n)); AS_TRY(bs.alloc(n));
        degree_rows<<<grid(n), kB, 0, s>>>(off1[0].p, off1[1].p, n, deg.p);
        bucket_keys<<<grid(n), kB, 0, s>>>(deg.p, n, bk.p);
        AS_TRY(so.keys(bk.p, bs.p, n, 32 + 7));
        order_to_perm<<<grid(n), kB, 0, s>>>(bs.p, n, perm.p);
        AS_TRY(hipStreamSynchronize(s));
    }
    // final lists: stable sort by (perm[row], perm[neighbour]) from the staged order
    HostCsr* outc[2] = {&g.out, &g.in};
    ScopedBuf<uint64_t> fkey[2];
    ScopedBuf<int32_t> fadj[2], fw[2];
    ScopedBuf<int64_t> foff[2];
    ScopedBuf<uint32_t> fcol[2];
    for (int d = 0; d < 2; ++d) {
        const int64_t c = cnt[d];
        ScopedBuf<uint64_t> kt;
        ScopedBuf<uint32_t> vt, vs;
        AS_TRY(kt.alloc(c)); AS_TRY(vt.alloc(c)); AS_TRY(vs.alloc(c)); AS_TRY(fkey[d].alloc(c));
        if (c) rekey<<<grid(c), kB, 0, s>>>(k1[d].p, c, b, perm.p, kt.p, vt.p);
        if (c) AS_TRY(so.pairs(kt.p, fkey[d].p, vt.p, vs.p, c, bits));
        k1[d].release();
        AS_TRY(foff[d].alloc(n + 1));
        row_offsets<<<grid(n + 1), kB, 0, s>>>(fkey[d].p, c, b, n, foff[d].p);
        AS_TRY(fadj[d].alloc(c));
        if (weighted) AS_TRY(fw[d].alloc(c));
        if (keep_col) AS_TRY(fcol[d].alloc(c));
        // payload chain: sorted position -> kept index (vs) -> staged entry (v1)
        if (c)
            emit_list<<<grid(c), kB, 0, s>>>(fkey[d].p, vs.p, c, b, v1[d].p, p_w, nullptr, fadj[d].p,
                                             weighted ? fw[d].p : nullptr, nullptr);
        if (keep_col && c) {
            ScopedBuf<uint32_t> staged;              // staged entry of every final entry
            AS_TRY(staged.alloc(c));
            gather_i32<<<grid(c), kB, 0, s>>>(vs.p, reinterpret_cast<const int32_t*>(v1[d].p), c,
                                              reinterpret_cast<int32_t*>(staged.p));
            gather_i32<<<grid(c), kB, 0, s>>>(staged.p, reinterpret_cast<const int32_t*>(col.p), c,
                                              reinterpret_cast<int32_t*>(fcol[d].p));
            AS_TRY(hipStreamSynchronize(s));
        }
        HostCsr& hc = *outc[d];
        AS_TRY(download(hc.off, foff[d].p, n + 1, s));
        if (weighted) {                              // weight_sorted_push reads the host lists
            AS_TRY(download(hc.adj, fadj[d].p, c, s));
            AS_TRY(download(hc.w, fw[d].p, c, s));
        }
        v1[d].release();
    }
    AS_TRY(download(g.perm, perm.p, n, s));
    // views: the push lists equal the stored opposite lists unless rows were cut or a
    // neighbour's opposite entry is missing (count check, graph_build.cpp finish_views)
    bool consistent = g.truncated == 0;
    if (consistent) {
        ScopedBuf<uint32_t> tc;
        ScopedBuf<int> bad;
        AS_TRY(tc.alloc(n)); AS_TRY(bad.alloc(1));
        AS_TRY(hipMemsetAsync(tc.p, 0, n * 4, s));
        AS_TRY(hipMemsetAsync(bad.p, 0, sizeof(int), s));
        if (cnt[0]) count_targets<<<grid(cnt[0]), kB, 0, s>>>(fadj[0].p, cnt[0], tc.p);
        count_mismatch<<<grid(n), kB, 0, s>>>(tc.p, foff[1].p, n, bad.p);
        int hb = 0;
        AS_TRY(hipMemcpyAsync(&hb, bad.p, sizeof(int), hipMemcpyDeviceToHost, s));
        AS_TRY(hipStreamSynchronize(s));
        consistent = hb == 0;
    }
    g.has_transpose = !consistent;
    if (!consistent) {
        // pull lists of the scope: inE = OUT rows, outE = IN rows, bothE = both (source order,
        // OUT before IN for one source: the host transpose_lists order)
        std::vector<int> lists = g.scope == TGO_SCOPE_IN_E ? std::vector<int>{0}
                               : g.scope == TGO_SCOPE_OUT_E ? std::vector<int>{1} : std::vector<int>{0, 1};
        int64_t c = 0;
        for (int d : lists) c += cnt[d];
        ScopedBuf<uint64_t> tk, ts;
        ScopedBuf<uint32_t> tv, tvs;
        ScopedBuf<int32_t> tw;
        AS_TRY(tk.alloc(c)); AS_TRY(ts.alloc(c)); AS_TRY(tv.alloc(c)); AS_TRY(tvs.alloc(c));
        if (weighted) AS_TRY(tw.alloc(c));
        int64_t at = 0;
        for (int d : lists) {
            if (cnt[d]) transpose_keys<<<grid(cnt[d]), kB, 0, s>>>(fkey[d].p, cnt[d], b, tk.p + at, tv.p + at);
            if (weighted && cnt[d])
                AS_TRY(hipMemcpyAsync(tw.p + at, fw[d].p, cnt[d] * 4, hipMemcpyDeviceToDevice, s));
            at += cnt[d];
        }
        if (lists.size() == 2 && cnt[0] && cnt[1])      // the second list's payloads index the concatenation
            shift_u32<<<grid(cnt[1]), kB, 0, s>>>(tv.p + cnt[0], cnt[1], static_cast<uint32_t>(cnt[0]));
        if (c) AS_TRY(so.pairs(tk.p, ts.p, tv.p, tvs.p, c, bits));
        ScopedBuf<int64_t> off;
        AS_TRY(off.alloc(n + 1));
        row_offsets<<<grid(n + 1), kB, 0, s>>>(ts.p, c, b, n, off.p);
        ScopedBuf<int32_t> adj, w;
        AS_TRY(adj.alloc(c));
        if (weighted) AS_TRY(w.alloc(c));
        if (c) emit_list<<<grid(c), kB, 0, s>>>(ts.p, tvs.p, c, b, nullptr, tw.p, nullptr, adj.p,
                                                weighted ? w.p : nullptr, nullptr);
        AS_TRY(download(g.push_t.off, off.p, n + 1, s));
        if (weighted) {
            AS_TRY(download(g.push_t.adj, adj.p, c, s));
            AS_TRY(download(g.push_t.w, w.p, c, s));
        }
        AS_TRY(hipStreamSynchronize(s));
        g.push_t.dadj.own(adj.take(), c);
        if (weighted) g.push_t.dw.own(w.take(), c);
    }
    AS_TRY(hipStreamSynchronize(s));
    for (int d = 0; d < 2; ++d) {                    // adopted by upload_graph
        outc[d]->dadj.own(fadj[d].take(), cnt[d]);
        if (weighted) outc[d]->dw.own(fw[d].take(), cnt[d]);
        if (keep_col) outc[d]->dcol.own(fcol[d].take(), cnt[d]);
    }
    st = RowStaging();
    return TGO_OK;
}

}  // namespace tgo

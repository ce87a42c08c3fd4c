// bfs.hip — frontier kernels for ShortestDistanceVertexProgram on gfx950.
//
// Reference semantics (ShortestDistanceVertexProgram.java:96-130 over Fulgora's pull
// gather, VertexMemoryHandler.java:77-103): at iteration i every vertex v takes the
// minimum over its reversed-scope neighbours w that SENT at iteration i-1 (double
// buffered, VertexState.java:55-89) of msg(w)+weight, and keeps it if strictly smaller.
// With unit weights this is level-synchronous BFS, exactly: a vertex first reached at
// iteration i has distance i and never improves.  The device executes only the frontier
// (the reference executes every vertex every superstep), in either direction:
//   top-down  : frontier vertices push over the transposed (push) view, edge-balanced
//               load-balanced search over the exclusive scan of frontier degrees;
//   bottom-up : every unvisited vertex pulls over its own list and stops at the first
//               neighbour in the frontier bitmap (one wave per 64-vertex bitmap word,
//               so visited/next bitmap words are written without atomics).
// Wave = 64 lanes; ballots are 64-bit.
#include <cstdlib>
#include <hip/hip_runtime.h>
#include <hipcub/hipcub.hpp>
#include "frontier.hpp"

namespace tgo {

namespace {

// bottom-up: longer lists are scanned by the whole wave.  256 (round 4; 32 before): single-
// source hmean over 8 RMAT-24 roots 277-280 GTEPS at 32, 240-245 at 16, 273-276 at 64, 300-314 at
// 128, 322-329 at 256, 316-320 at 512, 318-324 at 1024 (profiles/r04za_bfs_serial_ab.log) — a
// lane's own walk stops at its first frontier hit, the wave's walk pays a round trip per 64
constexpr int64_t kSerialScan = 256;

__global__ void fill_i32(int32_t* p, int32_t v, int64_t n) {
    for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) p[i] = v;
}
__global__ void fill_i64(int64_t* p, int64_t v, int64_t n) {
    for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) p[i] = v;
}

__global__ void bfs_seed(View push, int32_t* level, uint64_t* vb, uint64_t* fb, int32_t* q, int64_t* qdeg, int64_t seed) {
    if (threadIdx.x == 0 && blockIdx.x == 0) {
        level[seed] = 0;
        vb[seed >> 6] |= 1ULL << (seed & 63);
        fb[seed >> 6] |= 1ULL << (seed & 63);
        q[0] = static_cast<int32_t>(seed);
        qdeg[0] = push_degree(push, seed);
    }
}

// Top-down: load-balanced search over the exclusive scan qpre[0..qlen] of frontier degrees.
__global__ void __launch_bounds__(kBlock) td_expand(View push, const int32_t* __restrict__ q,
        const int64_t* __restrict__ qpre, int64_t qlen, int32_t* __restrict__ level,
        uint64_t* __restrict__ vb, uint64_t* __restrict__ nb, int32_t* __restrict__ qn,
        int64_t* __restrict__ qdeg_n, Counters* cnt, int32_t next_level) {
    __shared__ AppendLds sh;
    unsigned long long mf = 0;
    for_each_queue_edge(q, qpre, qlen, [&](bool valid, int32_t u, int64_t o) {
        bool take = false;
        int32_t v = 0;
        int64_t vdeg = 0;
        if (valid) {
            int32_t w;
            entry_at(push, u, o, v, w);
            const uint64_t bit = 1ULL << (v & 63);
            if (!(vb[v >> 6] & bit)) {
                const unsigned long long old = atomicOr(reinterpret_cast<unsigned long long*>(&vb[v >> 6]), bit);
                if (!(old & bit)) {
                    take = true;
                    level[v] = next_level;
                    atomicOr(reinterpret_cast<unsigned long long*>(&nb[v >> 6]), bit);
                    vdeg = push_degree(push, v);
                }
            }
        }
        block_append(take, v, vdeg, qn, qdeg_n, cnt, sh, mf);
    });
    block_flush(cnt, sh, mf);
}

// Bottom-up: one wave per 64-vertex bitmap word.  The next frontier is counted (vertices,
// push entries), not queued: bfs_queue builds the queue from nb when the next level is
// top-down.  No block barrier inside, so waves with long lists do not hold up the block.
template <int kS>
__global__ void __launch_bounds__(kBlock) bu_step(View pull, View push, int64_t n,
        const uint64_t* __restrict__ fb, uint64_t* __restrict__ vb, uint64_t* __restrict__ nb,
        int32_t* __restrict__ level, Counters* cnt, int32_t next_level, int64_t serial) {
    unsigned long long nv = 0, mf = 0;
    const int64_t words = (n + 63) >> 6;
    for (int64_t b = static_cast<int64_t>(blockIdx.x) * kWavesPerBlock; b < words;
         b += static_cast<int64_t>(gridDim.x) * kWavesPerBlock) {
        const int64_t wd = b + (threadIdx.x >> 6);
        const uint64_t vis = wd < words ? vb[wd] : ~0ULL;
        const int64_t v = (wd << 6) + lane();
        bool found = false;
        const bool open = v < n && !((vis >> lane()) & 1ULL);
        int64_t b0 = 0, e0 = 0, b1 = 0, e1 = 0;
        if (open) {
            b0 = pull.off0[v]; e0 = pull.off0[v + 1];
            if (pull.nlists > 1) { b1 = pull.off1[v]; e1 = pull.off1[v + 1]; }
        }
        const int64_t deg = (e0 - b0) + (e1 - b1);
        // short lists: the lane scans its own list and stops at the first frontier hit
        if (open && deg <= serial) {
            // kS entries per step: their index loads and bitmap probes issue together, so a
            // lane pays one dependent round trip per kS entries instead of per entry.  No branch
            // around a load (positions past the list re-read its last entry and are masked):
            // a conditional load per entry made the compiler wait for each probe in turn.
            for (int l = 0; l < 2 && !found; ++l) {
                const int32_t* adj = l == 0 ? pull.adj0 : pull.adj1;
                const int64_t e = l == 0 ? e0 : e1;
                for (int64_t k = l == 0 ? b0 : b1; k < e && !found; k += kS) {
                    int32_t u[kS];
#pragma unroll
                    for (int j = 0; j < kS; ++j) u[j] = adj[min(k + j, e - 1)];
                    uint64_t wv[kS];
#pragma unroll
                    for (int j = 0; j < kS; ++j) wv[j] = fb[u[j] >> 6];
                    uint64_t f = 0;
#pragma unroll
                    for (int j = 0; j < kS; ++j) f |= k + j < e ? wv[j] >> (u[j] & 63) : 0;
                    found = (f & 1ULL) != 0;
                }
            }
        }
        // long lists: the whole wave scans one list 64 entries at a time (ballot exit)
        unsigned long long big = __ballot(open && deg > serial);
        while (big) {
            const int src = __ffsll(static_cast<long long>(big)) - 1;
            big &= big - 1;
            bool hit = false;
            for (int l = 0; l < 2 && !hit; ++l) {
                const int64_t bb = __shfl(l == 0 ? b0 : b1, src, 64);
                const int64_t ee = __shfl(l == 0 ? e0 : e1, src, 64);
                const int32_t* adj = l == 0 ? pull.adj0 : pull.adj1;
                for (int64_t k = bb; k < ee; k += 64) {
                    bool h = false;
                    if (k + lane() < ee) {
                        const int32_t u = adj[k + lane()];
                        h = (fb[u >> 6] >> (u & 63)) & 1ULL;
                    }
                    if (__ballot(h)) { hit = true; break; }
                }
            }
            if (lane() == src) found = hit;
        }
        const unsigned long long fm = __ballot(found);
        if (lane() == 0 && wd < words) {
            nb[wd] = fm;
            if (fm) vb[wd] = vis | fm;
        }
        if (found) {
            level[v] = next_level;
            ++nv;
            mf += static_cast<unsigned long long>(push_degree(push, v));
        }
    }
    count_flush(cnt, nv, mf);
}

// Queue of the frontier bitmap fb (after a bottom-up level), push degrees for the scan.
__global__ void __launch_bounds__(kBlock) bfs_queue(View push, int64_t n, const uint64_t* __restrict__ fb,
        int32_t* __restrict__ qn, int64_t* __restrict__ qdeg, Counters* cnt) {
    const int64_t words = (n + 63) >> 6;
    auto probe = [&](int64_t wd, Take* t, bool) -> bool {
        const int64_t v = (wd << 6) + lane();
        const bool take = v < n && ((fb[wd] >> lane()) & 1ULL);
        t[0] = {take, static_cast<int32_t>(v), take ? push_degree(push, v) : 0};
        return __ballot(take) != 0;
    };
    chunk_extract_live<1>(words, [&](int64_t wd) { return fb[wd] != 0; }, probe, qn, qdeg, cnt);
}

// Partitioned levels with device-resident counts: {qlen, push entries} for the caller's
// all-reduce, and qlen for the ctx's own lazy read.
__global__ void publish_counts(const Counters* __restrict__ c, int64_t* __restrict__ out, int64_t* __restrict__ slot) {
    if (threadIdx.x == 0 && blockIdx.x == 0) {
        out[0] = static_cast<int64_t>(c->qlen);
        out[1] = static_cast<int64_t>(c->mf);
        slot[0] = static_cast<int64_t>(c->qlen);
    }
}

__global__ void level_to_dist(const int32_t* level, int64_t* dist, int64_t n) {
    for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
        const int32_t l = level[i];
        dist[i] = l >= 0 ? static_cast<int64_t>(l) : INT64_MIN;
    }
}

// reached vertices and their list entries (m_R) — for GTEPS / roofline accounting.
__global__ void reach_stats(View v, const int64_t* dist, int64_t n, unsigned long long* out2) {
    unsigned long long r = 0, m = 0;
    for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
        if (dist[i] != INT64_MIN) { ++r; m += static_cast<unsigned long long>(push_degree(v, i)); }
    }
    for (int off = 32; off > 0; off >>= 1) { r += __shfl_xor(r, off, 64); m += __shfl_xor(m, off, 64); }
    if (lane() == 0) { atomicAdd(&out2[0], r); atomicAdd(&out2[1], m); }
}

__global__ void degree_i64(View v, const int32_t* q, int64_t qlen, int64_t* qdeg) {
    for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < qlen; i += (int64_t)gridDim.x * blockDim.x)
        qdeg[i] = push_degree(v, q[i]);
}

// ---------------------------------------------------------------- SSSP (hop-bounded Jacobi)
__global__ void sssp_seed(View push, int64_t* dist, int64_t* msg, uint64_t* vb, int32_t* q, int64_t* qdeg, int64_t seed) {
    if (threadIdx.x == 0 && blockIdx.x == 0) {
        dist[seed] = 0;
        msg[seed] = 0;
        q[0] = static_cast<int32_t>(seed);
        qdeg[0] = push_degree(push, seed);
    }
}

// Relax every push edge of the frontier with the frontier's iteration-(i-1) message
// (msg is a snapshot, so the update is Jacobi exactly like the reference's double buffer).
__global__ void __launch_bounds__(kBlock) sssp_relax(View push, const int32_t* __restrict__ q,
        const int64_t* __restrict__ qpre, int64_t qlen, const int64_t* __restrict__ msg,
        int64_t* __restrict__ dist, uint64_t* __restrict__ mark, int32_t* __restrict__ qn,
        int64_t* __restrict__ qdeg_n, Counters* cnt, int weighted) {
    __shared__ AppendLds sh;
    unsigned long long mf = 0;
    for_each_queue_edge(q, qpre, qlen, [&](bool valid, int32_t u, int64_t o) {
        bool take = false;
        int32_t v = 0;
        int64_t vdeg = 0;
        if (valid) {
            int32_t w;
            entry_at(push, u, o, v, w);
            if (!weighted) w = 1;
            if (w == kMissingWeight) {
                atomicOr(&cnt->err, 1ULL);          // edge.value(weight) on a missing key
            } else {
                const int64_t cand = static_cast<int64_t>(static_cast<uint64_t>(msg[u]) + static_cast<uint64_t>(static_cast<int64_t>(w)));
                if (cand < dist[v]) {
                    const long long old = atomicMin(reinterpret_cast<long long*>(&dist[v]), static_cast<long long>(cand));
                    if (cand < old) {
                        const uint64_t bit = 1ULL << (v & 63);
                        const unsigned long long ob = atomicOr(reinterpret_cast<unsigned long long*>(&mark[v >> 6]), bit);
                        if (!(ob & bit)) { take = true; vdeg = push_degree(push, v); }
                    }
                }
            }
        }
        block_append(take, v, vdeg, qn, qdeg_n, cnt, sh, mf);
    });
    block_flush(cnt, sh, mf);
}

__global__ void sssp_commit(const int32_t* q, int64_t qlen, const int64_t* dist, int64_t* msg) {
    for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < qlen; i += (int64_t)gridDim.x * blockDim.x) {
        const int32_t v = q[i];
        msg[v] = dist[v];
    }
}

__global__ void dist_finalize(int64_t* dist, int64_t n) {
    for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x)
        if (dist[i] == INT64_MAX) dist[i] = INT64_MIN;
}

// ---------------------------------------------------------------- 1-D partitioned BFS
// Top-down on a partition: every entry of the local frontier marks its (global) neighbour
// in a global "discovered" bitmap; the owners claim them after the all-to-all of slices.
__global__ void __launch_bounds__(kBlock) part_td_mark(View push, const int32_t* __restrict__ q,
        const int64_t* __restrict__ qpre, int64_t qlen, uint64_t* __restrict__ disc,
        const uint64_t* __restrict__ vb_local, int64_t lo, int64_t n_local) {
    for_each_queue_edge(q, qpre, qlen, [&](bool valid, int32_t u, int64_t o) {
        if (!valid) return;
        int32_t v, w;
        entry_at(push, u, o, v, w);
        const uint64_t bit = 1ULL << (v & 63);
        const int64_t vl = static_cast<int64_t>(v) - lo;
        if (vl >= 0 && vl < n_local && (vb_local[vl >> 6] & (1ULL << (vl & 63)))) return;   // owned & visited
        if (!(disc[v >> 6] & bit)) atomicOr(reinterpret_cast<unsigned long long*>(&disc[v >> 6]), bit);
    });
}

// Top-down on a partition with the owned targets claimed in place (tgo_part_bfs_run): an owned
// neighbour joins the next frontier here, as in td_expand (visited bit, level, next-frontier bit,
// queue slot); only remote neighbours are marked in the discovered bitmap for their owners'
// part_claim<true>.  nb (the owned next-frontier slice) is zeroed by the caller.
__global__ void __launch_bounds__(kBlock) part_td_claim(View push, const int32_t* __restrict__ q,
        const int64_t* __restrict__ qpre, int64_t qlen, uint64_t* __restrict__ disc, uint64_t* __restrict__ vb,
        uint64_t* __restrict__ nb, int32_t* __restrict__ level, int32_t* __restrict__ qn, int64_t* __restrict__ qdeg_n,
        Counters* cnt, int32_t next_level, int64_t lo, int64_t n_local) {
    __shared__ AppendLds sh;
    unsigned long long mf = 0;
    for_each_queue_edge(q, qpre, qlen, [&](bool valid, int32_t u, int64_t o) {
        bool take = false;
        int32_t vt = 0;
        int64_t vdeg = 0;
        if (valid) {
            int32_t v, w;
            entry_at(push, u, o, v, w);
            const int64_t vl = static_cast<int64_t>(v) - lo;
            if (vl >= 0 && vl < n_local) {
                const uint64_t bit = 1ULL << (vl & 63);
                if (!(vb[vl >> 6] & bit)) {
                    const unsigned long long old = atomicOr(reinterpret_cast<unsigned long long*>(&vb[vl >> 6]), bit);
                    if (!(old & bit)) {
                        take = true;
                        vt = static_cast<int32_t>(vl);
                        level[vl] = next_level;
                        atomicOr(reinterpret_cast<unsigned long long*>(&nb[vl >> 6]), bit);
                        vdeg = push_degree(push, vt);
                    }
                }
            } else {
                const uint64_t bit = 1ULL << (v & 63);
                if (!(disc[v >> 6] & bit)) atomicOr(reinterpret_cast<unsigned long long*>(&disc[v >> 6]), bit);
            }
        }
        block_append(take, vt, vdeg, qn, qdeg_n, cnt, sh, mf);
    });
    block_flush(cnt, sh, mf);
}

// Owner side: OR the received slices, claim the unvisited bits (one wave per word; two-pass
// chunked extraction, frontier.hpp).  kOr (after part_td_claim): nb already holds the owned
// claims, so only words that take something are visited in pass 2 and OR-ed into nb;
// otherwise nb is written for every word.
template <bool kOr>
__global__ void __launch_bounds__(kBlock) part_claim(View push, const uint64_t* __restrict__ recv,
        int nslices, int64_t words, int64_t n_local, uint64_t* __restrict__ vb, uint64_t* __restrict__ nb,
        int32_t* __restrict__ level, int32_t* __restrict__ qn, int64_t* __restrict__ qdeg_n, Counters* cnt,
        int32_t next_level) {
    auto probe = [&](int64_t wd, Take* t, bool commit) -> bool {
        uint64_t bits = 0;
        for (int s = 0; s < nslices; ++s) bits |= recv[static_cast<int64_t>(s) * words + wd];
        const uint64_t vis = vb[wd];
        const uint64_t fresh = bits & ~vis;
        const int64_t v = (wd << 6) + lane();
        const bool take = v < n_local && ((fresh >> lane()) & 1ULL);
        const unsigned long long tm = __ballot(take);
        if (commit) {
            if (lane() == 0) {
                if (kOr) {
                    if (tm) nb[wd] |= tm;
                } else {
                    nb[wd] = tm;
                }
                if (tm) vb[wd] = vis | tm;
            }
            if (take) level[v] = next_level;
        }
        t[0] = {take, static_cast<int32_t>(v), take ? push_degree(push, v) : 0};
        return kOr ? tm != 0 : true;            // (!kOr) nb[wd] is written for every word
    };
    chunk_extract<1>(words, probe, qn, qdeg_n, cnt);
}

// out[v] = in[perm[v]]: internal (degree-grouped) order -> the API's row order.
template <class T>
__global__ void gather_perm(const T* __restrict__ in, const int32_t* __restrict__ perm, T* __restrict__ out, int64_t n) {
    for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x)
        out[i] = in[perm[i]];
}

inline int grid_for(int64_t work, int block = kBlock, int cap = 256 * 8) {
    int64_t g = (work + block - 1) / block;
    if (g < 1) g = 1;
    if (g > cap) g = cap;
    return static_cast<int>(g);
}

}  // namespace

// ---------------------------------------------------------------- launchers
hipError_t k_fill_i32(int32_t* p, int32_t v, int64_t n, hipStream_t s) {
    fill_i32<<<grid_for(n), kBlock, 0, s>>>(p, v, n);
    return hipGetLastError();
}
hipError_t k_fill_i64(int64_t* p, int64_t v, int64_t n, hipStream_t s) {
    fill_i64<<<grid_for(n), kBlock, 0, s>>>(p, v, n);
    return hipGetLastError();
}
hipError_t k_bfs_seed(const View& push, int32_t* level, uint64_t* vb, uint64_t* fb, int32_t* q,
                      int64_t* qdeg, int64_t seed, hipStream_t s) {
    bfs_seed<<<1, 64, 0, s>>>(push, level, vb, fb, q, qdeg, seed);
    return hipGetLastError();
}
hipError_t k_td_expand(const View& push, const int32_t* q, const int64_t* qpre, int64_t qlen,
                       int32_t* level, uint64_t* vb, uint64_t* nb, int32_t* qn, int64_t* qdeg_n,
                       Counters* cnt, int32_t next_level, hipStream_t s) {
    td_expand<<<256 * 8, kBlock, 0, s>>>(push, q, qpre, qlen, level, vb, nb, qn, qdeg_n, cnt, next_level);
    return hipGetLastError();
}
hipError_t k_bu_step(const View& pull, const View& push, int64_t n, const uint64_t* fb, uint64_t* vb, uint64_t* nb,
                     int32_t* level, Counters* cnt, int32_t next_level, hipStream_t s) {
    // one wave per bitmap word in a grid-stride loop: a wave's dependent probe chain overlaps
    // with thousands of others.
    const int64_t words = (n + 63) / 64;
    // TGO_BFS_SERIAL: lists up to this many entries are scanned by their own lane (kSerialScan default)
    static const int64_t serial = [] { const char* e = std::getenv("TGO_BFS_SERIAL"); return e ? std::atoll(e) : kSerialScan; }();
    // TGO_BFS_BU_STEP (A/B): entries per dependent round trip of a lane's own list — 2 since the
    // trips are branch-free (round 6, RMAT-24 16 roots, one box: 4 -> 2 hmean 360 -> 374 GTEPS,
    // 8: 313; a second box: 2 371, 4 374, 1 363 — 2 and 4 within noise there;
    // profiles/r06bu_bfs_bu_step_ab.log)
    static const int bs = [] { const char* e = std::getenv("TGO_BFS_BU_STEP"); return e ? std::atoi(e) : 2; }();
    // 2048 blocks (8192 waves: one resident round at 8 waves per SIMD), each wave walking 32
    // words at RMAT-24: hmean 326-331 -> 368-371 GTEPS over the 64 bench roots against 8192
    // blocks (4096: 346-360, 1024: 327, 16384: 276-279; profiles/r05bg_bfs_bu_grid_ab.log).
    // (The multi-source pull, same one-wave-per-word shape at 7 waves per SIMD, is best at 8192:
    // 3.66-3.68 ms per sweep against 4.14 at 2048 and 4.43-4.53 at its resident 1792.)
    const int g = grid_for(words * 64, kBlock, 2048);
    if (bs == 8)
        bu_step<8><<<g, kBlock, 0, s>>>(pull, push, n, fb, vb, nb, level, cnt, next_level, serial);
    else if (bs == 4)
        bu_step<4><<<g, kBlock, 0, s>>>(pull, push, n, fb, vb, nb, level, cnt, next_level, serial);
    else if (bs == 1)
        bu_step<1><<<g, kBlock, 0, s>>>(pull, push, n, fb, vb, nb, level, cnt, next_level, serial);
    else
        bu_step<2><<<g, kBlock, 0, s>>>(pull, push, n, fb, vb, nb, level, cnt, next_level, serial);
    return hipGetLastError();
}
hipError_t k_bfs_queue(const View& push, int64_t n, const uint64_t* fb, int32_t* qn, int64_t* qdeg, Counters* cnt,
                       hipStream_t s) {
    bfs_queue<<<extract_grid((n + 63) / 64), kBlock, 0, s>>>(push, n, fb, qn, qdeg, cnt);
    return hipGetLastError();
}
__global__ void publish_counters(const Counters* c, unsigned long long* host, unsigned long long seq) {
    const int i = threadIdx.x;
    const unsigned long long* w = reinterpret_cast<const unsigned long long*>(c);
    if (i < kCounterWords) {
        __hip_atomic_store(&host[i], w[i], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        __threadfence_system();
    }
    __syncthreads();
    if (i == 0) __hip_atomic_store(&host[kCounterWords], seq, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
}
// publish_counters for `count` arbitrary device words (the partitioned drivers' counts).
__global__ void publish_words(const unsigned long long* src, int count, unsigned long long* host, unsigned long long seq) {
    const int i = threadIdx.x;
    if (i < count) {
        __hip_atomic_store(&host[i], src[i], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        __threadfence_system();
    }
    __syncthreads();
    if (i == 0) __hip_atomic_store(&host[kCounterWords], seq, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
}
// Grid-stride: the launch grid is capped (grid_for: 2048 blocks = 524 288 threads), and RMAT-27
// has 2.1 M bitmap words — a one-thread-per-word form left the tail of nb uncleared there.
__global__ void level_prep(Counters* cnt, uint64_t* nb, int64_t words, int64_t* tail) {
    const int64_t i0 = static_cast<int64_t>(blockIdx.x) * blockDim.x + threadIdx.x;
    for (int64_t i = i0; i < words; i += static_cast<int64_t>(gridDim.x) * blockDim.x) nb[i] = 0;
    if (cnt && i0 < kCounterWords) reinterpret_cast<unsigned long long*>(cnt)[i0] = 0;
    if (tail && i0 == 0) *tail = 0;
}
// The end of a one-GPU BFS level in one launch (publish_counters + the next level's
// level_prep): block 0 publishes the counters to the host-mapped page, then zeroes them and the
// scan tail qdeg[qlen] at the new queue length; every block clears `clear` (the frontier bitmap
// the level just consumed, the next level's nb after the swap).  One dispatch fewer per level.
__global__ void level_turn(Counters* c, unsigned long long* host, unsigned long long seq, uint64_t* __restrict__ clear,
                           int64_t words, int64_t* __restrict__ qdeg) {
    const int64_t i0 = static_cast<int64_t>(blockIdx.x) * blockDim.x + threadIdx.x;
    for (int64_t i = i0; i < words; i += static_cast<int64_t>(gridDim.x) * blockDim.x) clear[i] = 0;
    if (blockIdx.x != 0) return;
    const int i = threadIdx.x;
    unsigned long long* w = reinterpret_cast<unsigned long long*>(c);
    const unsigned long long qlen = c->qlen;
    if (i < kCounterWords) {
        __hip_atomic_store(&host[i], w[i], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        __threadfence_system();
    }
    __syncthreads();                          // every word read before any is zeroed
    if (i == 0) {
        qdeg[qlen] = 0;
        __hip_atomic_store(&host[kCounterWords], seq, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
    }
    if (i < kCounterWords) w[i] = 0;
}
hipError_t k_level_turn(Counters* c, unsigned long long* host, unsigned long long seq, uint64_t* clear, int64_t words,
                        int64_t* qdeg, hipStream_t s) {
    if (kBlock < kCounterWords) return hipErrorInvalidValue;
    level_turn<<<grid_for(std::max<int64_t>(words, kCounterWords)), kBlock, 0, s>>>(c, host, seq, clear, words, qdeg);
    return hipGetLastError();
}
hipError_t k_publish_counters(const Counters* c, unsigned long long* host, unsigned long long seq, hipStream_t s) {
    publish_counters<<<1, 64, 0, s>>>(c, host, seq);
    return hipGetLastError();
}
hipError_t k_publish_words(const int64_t* src, int count, unsigned long long* host, unsigned long long seq, hipStream_t s) {
    if (count < 0 || count > kCounterWords) return hipErrorInvalidValue;
    publish_words<<<1, 64, 0, s>>>(reinterpret_cast<const unsigned long long*>(src), count, host, seq);
    return hipGetLastError();
}
hipError_t k_level_prep(Counters* cnt, uint64_t* nb, int64_t words, int64_t* tail, hipStream_t s) {
    const int64_t n = std::max<int64_t>(words, kCounterWords);
    level_prep<<<grid_for(n), kBlock, 0, s>>>(cnt, nb, words, tail);
    return hipGetLastError();
}
hipError_t k_publish_counts(const Counters* c, int64_t* out, int64_t* slot, hipStream_t s) {
    publish_counts<<<1, 64, 0, s>>>(c, out, slot);
    return hipGetLastError();
}
hipError_t k_level_to_dist(const int32_t* level, int64_t* dist, int64_t n, hipStream_t s) {
    level_to_dist<<<grid_for(n), kBlock, 0, s>>>(level, dist, n);
    return hipGetLastError();
}
hipError_t k_reach_stats(const View& v, const int64_t* dist, int64_t n, unsigned long long* out2, hipStream_t s) {
    reach_stats<<<grid_for(n), kBlock, 0, s>>>(v, dist, n, out2);
    return hipGetLastError();
}
hipError_t k_degree_i64(const View& v, const int32_t* q, int64_t qlen, int64_t* qdeg, hipStream_t s) {
    degree_i64<<<grid_for(qlen), kBlock, 0, s>>>(v, q, qlen, qdeg);
    return hipGetLastError();
}
hipError_t k_sssp_seed(const View& push, int64_t* dist, int64_t* msg, uint64_t* vb, int32_t* q,
                       int64_t* qdeg, int64_t seed, hipStream_t s) {
    sssp_seed<<<1, 64, 0, s>>>(push, dist, msg, vb, q, qdeg, seed);
    return hipGetLastError();
}
hipError_t k_sssp_relax(const View& push, const int32_t* q, const int64_t* qpre, int64_t qlen,
                        const int64_t* msg, int64_t* dist, uint64_t* mark, int32_t* qn,
                        int64_t* qdeg_n, Counters* cnt, int weighted, hipStream_t s) {
    sssp_relax<<<256 * 8, kBlock, 0, s>>>(push, q, qpre, qlen, msg, dist, mark, qn, qdeg_n, cnt, weighted);
    return hipGetLastError();
}
hipError_t k_sssp_commit(const int32_t* q, int64_t qlen, const int64_t* dist, int64_t* msg,
                         uint64_t* mark, hipStream_t s) {
    (void)mark;
    sssp_commit<<<grid_for(qlen), kBlock, 0, s>>>(q, qlen, dist, msg);
    return hipGetLastError();
}
hipError_t k_part_td_mark(const View& push, const int32_t* q, const int64_t* qpre, int64_t qlen,
                          uint64_t* disc, const uint64_t* vb_local, int64_t lo, int64_t n_local, hipStream_t s) {
    part_td_mark<<<256 * 8, kBlock, 0, s>>>(push, q, qpre, qlen, disc, vb_local, lo, n_local);
    return hipGetLastError();
}
hipError_t k_part_claim(const View& push, const uint64_t* recv, int nslices, int64_t words, int64_t n_local,
                        uint64_t* vb, uint64_t* nb, int32_t* level, int32_t* qn, int64_t* qdeg_n,
                        Counters* cnt, int32_t next_level, hipStream_t s, bool or_into_nb) {
    if (or_into_nb)
        part_claim<true><<<extract_grid(words), kBlock, 0, s>>>(push, recv, nslices, words, n_local, vb, nb, level, qn,
                                                                qdeg_n, cnt, next_level);
    else
        part_claim<false><<<extract_grid(words), kBlock, 0, s>>>(push, recv, nslices, words, n_local, vb, nb, level, qn,
                                                                 qdeg_n, cnt, next_level);
    return hipGetLastError();
}
hipError_t k_part_td_claim(const View& push, const int32_t* q, const int64_t* qpre, int64_t qlen, uint64_t* disc,
                           uint64_t* vb, uint64_t* nb, int32_t* level, int32_t* qn, int64_t* qdeg_n, Counters* cnt,
                           int32_t next_level, int64_t lo, int64_t n_local, hipStream_t s) {
    part_td_claim<<<256 * 8, kBlock, 0, s>>>(push, q, qpre, qlen, disc, vb, nb, level, qn, qdeg_n, cnt, next_level, lo,
                                             n_local);
    return hipGetLastError();
}
hipError_t k_unpermute_i64(const int64_t* in, const int32_t* perm, int64_t* out, int64_t n, hipStream_t s) {
    gather_perm<int64_t><<<grid_for(n), kBlock, 0, s>>>(in, perm, out, n);
    return hipGetLastError();
}
hipError_t k_unpermute_i32(const int32_t* in, const int32_t* perm, int32_t* out, int64_t n, hipStream_t s) {
    gather_perm<int32_t><<<grid_for(n), kBlock, 0, s>>>(in, perm, out, n);
    return hipGetLastError();
}
hipError_t k_dist_finalize(int64_t* dist, int64_t n, hipStream_t s) {
    dist_finalize<<<grid_for(n), kBlock, 0, s>>>(dist, n);
    return hipGetLastError();
}

hipError_t scan_exclusive_i64(void*& tmp, size_t& tmp_bytes, const int64_t* in, int64_t* out,
                              int64_t n, hipStream_t s) {
    size_t need = 0;
    hipError_t e = hipcub::DeviceScan::ExclusiveSum(nullptr, need, in, out, static_cast<int>(n), s);
    if (e != hipSuccess) return e;
    if (need > tmp_bytes) {
        if (tmp) (void)hipFree(tmp);
        tmp = nullptr;
        e = hipMalloc(&tmp, need);
        if (e != hipSuccess) { tmp_bytes = 0; return e; }
        tmp_bytes = need;
    }
    return hipcub::DeviceScan::ExclusiveSum(tmp, tmp_bytes, in, out, static_cast<int>(n), s);
}

}  // namespace tgo

// msbfs.hip — multi-source BFS: up to 64 ShortestDistanceVertexProgram runs with unit
// weights executed together (bit-parallel frontiers; Then et al., "The More the Merrier",
// VLDB 2014).
//
// Per vertex v a 64-bit mask holds one bit per source: vis[v] (reached), fr[v] (reached at
// the current level), nx[v] (reached at the next level).  A level of all sources is
//   pull : nx[v] = (OR over v's reversed-scope neighbours u of fr[u]) & ~vis[v]
//   push : for every frontier vertex u and push-neighbour v: atomicOr(nx[v], fr[u])
// so one pass over the adjacency serves every source whose frontier touches it — the
// adjacency is read once per level instead of once per level per source.  Each source's
// result is identical to its own single-source run (Jacobi: fr is the previous level's
// snapshot).  Levels are stored as bit planes (engine.hpp LevelPlanes): discovering the
// sources `fresh` of v at level L ORs `fresh` into plane k of v for every set bit k of L —
// at most log2(L)+1 coalesced 8-byte writes per vertex and level, and planes are zeroed
// only when the sweep first reaches level 2^k.
#include <cstdlib>
#include <hip/hip_runtime.h>
#include "frontier.hpp"

namespace tgo {
namespace {

constexpr int kMaxSources = 64;

__device__ __forceinline__ int32_t view_entry(const View& v, int64_t u, int64_t o) {
    const int64_t b0 = v.off0[u];
    const int64_t d0 = v.off0[u + 1] - b0;
    return o < d0 ? v.adj0[b0 + o] : v.adj1[v.off1[u] + (o - d0)];
}

// Record the level of every newly reached source of v: bit k of the level goes into plane k,
// one coalesced 8-byte OR per set level bit (the lane owns v).
__device__ __forceinline__ void record_level(int64_t v, uint64_t fresh, int32_t level, const LevelPlanes& pl) {
    for (int k = 0; k < kLevelPlanes && (level >> k); ++k)
        if ((level >> k) & 1) pl.p[k * pl.stride + v] |= fresh;
}

// End of a counting kernel: per-thread sums of the next frontier (vertices, their push
// entries, source bits) reduced over the block, one atomicAdd per block and counter.  No
// per-word block barrier: a pull level's waves finish their words independently (lists are
// skewed; a barrier per word made every wave wait for the block's longest list).
__device__ __forceinline__ void count_flush(Counters* cnt, unsigned long long nv, unsigned long long mf,
                                            unsigned long long bits) {
    __shared__ unsigned long long s_nv[kWavesPerBlock], s_mf[kWavesPerBlock], s_bits[kWavesPerBlock];
    for (int off = 32; off > 0; off >>= 1) {
        nv += __shfl_xor(nv, off, 64);
        mf += __shfl_xor(mf, off, 64);
        bits += __shfl_xor(bits, off, 64);
    }
    if (lane() == 0) { s_nv[threadIdx.x >> 6] = nv; s_mf[threadIdx.x >> 6] = mf; s_bits[threadIdx.x >> 6] = bits; }
    __syncthreads();
    if (threadIdx.x == 0) {
        unsigned long long a = 0, m = 0, c = 0;
        for (int w = 0; w < kWavesPerBlock; ++w) { a += s_nv[w]; m += s_mf[w]; c += s_bits[w]; }
        if (a) atomicAdd(&cnt->qlen, a);
        if (m) atomicAdd(&cnt->mf, m);
        if (c) atomicAdd(&cnt->red[0], c);
    }
}

// fr_rows: seeds at rows >= fr_rows (entry-less rows of a partitioned layout) are reached
// but left out of the frontier mask — they have no entries to push or be pulled through,
// and keeping them out leaves the masks' entry-less tail zero for the whole sweep.
// One lane per seed (a single thread's 64 dependent read-modify-writes took 37 us).
__global__ void ms_seed(const int64_t* __restrict__ seeds, int nseeds, uint64_t* vis, uint64_t* fr, int64_t fr_rows) {
    const int r = static_cast<int>(threadIdx.x);
    if (blockIdx.x != 0 || r >= nseeds) return;
    const int64_t s = seeds[r];
    if (s < 0) return;                           // partitioned: seed owned by another rank
    atomicOr(reinterpret_cast<unsigned long long*>(&vis[s]), 1ULL << r);
    if (s < fr_rows) atomicOr(reinterpret_cast<unsigned long long*>(&fr[s]), 1ULL << r);
}

// Pull level over the active vertices: OR the neighbours' frontier masks, stop as soon as
// every still-unreached source of v is covered.  One vertex per lane; lists longer than
// kCoop are OR-reduced by the whole wave.
constexpr int64_t kCoop = 64;
// fbm (optional): bit u set iff fr[u] != 0.  The 2 MB bitmap stays in every XCD's L2, so a
// neighbour outside every source's frontier costs an L2 probe instead of an 8-byte mask
// gather from the 134 MB mask array (mostly cold, low-degree vertices: the misses).
__device__ __forceinline__ bool in_frontier(const uint64_t* __restrict__ fbm, int32_t u) {
    return !fbm || ((fbm[u >> 6] >> (u & 63)) & 1ULL);
}
// The filter only for neighbours u >= from (the cold ids): hot neighbours' masks sit in L2 and
// are mostly frontier members at the dense levels, so probing the bitmap first only adds a
// dependent load there; a cold neighbour outside every frontier costs an L2 probe instead of
// an Infinity-Cache / HBM gather (at RMAT-24's first pull level ~88 % of them).
__device__ __forceinline__ bool maybe_frontier(const uint64_t* __restrict__ fbm, int32_t u, int32_t from) {
    return u < from || in_frontier(fbm, u);
}
// Diagnostic tallies of a pull level (TGO_MS_DIAG=1 with TGO_TRACE=1; off in the product):
// [0] list entries examined, [1] mask gathers of hot neighbours (u < kDiagHot), [2] of cold
// ones, [3] open vertices, [4] open vertices whose walk stopped early (every open source covered);
// long lists (wave-cooperative): [5] entries examined, [6] lists, [7] lists that stopped early,
// [8] / [9] their hot / cold mask gathers
constexpr int32_t kDiagHot = 393216;
constexpr int kDiagWords = 10;
__device__ unsigned long long g_ms_diag[kDiagWords];
// kStep: entries per dependent round trip of a lane's own list; kLong: entries per lane per
// trip of a wave-cooperative long list (kLong * 64 per trip)
// cs (MsColdSplit, hot_lim < INT32_MAX): the walk reads only neighbours < hot_lim (lists are
// sorted, so it stops at the first cold one); a row it does not cover whose lists go on past
// hot_lim is left to the blocked cold pass: its partial mask to cs.acc, cs.need set, nothing
// written (ms_cold ORs its cold neighbours in, ms_finish settles it).
// kRamp: a long list's first trip reads 64 entries only (its head of hubs often covers every
// open source), the later ones kLong * 64.
template <int kStep, bool kDiag = false, int kLong = 4, bool kRamp = false>
__global__ void __launch_bounds__(kBlock) ms_pull(View pull, View push, int64_t n_active, uint64_t full,
        const uint64_t* __restrict__ fr, const uint64_t* __restrict__ fbm, uint64_t* __restrict__ vis,
        uint64_t* __restrict__ nx, LevelPlanes lvl, Counters* cnt, int32_t next_level, int32_t filter_from,
        uint64_t dense, const uint64_t* __restrict__ cand, MsColdSplit cs, int64_t coop) {
    const int32_t hot_lim = cs.hot_lim;
    unsigned long long nv = 0, mf = 0, bits = 0;
    unsigned long long dg[kDiagWords] = {0, 0, 0, 0, 0, 0, 0, 0, 0, 0};
    const int64_t words = (n_active + 63) >> 6;
    // wave w of the block takes word b + w; words past the end run as all-closed lanes.  No
    // block barrier inside: the next frontier is only counted here (ms_queue builds its queue
    // if the next level pushes)
    for (int64_t b = static_cast<int64_t>(blockIdx.x) * kWavesPerBlock; b < words; b += static_cast<int64_t>(gridDim.x) * kWavesPerBlock) {
        const int64_t wd = b + (threadIdx.x >> 6);
        const int64_t v = (wd << 6) + lane();
        const uint64_t seen = v < n_active ? vis[v] : full;
        const uint64_t open = full & ~seen;
        // the walk only has to cover the dense sources; the sparse ones come from the push
        // candidates (cand, exact over every entry of their frontiers)
        const uint64_t want = open & dense;
        int64_t b0 = 0, e0 = 0, b1 = 0, e1 = 0;
        if (open) {
            b0 = pull.off0[v]; e0 = pull.off0[v + 1];
            if (pull.nlists > 1) { b1 = pull.off1[v]; e1 = pull.off1[v + 1]; }
        }
        const int64_t deg = (e0 - b0) + (e1 - b1);
        uint64_t acc = 0;
        bool cut = false;                                     // a list went on past hot_lim
        if (want && deg <= coop) {
            for (int l = 0; l < 2 && (acc & want) != want; ++l) {
                const int32_t* adj = l == 0 ? pull.adj0 : pull.adj1;
                const int64_t e = l == 0 ? e0 : e1;
                bool cutl = false;
                // kStep entries per dependent round trip: their index loads issue together,
                // then their bitmap probes, then their mask gathers (lists rarely cover every
                // open source early).  No branch inside a trip: positions past the list re-read
                // its last entry, a filtered entry gathers mask 0's line (one L1 line for the
                // wave) and drops it — a conditional load per entry made the compiler wait for
                // every outstanding load before the next, one load in flight per lane
                for (int64_t k = l == 0 ? b0 : b1; k < e && (acc & want) != want && !cutl; k += kStep) {
                    int32_t u[kStep];
                    bool ok[kStep], f[kStep];
#pragma unroll
                    for (int j = 0; j < kStep; ++j) {
                        u[j] = __builtin_nontemporal_load(adj + min(k + j, e - 1));
                        const bool in = k + j < e;
                        cutl |= in && u[j] >= hot_lim;
                        ok[j] = in && u[j] < hot_lim;
                        f[j] = ok[j];
                    }
                    if (fbm) {                                        // kernel-uniform
                        uint64_t bw[kStep];
#pragma unroll
                        for (int j = 0; j < kStep; ++j) bw[j] = fbm[(f[j] && u[j] >= filter_from ? u[j] : 0) >> 6];
#pragma unroll
                        for (int j = 0; j < kStep; ++j)
                            f[j] = f[j] && (u[j] < filter_from || ((bw[j] >> (u[j] & 63)) & 1ULL));
                    }
                    uint64_t mk[kStep];
#pragma unroll
                    for (int j = 0; j < kStep; ++j) mk[j] = fr[f[j] ? u[j] : 0];
                    uint64_t m = 0;
#pragma unroll
                    for (int j = 0; j < kStep; ++j) m |= f[j] ? mk[j] : 0ULL;
                    acc |= m;
                    if (kDiag)
                        for (int j = 0; j < kStep; ++j)
                            if (ok[j]) { ++dg[0]; ++dg[u[j] < kDiagHot ? 1 : 2]; }
                }
                cut |= cutl;
            }
            if (kDiag) { ++dg[3]; if ((acc & want) == want) ++dg[4]; }
        }
        unsigned long long big = __ballot(want != 0 && deg > coop);
        while (big) {
            const int src = __ffsll(static_cast<long long>(big)) - 1;
            big &= big - 1;
            const uint64_t wsrc = __shfl(want, src, 64);
            uint64_t a = 0;
            bool wcut = false;                                // wave-uniform
            for (int l = 0; l < 2; ++l) {
                const int64_t bb = __shfl(l == 0 ? b0 : b1, src, 64);
                const int64_t ee = __shfl(l == 0 ? e0 : e1, src, 64);
                const int32_t* adj = l == 0 ? pull.adj0 : pull.adj1;
                bool done = false;
                bool first = kRamp && l == 0;
                for (int64_t k = bb; k < ee && !done;) {
                    const int jl = first ? 1 : kLong;                 // wave-uniform
                    int32_t u[kLong];
                    bool hc = false;
#pragma unroll
                    for (int j = 0; j < kLong; ++j) {
                        const int64_t x = k + j * 64 + lane();
                        u[j] = (j < jl && x < ee) ? __builtin_nontemporal_load(adj + x) : -1;
                        if (u[j] >= hot_lim) { u[j] = -1; hc = true; }
                    }
                    k += static_cast<int64_t>(jl) * 64;
                    first = false;
                    if (__ballot(hc)) { done = true; wcut = true; }   // the rest of the list is cold
                    bool f[kLong];
#pragma unroll
                    for (int j = 0; j < kLong; ++j) f[j] = u[j] >= 0 && maybe_frontier(fbm, u[j], filter_from);
                    uint64_t m = 0;
#pragma unroll
                    for (int j = 0; j < kLong; ++j)
                        if (f[j]) m |= fr[u[j]];
                    for (int off = 32; off > 0; off >>= 1) m |= __shfl_xor(m, off, 64);
                    if (kDiag)
                        for (int j = 0; j < kLong; ++j)
                            if (u[j] >= 0) ++dg[u[j] < kDiagHot ? 8 : 9];
                    a |= m;
                    done = done || (a & wsrc) == wsrc;
                    if (kDiag && lane() == src)
                        for (int j = 0; j < kLong; ++j) dg[5] += u[j] >= 0 ? 1 : 0;
                }
                if ((a & wsrc) == wsrc) break;
            }
            if (lane() == src) {
                acc = a;
                cut = wcut;
                if (kDiag) { ++dg[6]; if ((a & wsrc) == wsrc) ++dg[7]; }
            }
        }
        if (cut && (acc & want) != want && v < n_active) {   // left to the cold pass
            cs.acc[v] = acc;
            cs.need[v] = 1;
            continue;
        }
        if (cand && open && v < n_active) acc |= cand[v];
        const uint64_t fresh = acc & open;
        if (v < n_active) {
            nx[v] = fresh;
            if (fresh) vis[v] = seen | fresh;
        }
        if (fresh) {
            record_level(v, fresh, next_level, lvl);
            ++nv;
            mf += static_cast<unsigned long long>(push_degree(push, v));
            bits += static_cast<unsigned long long>(__popcll(fresh));
        }
    }
    if (kDiag) {
        for (int i = 0; i < kDiagWords; ++i) {
            unsigned long long x = dg[i];
            for (int off = 32; off > 0; off >>= 1) x += __shfl_xor(x, off, 64);
            if (lane() == 0 && x) atomicAdd(&g_ms_diag[i], x);
        }
    }
    count_flush(cnt, nv, mf, bits);
}

// Blocked cold pass of a split pull level: the cold entries (neighbour >= hot_lim) of every row,
// sorted by (segment of the neighbour, row), the XCD-major way: XCD x walks the x-th eighth of
// the entries in order with its blocks as one grid-stride window, so the segment of masks it
// reads (3 MB) stays in its L2.  A row the hot walk left open ORs its cold neighbours' masks:
// a wave reduces each run of one row (the entries are row-contiguous inside a segment) and the
// run's first lane ORs the result into cs.acc.
__global__ void __launch_bounds__(kBlock) ms_cold(const int32_t* __restrict__ cadj, const int32_t* __restrict__ crow,
        int64_t C, const uint64_t* __restrict__ fr, const uint8_t* __restrict__ need, uint64_t* __restrict__ acc) {
    const int x = static_cast<int>(blockIdx.x & 7u);
    const int64_t per = gridDim.x >> 3;                      // blocks per XCD (grid is a multiple of 8)
    const int64_t lo = C * x / 8, hi = C * (x + 1) / 8;
    const int64_t span = (hi - lo + 63) & ~int64_t(63);
    for (int64_t e0 = lo + static_cast<int64_t>(blockIdx.x >> 3) * kBlock; e0 < lo + span; e0 += per * kBlock) {
        const int64_t e = e0 + threadIdx.x;                   // wave-uniform trips (kBlock = 4 waves)
        int32_t v = -1;
        uint64_t m = 0;
        if (e < hi) {
            v = crow[e];
            if (need[v]) m = fr[cadj[e]];
        }
        // OR of the run of v from this lane on (rows are contiguous, so lane + o shares v only
        // if every lane between does)
        for (int o = 1; o < 64; o <<= 1) {
            const uint64_t y = __shfl_down(m, o, 64);
            const int32_t w = __shfl_down(v, o, 64);
            if (lane() + o < 64 && w == v) m |= y;
        }
        const int32_t prev = __shfl_up(v, 1, 64);
        if (v >= 0 && m && (lane() == 0 || prev != v)) atomicOr(reinterpret_cast<unsigned long long*>(&acc[v]), m);
    }
}

// The rows the cold pass completed: their mask (hot walk | cold pass | the split's push
// candidates) settled like the pull's own rows, counted into the same counters.
__global__ void __launch_bounds__(kBlock) ms_finish(View push, int64_t n_active, uint64_t full,
        uint64_t* __restrict__ vis, uint64_t* __restrict__ nx, const uint64_t* __restrict__ cand, LevelPlanes lvl,
        Counters* cnt, int32_t next_level, uint8_t* __restrict__ need, const uint64_t* __restrict__ acc) {
    unsigned long long nv = 0, mf = 0, bits = 0;
    for (int64_t v = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; v < n_active; v += (int64_t)gridDim.x * blockDim.x) {
        if (!need[v]) continue;
        need[v] = 0;
        const uint64_t seen = vis[v];
        uint64_t a = acc[v];
        if (cand) a |= cand[v];
        const uint64_t fresh = a & full & ~seen;
        nx[v] = fresh;
        if (fresh) {
            vis[v] = seen | fresh;
            record_level(v, fresh, next_level, lvl);
            ++nv;
            mf += static_cast<unsigned long long>(push_degree(push, v));
            bits += static_cast<unsigned long long>(__popcll(fresh));
        }
    }
    count_flush(cnt, nv, mf, bits);
}

// Cold layout build: flags / positions of the entries >= hot of one list, then the (segment,
// row) keys and neighbour payloads at their compacted positions.
__global__ void cold_flags(const int32_t* __restrict__ adj, int64_t m, int32_t hot, uint32_t* __restrict__ flag) {
    for (int64_t k = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; k < m; k += (int64_t)gridDim.x * blockDim.x)
        flag[k] = adj[k] >= hot ? 1u : 0u;
}
__global__ void cold_emit(const int64_t* __restrict__ off, int64_t n, const int32_t* __restrict__ adj, int64_t m,
                          const uint32_t* __restrict__ flag, const uint64_t* __restrict__ pos, int64_t base, int32_t hot,
                          int64_t seg, uint64_t* __restrict__ key, int32_t* __restrict__ val) {
    for (int64_t k = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; k < m; k += (int64_t)gridDim.x * blockDim.x) {
        if (!flag[k]) continue;
        int64_t a = 0, b = n;                                 // row: last r with off[r] <= k
        while (b - a > 1) { const int64_t c = (a + b) >> 1; if (off[c] <= k) a = c; else b = c; }
        const int64_t p = base + static_cast<int64_t>(pos[k]);
        const uint64_t sg = static_cast<uint64_t>((adj[k] - hot) / seg);
        key[p] = (sg << 32) | static_cast<uint64_t>(a);
        val[p] = adj[k];
    }
}
__global__ void low_rows(const uint64_t* __restrict__ key, int64_t m, int32_t* __restrict__ row) {
    for (int64_t k = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; k < m; k += (int64_t)gridDim.x * blockDim.x)
        row[k] = static_cast<int32_t>(static_cast<uint32_t>(key[k]));
}

// Per-source frontier sizes of a pull level (vertices whose mask holds the source's bit):
// one wave per 64-vertex word, one coalesced mask load, then a 64 x 64 bit transpose across
// the lanes (6 shuffle stages swapping off-diagonal blocks) so lane b holds source b's column
// and adds its popcount.  One atomicAdd per lane and block.
__global__ void __launch_bounds__(kBlock) ms_source_counts(const uint64_t* __restrict__ fr, int64_t n_active,
                                                           unsigned long long* __restrict__ out) {
    __shared__ unsigned long long s_sum[kWavesPerBlock][64];
    const int64_t words = (n_active + 63) >> 6;
    unsigned long long sum = 0;
    const int64_t nw = (static_cast<int64_t>(gridDim.x) * blockDim.x) >> 6;
    for (int64_t w0 = (static_cast<int64_t>(blockIdx.x) * blockDim.x + threadIdx.x) >> 6; w0 < words; w0 += 4 * nw) {
      uint64_t mw[4];
#pragma unroll
      for (int u = 0; u < 4; ++u) {                              // four words' loads in flight
          const int64_t v = ((w0 + u * nw) << 6) + lane();
          mw[u] = (w0 + u * nw < words && v < n_active) ? fr[v] : 0;
      }
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        const uint64_t mine = mw[u];
        if (!__ballot(mine != 0)) continue;                      // wave-uniform
        uint64_t x = mine;
        constexpr uint64_t kLow[6] = {0x00000000FFFFFFFFULL, 0x0000FFFF0000FFFFULL, 0x00FF00FF00FF00FFULL,
                                      0x0F0F0F0F0F0F0F0FULL, 0x3333333333333333ULL, 0x5555555555555555ULL};
#pragma unroll
        for (int st = 0; st < 6; ++st) {
            const int j = 32 >> st;
            const uint64_t m = kLow[st];
            const uint64_t y = __shfl_xor(x, j, 64);
            x = (lane() & j) ? (((y & ~m) >> j) | (x & ~m)) : ((x & m) | ((y & m) << j));
        }
        sum += static_cast<unsigned long long>(__popcll(x));
      }
    }
    s_sum[threadIdx.x >> 6][lane()] = sum;
    __syncthreads();
    if (threadIdx.x < 64) {
        unsigned long long t = 0;
        for (int w = 0; w < kWavesPerBlock; ++w) t += s_sum[w][threadIdx.x];
        if (t) atomicAdd(&out[threadIdx.x], t);
    }
}

// Wave-wide (all lanes call it): lane b adds the degrees of the lanes whose mask holds bit b.
// The masks are transposed across the wave (as in ms_source_counts) so lane b holds source b's
// column x, and with D_k the ballot of bit k of the lanes' degrees the column's sum is
// sum_k 2^k popcount(x & D_k).
__device__ __forceinline__ void source_columns_add(uint64_t mine, unsigned long long deg, unsigned long long& sum) {
    uint64_t x = mine;
    constexpr uint64_t kLow[6] = {0x00000000FFFFFFFFULL, 0x0000FFFF0000FFFFULL, 0x00FF00FF00FF00FFULL,
                                  0x0F0F0F0F0F0F0F0FULL, 0x3333333333333333ULL, 0x5555555555555555ULL};
#pragma unroll
    for (int st = 0; st < 6; ++st) {
        const int j = 32 >> st;
        const uint64_t m = kLow[st];
        const uint64_t y = __shfl_xor(x, j, 64);
        x = (lane() & j) ? (((y & ~m) >> j) | (x & ~m)) : ((x & m) | ((y & m) << j));
    }
    unsigned long long dor = deg;                                // the wave's highest degree bit
    for (int off = 32; off > 0; off >>= 1) dor |= __shfl_xor(dor, off, 64);
    const int kb = dor ? 64 - __clzll(static_cast<long long>(dor)) : 0;
    for (int k = 0; k < kb; ++k) {
        const uint64_t dk = __ballot((deg >> k) & 1ULL);
        sum += static_cast<unsigned long long>(__popcll(x & dk)) << k;
    }
}
// Block end of a per-source sum: the block's lanes b added into out[b] with one atomic each.
__device__ __forceinline__ void source_sums_flush(unsigned long long sum, unsigned long long* __restrict__ out) {
    __shared__ unsigned long long s_sum[kWavesPerBlock][64];
    s_sum[threadIdx.x >> 6][lane()] = sum;
    __syncthreads();
    if (threadIdx.x < 64) {
        unsigned long long t = 0;
        for (int w = 0; w < kWavesPerBlock; ++w) t += s_sum[w][threadIdx.x];
        if (t) atomicAdd(&out[threadIdx.x], t);
    }
}

// Exact push entries per source of the frontier, for the sources in `cand`: one wave per
// 64-vertex word; the lanes load their vertex's mask (and push degree when it is in the
// frontier), the masks are transposed across the wave (as in ms_source_counts) so lane b holds
// source b's column, and lane b adds the degrees of the column's set bits bit-sliced: with D_k
// the ballot of bit k of the lanes' degrees, the column's sum is sum_k 2^k popcount(x & D_k) —
// one ballot per degree bit instead of one permute per set bit (a word of hubs, each in every
// source's frontier, took 64 permute trips: 158 us at RMAT-24's first pull level).
__global__ void __launch_bounds__(kBlock) ms_source_entries(View push, const uint64_t* __restrict__ fr,
        int64_t n_active, uint64_t cand, unsigned long long* __restrict__ out) {
    const int64_t words = (n_active + 63) >> 6;
    unsigned long long sum = 0;
    const int64_t nw = (static_cast<int64_t>(gridDim.x) * blockDim.x) >> 6;
    for (int64_t w0 = (static_cast<int64_t>(blockIdx.x) * blockDim.x + threadIdx.x) >> 6; w0 < words; w0 += 4 * nw) {
      uint64_t mw[4];
      unsigned long long dw[4];
#pragma unroll
      for (int u = 0; u < 4; ++u) {                              // four words' loads in flight
          const int64_t v = ((w0 + u * nw) << 6) + lane();
          mw[u] = (w0 + u * nw < words && v < n_active) ? (fr[v] & cand) : 0;
      }
#pragma unroll
      for (int u = 0; u < 4; ++u) {
          const int64_t v = ((w0 + u * nw) << 6) + lane();
          dw[u] = mw[u] ? static_cast<unsigned long long>(push_degree(push, v)) : 0ULL;
      }
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        const uint64_t mine = mw[u];
        if (!__ballot(mine != 0)) continue;                      // wave-uniform
        source_columns_add(mine, dw[u], sum);
      }
    }
    source_sums_flush(sum, out);
}

// Frontier bitmap of a pull level: one wave per 64-vertex word, a ballot of fr != 0.
__global__ void __launch_bounds__(kBlock) ms_fbitmap(const uint64_t* __restrict__ fr, int64_t n,
                                                     uint64_t* __restrict__ fbm) {
    const int64_t words = (n + 63) >> 6;
    for (int64_t wd = (static_cast<int64_t>(blockIdx.x) * blockDim.x + threadIdx.x) >> 6; wd < words;
         wd += (static_cast<int64_t>(gridDim.x) * blockDim.x) >> 6) {
        const int64_t v = (wd << 6) + lane();
        const unsigned long long b = __ballot(v < n && fr[v] != 0);
        if (lane() == 0) fbm[wd] = b;
    }
}

// Push level: edge-balanced over the frontier queue (exclusive scan of degrees in qpre).  A
// tile's queue slice (entry, scan offset, list bounds, mask) is staged in LDS once, and each
// thread's kEdgesPerThread edges go through the dependent chain in stages — owning entry,
// neighbour index, the neighbour's masks, the atomic — so every stage's loads are in flight
// together (one edge at a time left each thread waiting out index -> masks -> atomic per edge:
// 463 us for the 12.7 M entries of RMAT-24's second level).  The staged slice holds 512
// entries (18 KB of LDS, eight blocks a CU); a tile touching more (low-degree frontiers)
// searches the global scan instead.
constexpr int kPushLds = 514;
// kE: edges per thread (a tile is kBlock * kE edges).  4 (round 5): 50 VGPRs, 8 waves per SIMD
// — the RMAT-24 sweep 3.76 -> 3.68 ms against 8 (86 VGPRs, 5 waves;
// profiles/r05ms1_ms_push_e_ab.log); TGO_MS_PUSH_E=8 for the A/B
template <int kE = 4>
__global__ void __launch_bounds__(kBlock) ms_push(View push, const int32_t* __restrict__ q,
        const int64_t* __restrict__ qpre, int64_t qlen, const uint64_t* __restrict__ fr,
        const uint64_t* __restrict__ vis, uint64_t* __restrict__ nx, PackTouch touch, uint64_t mask, bool probe,
        uint64_t* __restrict__ own_nx, int64_t own_lo) {
    __shared__ int64_t s_pre[kPushLds];
    __shared__ int64_t s_b0[kPushLds];     // list 0 begin
    __shared__ int64_t s_b1[kPushLds];     // list 1 begin minus list 0's length (o >= d0 reads adj1[s_b1 + o])
    __shared__ int32_t s_d0[kPushLds];     // list 0 length
    __shared__ uint64_t s_m[kPushLds];
    __shared__ int64_t s_lo, s_hi;
    const int64_t total = qpre[qlen];
    const int64_t ntiles = (total + (kBlock * kE) - 1) / (kBlock * kE);
    for (int64_t tile = blockIdx.x; tile < ntiles; tile += gridDim.x) {
        const int64_t t0 = tile * (kBlock * kE);
        const int64_t t1 = min(total, t0 + (kBlock * kE));
        tile_bounds(qpre, qlen, t0, t1, s_lo, s_hi);
        __syncthreads();
        const int64_t lo = s_lo, hi = s_hi;
        const int64_t span = hi - lo + 1;
        const bool in_lds = span + 1 <= kPushLds;             // block-uniform
        if (in_lds) {
            for (int64_t i = threadIdx.x; i <= span; i += kBlock) {
                s_pre[i] = qpre[lo + i];
                if (i < span) {
                    const int32_t u = q[lo + i];
                    const int64_t b0 = push.off0[u];
                    const int64_t d0 = push.off0[u + 1] - b0;
                    s_b0[i] = b0;
                    s_d0[i] = static_cast<int32_t>(min<int64_t>(d0, INT32_MAX));
                    s_b1[i] = push.nlists > 1 ? push.off1[u] - d0 : 0;
                    s_m[i] = fr[u] & mask;
                }
            }
        }
        __syncthreads();
        int32_t v[kE];
        uint64_t m[kE];
        if (in_lds) {
            int64_t ia[kE], o[kE];
#pragma unroll
            for (int k = 0; k < kE; ++k) {       // 1: owning entry (LDS search)
                const int64_t j = t0 + k * kBlock + threadIdx.x;
                ia[k] = -1;
                o[k] = 0;
                if (j >= t1) continue;
                int64_t a = 0, b = span;
                while (b - a > 1) { const int64_t c = (a + b) >> 1; if (s_pre[c] <= j) a = c; else b = c; }
                ia[k] = a;
                o[k] = j - s_pre[a];
            }
#pragma unroll
            for (int k = 0; k < kE; ++k) {       // 2: neighbour index
                v[k] = -1;
                m[k] = 0;
                if (ia[k] < 0) continue;
                m[k] = s_m[ia[k]];
                if (!m[k]) continue;
                v[k] = o[k] < s_d0[ia[k]] ? push.adj0[s_b0[ia[k]] + o[k]] : push.adj1[s_b1[ia[k]] + o[k]];
            }
        } else {                                              // a huge slice: global search
#pragma unroll
            for (int k = 0; k < kE; ++k) {
                const int64_t j = t0 + k * kBlock + threadIdx.x;
                v[k] = -1;
                m[k] = 0;
                if (j >= t1) continue;
                int64_t a = lo, b = hi + 1;
                while (b - a > 1) { const int64_t c = (a + b) >> 1; if (qpre[c] <= j) a = c; else b = c; }
                const int32_t u = q[a];
                m[k] = fr[u] & mask;
                if (m[k]) v[k] = view_entry(push, u, j - qpre[a]);
            }
        }
        uint64_t cv[kE], cn[kE];
        uint64_t* tgt[kE];
#pragma unroll
        for (int k = 0; k < kE; ++k) {           // 3: the neighbour's masks
            cv[k] = 0;
            cn[k] = 0;
            tgt[k] = nullptr;
            if (v[k] < 0) continue;
            // partitioned graphs pass vis = nullptr: remote vertices' masks are not local; with
            // own_nx the owned range [own_lo, own_lo + n_local) goes straight to the next masks
            const int64_t ov = static_cast<int64_t>(v[k]) - own_lo;
            tgt[k] = (own_nx && ov >= 0 && ov < touch.n_local) ? own_nx + ov : nx + v[k];
            if (vis) cv[k] = vis[v[k]];
            if (probe) cn[k] = *tgt[k];
        }
#pragma unroll
        for (int k = 0; k < kE; ++k) {           // 4: the atomic
            if (v[k] < 0) continue;
            const uint64_t mk = m[k] & ~cv[k];
            if (mk && (cn[k] & mk) != mk) {
                atomicOr(reinterpret_cast<unsigned long long*>(tgt[k]), mk);
                if (touch.flag && tgt[k] == nx + v[k])
                    touch.flag[(v[k] / touch.n_local) * touch.cps + (v[k] % touch.n_local) / kPackChunk] = 1;
            }
        }
        __syncthreads();
    }
}

// Target-ranged push (a small frontier of long lists, e.g. RMAT-24's second level: 1355
// vertices, 12.7 M entries): the targets are cut into ranges of S vertices, and the edges are
// enumerated range-major — (range r, frontier entry i) pairs, each the run of entry i's sorted
// lists that lands in range r.  XCD x walks the x-th eighth of that enumeration in order with
// its blocks as one window, so the candidate / reached masks of the ranges it is on stay in its
// L2 and the atomics hit there (in queue order every XCD touched the whole 134 MB mask array).
// P0 / P1 [i * (R + 1) + r]: the first position of entry i's list 0 / 1 with target >= r * S.
__global__ void ms_range_bounds(View push, const int32_t* __restrict__ q, int64_t qlen, int64_t R, int64_t S,
                                int64_t* __restrict__ P0, int64_t* __restrict__ P1) {
    const int64_t R1 = R + 1;
    for (int64_t t = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; t < qlen * R1; t += (int64_t)gridDim.x * blockDim.x) {
        const int64_t i = t / R1, r = t - i * R1;
        const int32_t u = q[i];
        const int64_t key = r * S;
#pragma unroll
        for (int l = 0; l < 2; ++l) {
            if (l == 1 && push.nlists < 2) { P1[t] = 0; break; }
            const int64_t* off = l == 0 ? push.off0 : push.off1;
            const int32_t* adj = l == 0 ? push.adj0 : push.adj1;
            int64_t a = off[u], b = off[u + 1];             // first position with adj >= key
            if (r == R) a = b;
            while (a < b) { const int64_t c = (a + b) >> 1; if (static_cast<int64_t>(adj[c]) < key) a = c + 1; else b = c; }
            (l == 0 ? P0 : P1)[t] = a;
        }
    }
}
// cnt[r * qlen + i] = entries of pair (r, i); cnt[R * qlen] = 0 (for the exclusive scan)
__global__ void ms_range_counts(View push, int64_t qlen, int64_t R, const int64_t* __restrict__ P0,
                                const int64_t* __restrict__ P1, int64_t* __restrict__ cnt) {
    const int64_t R1 = R + 1;
    for (int64_t p = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; p <= R * qlen; p += (int64_t)gridDim.x * blockDim.x) {
        if (p == R * qlen) { cnt[p] = 0; continue; }
        const int64_t r = p / qlen, i = p - r * qlen;
        const int64_t t = i * R1 + r;
        int64_t c = P0[t + 1] - P0[t];
        if (push.nlists > 1) c += P1[t + 1] - P1[t];
        cnt[p] = c;
    }
}
__global__ void __launch_bounds__(kBlock) ms_push_ranged(View push, const int32_t* __restrict__ q, int64_t qlen,
        int64_t R, const int64_t* __restrict__ P0, const int64_t* __restrict__ P1, const int64_t* __restrict__ pre,
        const uint64_t* __restrict__ fr, const uint64_t* __restrict__ vis, uint64_t* __restrict__ nx, uint64_t mask) {
    __shared__ int64_t s_pre[kPushLds];
    __shared__ int64_t s_b0[kPushLds];
    __shared__ int64_t s_b1[kPushLds];
    __shared__ int32_t s_d0[kPushLds];
    __shared__ uint64_t s_m[kPushLds];
    __shared__ int64_t s_lo, s_hi;
    const int64_t npairs = R * qlen, R1 = R + 1;
    const int64_t total = pre[npairs];
    const int64_t ntiles = (total + kTileEdges - 1) / kTileEdges;
    const int64_t x = blockIdx.x & 7, per = gridDim.x >> 3;       // grid: a multiple of 8
    const int64_t tlo = ntiles * x / 8, thi = ntiles * (x + 1) / 8;
    // the pair's list bounds and mask (pair p = r * qlen + i)
    auto pair_info = [&](int64_t p, int64_t& b0, int32_t& d0, int64_t& b1, uint64_t& m) {
        const int64_t r = p / qlen, i = p - r * qlen;
        const int64_t t = i * R1 + r;
        b0 = P0[t];
        const int64_t c0 = P0[t + 1] - b0;
        d0 = static_cast<int32_t>(c0);
        b1 = push.nlists > 1 ? P1[t] - c0 : 0;
        m = fr[q[i]] & mask;
    };
    for (int64_t tile = tlo + (blockIdx.x >> 3); tile < thi; tile += per) {   // block-uniform trips
        const int64_t t0 = tile * kTileEdges;
        const int64_t t1 = min(total, t0 + kTileEdges);
        tile_bounds(pre, npairs, t0, t1, s_lo, s_hi);
        __syncthreads();
        const int64_t lo = s_lo, hi = s_hi;
        const int64_t span = hi - lo + 1;
        const bool in_lds = span + 1 <= kPushLds;              // block-uniform
        if (in_lds)
            for (int64_t i = threadIdx.x; i <= span; i += kBlock) {
                s_pre[i] = pre[lo + i];
                if (i < span) pair_info(lo + i, s_b0[i], s_d0[i], s_b1[i], s_m[i]);
            }
        __syncthreads();
        int32_t v[kEdgesPerThread];
        uint64_t m[kEdgesPerThread];
#pragma unroll
        for (int k = 0; k < kEdgesPerThread; ++k) {            // owning pair, neighbour index
            const int64_t j = t0 + k * kBlock + threadIdx.x;
            v[k] = -1;
            m[k] = 0;
            if (j >= t1) continue;
            int64_t b0, b1, o;
            int32_t d0;
            if (in_lds) {
                int64_t a = 0, b = span;
                while (b - a > 1) { const int64_t c = (a + b) >> 1; if (s_pre[c] <= j) a = c; else b = c; }
                b0 = s_b0[a]; d0 = s_d0[a]; b1 = s_b1[a]; m[k] = s_m[a];
                o = j - s_pre[a];
            } else {
                int64_t a = lo, b = hi + 1;
                while (b - a > 1) { const int64_t c = (a + b) >> 1; if (pre[c] <= j) a = c; else b = c; }
                pair_info(a, b0, d0, b1, m[k]);
                o = j - pre[a];
            }
            if (m[k]) v[k] = o < d0 ? push.adj0[b0 + o] : push.adj1[b1 + o];
        }
        uint64_t cv[kEdgesPerThread], cn[kEdgesPerThread];
#pragma unroll
        for (int k = 0; k < kEdgesPerThread; ++k) {            // the neighbour's masks
            cv[k] = 0;
            cn[k] = 0;
            if (v[k] < 0) continue;
            if (vis) cv[k] = vis[v[k]];
            cn[k] = nx[v[k]];
        }
#pragma unroll
        for (int k = 0; k < kEdgesPerThread; ++k) {            // the atomic
            if (v[k] < 0) continue;
            const uint64_t mk = m[k] & ~cv[k];
            if (mk && (cn[k] & mk) != mk) atomicOr(reinterpret_cast<unsigned long long*>(&nx[v[k]]), mk);
        }
        __syncthreads();
    }
}

// After a push level: settle the candidates (nx & ~vis), record levels, build the queue
// (two-pass chunked extraction, frontier.hpp).
// srcent (optional): the new frontier's push entries per source added in (the next level's
// source split reads them instead of a pass of its own, ms_source_entries).
__global__ void __launch_bounds__(kBlock) ms_settle(View push, int64_t n_active, uint64_t* __restrict__ vis,
        uint64_t* __restrict__ nx, LevelPlanes lvl, int32_t* __restrict__ qn,
        int64_t* __restrict__ qdeg, Counters* cnt, int32_t next_level, unsigned long long* __restrict__ srcent) {
    const int64_t words = (n_active + 63) >> 6;
    unsigned long long ssum = 0;
    auto probe = [&](int64_t wd, Take* t, bool commit) -> bool {
        const int64_t v = (wd << 6) + lane();
        uint64_t fresh = 0, c = 0;
        if (v < n_active) {
            c = nx[v];
            if (c) {
                const uint64_t seen = vis[v];
                fresh = c & ~seen;
                if (commit) {
                    nx[v] = fresh;
                    if (fresh) { vis[v] = seen | fresh; record_level(v, fresh, next_level, lvl); }
                }
            }
        }
        t[0] = {fresh != 0, static_cast<int32_t>(v), fresh ? push_degree(push, v) : 0};
        // the probe runs wave-uniformly; the commit pass visits each word once
        if (commit && srcent && __ballot(fresh != 0)) source_columns_add(fresh, static_cast<unsigned long long>(t[0].deg), ssum);
        return __ballot(c != 0) != 0;                           // words with candidates are rewritten
    };
    chunk_extract<1>(words, probe, qn, qdeg, cnt);
    if (srcent) source_sums_flush(ssum, srcent);                 // grid-uniform
}

// The settle of a push level whose next level will likely pull: the same masks, levels and
// counts as ms_settle without the frontier queue (a pull needs none; ms_queue builds it if the
// next level pushes after all) — one pass instead of the extraction's two, four words in
// flight per wave.  srcent as in ms_settle.
__global__ void __launch_bounds__(kBlock) ms_settle_count(View push, int64_t n_active, uint64_t* __restrict__ vis,
        uint64_t* __restrict__ nx, LevelPlanes lvl, Counters* cnt, int32_t next_level,
        unsigned long long* __restrict__ srcent) {
    unsigned long long nv = 0, mf = 0, bits = 0, ssum = 0;
    const int64_t words = (n_active + 63) >> 6;
    const int64_t nw = (static_cast<int64_t>(gridDim.x) * blockDim.x) >> 6;
    for (int64_t w0 = (static_cast<int64_t>(blockIdx.x) * blockDim.x + threadIdx.x) >> 6; w0 < words; w0 += 4 * nw) {
        uint64_t c[4];
#pragma unroll
        for (int u = 0; u < 4; ++u) {
            const int64_t v = ((w0 + u * nw) << 6) + lane();
            c[u] = (w0 + u * nw < words && v < n_active) ? nx[v] : 0;
        }
#pragma unroll
        for (int u = 0; u < 4; ++u) {
            if (!__ballot(c[u] != 0)) continue;                  // wave-uniform
            const int64_t v = ((w0 + u * nw) << 6) + lane();
            uint64_t fresh = 0;
            int64_t deg = 0;
            if (c[u]) {
                const uint64_t seen = vis[v];
                fresh = c[u] & ~seen;
                nx[v] = fresh;
                if (fresh) {
                    vis[v] = seen | fresh;
                    record_level(v, fresh, next_level, lvl);
                    deg = push_degree(push, v);
                    ++nv;
                    mf += static_cast<unsigned long long>(deg);
                    bits += static_cast<unsigned long long>(__popcll(fresh));
                }
            }
            if (srcent && __ballot(fresh != 0)) source_columns_add(fresh, static_cast<unsigned long long>(deg), ssum);
        }
    }
    count_flush(cnt, nv, mf, bits);
    if (srcent) source_sums_flush(ssum, srcent);                 // grid-uniform
}

// The queue of a frontier produced by a pull level (which only counts): every active v with
// fr[v] != 0, push degrees for the scan.  Built only when the next level pushes.
__global__ void __launch_bounds__(kBlock) ms_queue(View push, int64_t n_active, const uint64_t* __restrict__ fr,
        int32_t* __restrict__ qn, int64_t* __restrict__ qdeg, Counters* cnt, uint64_t mask) {
    const int64_t words = (n_active + 63) >> 6;
    auto probe = [&](int64_t wd, Take* t, bool) -> bool {
        const int64_t v = (wd << 6) + lane();
        const bool take = v < n_active && (fr[v] & mask) != 0;
        t[0] = {take, static_cast<int32_t>(v), take ? push_degree(push, v) : 0};
        return __ballot(take) != 0;
    };
    chunk_extract<1>(words, probe, qn, qdeg, cnt);
}

// Partitioned push: OR the candidate-mask slices every rank sent for the owned vertices.
__global__ void or_slices(const uint64_t* __restrict__ recv, int nslices, int64_t n_local, uint64_t* __restrict__ out) {
    for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n_local; i += (int64_t)gridDim.x * blockDim.x) {
        uint64_t m = 0;
        for (int s = 0; s < nslices; ++s) m |= recv[static_cast<int64_t>(s) * n_local + i];
        out[i] = m;
    }
}

// Partitioned sparse push exchange: the nonzero candidate words of every owner's slice
// become (owner-local id, mask) pairs, rank-major and contiguous, so they go straight into
// an all-to-all with split sizes.  Each slice is cut into chunks of kPackChunk words (a
// multiple of 64, so a chunk never straddles slices); one wave owns one chunk.  Pass 0
// counts the chunk's nonzero words (cnt[c]); an exclusive scan gives each chunk its first
// pair; pass 1 writes the pairs in word order and clears the words (the candidate array is
// zero again for the next level).  No atomics: the pair order is deterministic.
// touched (optional): per-chunk flags set by ms_push — a chunk no push wrote is all zero and
// is skipped without reading its words; the write pass clears the flags it consumed.
// self >= 0: the chunks of that slice (the packing rank's own vertices) are not packed; their
// words stay for ms_or_local (no pairs to or from oneself).
template <bool kWrite>
__global__ void __launch_bounds__(kBlock) ms_pack(uint64_t* __restrict__ cand, int64_t n_local, int64_t cps,
        int64_t nchunks, int64_t* __restrict__ cnt, const int64_t* __restrict__ offs, int64_t* __restrict__ send,
        uint8_t* __restrict__ touched, int self) {
    const int64_t c = (blockIdx.x * (int64_t)blockDim.x + threadIdx.x) >> 6;
    if (c >= nchunks) return;
    const int64_t r = c / cps, j = c - r * cps;
    if ((touched && !touched[c]) || r == self) {
        if (!kWrite && lane() == 0) cnt[c] = 0;
        return;
    }
    const int64_t w0 = r * n_local + j * kPackChunk;
    const int64_t w1 = r * n_local + min(n_local, (j + 1) * kPackChunk);
    int64_t base = kWrite ? offs[c] : 0;
    for (int64_t g = w0; g < w1; g += 64) {
        const int64_t i = g + lane();
        const uint64_t m = cand[i];
        const uint64_t bal = __ballot(m != 0);
        if (kWrite && m) {
            const int64_t p = base + __popcll(bal & ((1ULL << lane()) - 1ULL));
            send[2 * p] = i - r * n_local;
            send[2 * p + 1] = static_cast<int64_t>(m);
            cand[i] = 0;
        }
        base += __popcll(bal);
    }
    if (!kWrite && lane() == 0) cnt[c] = base;
    if (kWrite && touched && lane() == 0) touched[c] = 0;
}
// Per-destination element counts of the packed pairs (2 int64 per pair) from the chunk
// offsets, for a device-side all-to-all of the split sizes.
__global__ void slice_elems(const int64_t* __restrict__ off, int64_t cps, int nranks, int64_t* __restrict__ out) {
    const int r = threadIdx.x;
    if (blockIdx.x == 0 && r < nranks) out[r] = 2 * (off[(r + 1) * cps] - off[r * cps]);
}
// Fixed-capacity form of the exchange (tgo_part_ms_pack_fixed): destination r's slot holds
// a header pair (count, 0) and up to `cap` pairs, so the all-to-all has equal splits known
// on the host before the level — no all-to-all of split sizes, no host read of them.  The
// caller's cap bounds the count (a rank's pairs for one owner <= its pushed entries <= the
// level's frontier entries); a count over cap is recorded in *ovf and fails the sweep.
__global__ void __launch_bounds__(kBlock) ms_pack_fixed(uint64_t* __restrict__ cand, int64_t n_local, int64_t cps,
        int64_t nchunks, const int64_t* __restrict__ offs, int64_t cap, int64_t* __restrict__ send, int* ovf,
        uint8_t* __restrict__ touched, int self) {
    const int64_t c = (blockIdx.x * (int64_t)blockDim.x + threadIdx.x) >> 6;
    if (c >= nchunks) return;
    const int64_t r = c / cps, j = c - r * cps;
    if ((touched && !touched[c]) || r == self) return;
    const int64_t w0 = r * n_local + j * kPackChunk;
    const int64_t w1 = r * n_local + min(n_local, (j + 1) * kPackChunk);
    int64_t base = offs[c] - offs[r * cps];                 // pair index within owner r's slot
    int64_t* slot = send + 2 * r * (cap + 1) + 2;
    for (int64_t g = w0; g < w1; g += 64) {
        const int64_t i = g + lane();
        const uint64_t m = cand[i];
        const uint64_t bal = __ballot(m != 0);
        if (m) {
            const int64_t p = base + __popcll(bal & ((1ULL << lane()) - 1ULL));
            if (p < cap) {
                slot[2 * p] = i - r * n_local;
                slot[2 * p + 1] = static_cast<int64_t>(m);
            } else {
                atomicOr(ovf, 1);
            }
            cand[i] = 0;
        }
        base += __popcll(bal);
    }
    if (touched && lane() == 0) touched[c] = 0;
}
__global__ void fixed_headers(const int64_t* __restrict__ off, int64_t cps, int nranks, int64_t cap,
                              int64_t* __restrict__ send) {
    const int r = threadIdx.x;
    if (blockIdx.x == 0 && r < nranks) {
        send[2 * r * (cap + 1)] = min(cap, off[(r + 1) * cps] - off[r * cps]);
        send[2 * r * (cap + 1) + 1] = 0;
    }
}
// Receiver side: slot s of recv came from sender s; OR its pairs into the owned words.
__global__ void ms_or_fixed(const int64_t* __restrict__ recv, int nslices, int64_t cap, uint64_t* __restrict__ nx) {
    const int64_t total = static_cast<int64_t>(nslices) * cap;
    for (int64_t k = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; k < total; k += (int64_t)gridDim.x * blockDim.x) {
        const int64_t s = k / cap, i = k - s * cap;
        const int64_t* slot = recv + 2 * s * (cap + 1);
        if (i >= slot[0]) continue;
        atomicOr(reinterpret_cast<unsigned long long*>(nx + slot[2 + 2 * i]), static_cast<unsigned long long>(slot[3 + 2 * i]));
    }
}

// Received pairs of one sender: OR the masks into the owned candidate words (several
// senders may name one vertex).
__global__ void ms_or_pairs(const int64_t* __restrict__ pairs, int64_t npairs, uint64_t* __restrict__ nx) {
    for (int64_t k = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; k < npairs; k += (int64_t)gridDim.x * blockDim.x)
        atomicOr(reinterpret_cast<unsigned long long*>(nx + pairs[2 * k]), static_cast<unsigned long long>(pairs[2 * k + 1]));
}

// The packing rank's own slice of the candidate words (left by ms_pack with self): OR into
// the owned next masks and clear, chunk by chunk (only chunks a push touched), flags reset.
__global__ void __launch_bounds__(kBlock) ms_or_local(uint64_t* __restrict__ cand_own, int64_t n_local, int64_t cps,
        uint8_t* __restrict__ touched_own, uint64_t* __restrict__ nx) {
    const int64_t j = (blockIdx.x * (int64_t)blockDim.x + threadIdx.x) >> 6;
    if (j >= cps) return;
    if (touched_own && !touched_own[j]) return;
    const int64_t w1 = min(n_local, (j + 1) * kPackChunk);
    for (int64_t i = j * kPackChunk + lane(); i < w1; i += 64) {
        const uint64_t m = cand_own[i];
        if (m) {
            nx[i] |= m;
            cand_own[i] = 0;
        }
    }
    if (touched_own && lane() == 0) touched_own[j] = 0;
}

// Per-source reached vertices / entries (stats, untimed): 64 counters per block in LDS.
__global__ void __launch_bounds__(kBlock) ms_reach(View v, const uint64_t* __restrict__ vis, int64_t n_active,
        int nsrc, unsigned long long* __restrict__ reached, unsigned long long* __restrict__ entries) {
    __shared__ unsigned long long s_r[kMaxSources], s_e[kMaxSources];
    if (threadIdx.x < kMaxSources) { s_r[threadIdx.x] = 0; s_e[threadIdx.x] = 0; }
    __syncthreads();
    for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n_active; i += (int64_t)gridDim.x * blockDim.x) {
        uint64_t b = vis[i];
        if (!b) continue;
        const unsigned long long d = static_cast<unsigned long long>(push_degree(v, i));
        while (b) {
            const int r = __ffsll(static_cast<long long>(b)) - 1;
            b &= b - 1;
            atomicAdd(&s_r[r], 1ULL);
            atomicAdd(&s_e[r], d);
        }
    }
    __syncthreads();
    if (threadIdx.x < nsrc) {
        atomicAdd(&reached[threadIdx.x], s_r[threadIdx.x]);
        atomicAdd(&entries[threadIdx.x], s_e[threadIdx.x]);
    }
}

// Source r's distances in row order: the level of (perm[v], r) read back from the planes
// (nplanes = planes written by this sweep); unreached = r's bit clear in vis.
__global__ void ms_extract(LevelPlanes lvl, int nplanes, const uint64_t* __restrict__ vis,
                           const int32_t* __restrict__ perm, int r, int64_t* __restrict__ dist, int64_t n) {
    for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
        const int64_t v = perm[i];
        int64_t l = INT64_MIN;
        if ((vis[v] >> r) & 1ULL) {
            l = 0;
            for (int k = 0; k < nplanes; ++k) l |= static_cast<int64_t>((lvl.p[k * lvl.stride + v] >> r) & 1ULL) << k;
        }
        dist[i] = l;
    }
}

inline int grid_for(int64_t work, int cap) {
    int64_t g = (work + kBlock - 1) / kBlock;
    if (g < 1) g = 1;
    if (g > cap) g = cap;
    return static_cast<int>(g);
}

}  // namespace

hipError_t k_ms_seed(const int64_t* seeds, int nseeds, uint64_t* vis, uint64_t* fr, int64_t fr_rows, hipStream_t s) {
    ms_seed<<<1, 64, 0, s>>>(seeds, nseeds, vis, fr, fr_rows);
    return hipGetLastError();
}
hipError_t k_ms_pull(const View& pull, const View& push, int64_t n_active, uint64_t full, const uint64_t* fr,
                     const uint64_t* fbm, uint64_t* vis, uint64_t* nx, LevelPlanes lvl, Counters* cnt,
                     int32_t next_level, hipStream_t s, int32_t filter_from, uint64_t dense, const uint64_t* cand,
                     MsColdSplit cs) {
    // TGO_MS_STEP: entries a lane loads per round trip of its own list (4 default since the
    // trips are branch-free, round 6: sweep 3.623 -> 3.562 ms against 8 with the branchy trips,
    // profiles/r06ms1_ms_branchfree_ab.log; 8 / 16 probes)
    static const int step = [] { const char* e = std::getenv("TGO_MS_STEP"); return e ? std::atoi(e) : 4; }();
    static const bool diag = [] { const char* e = std::getenv("TGO_MS_DIAG"); return e && std::atoi(e) != 0; }();
    // TGO_MS_LONG: entries per lane per trip of a long list.  1 (default, round 4): with the
    // source split most long walks stop early, and a 64-entry trip stops them soonest — sweep
    // 4.27 -> 3.69-3.74 ms against 4 (2: 4.00, 8: 4.60; profiles/r04z4_ms_pull_ab.log)
    static const int lng = [] { const char* e = std::getenv("TGO_MS_LONG"); return e ? std::atoi(e) : 1; }();
    // TGO_MS_RAMP=1 (with TGO_MS_LONG=4): a long list's first trip reads 64 entries
    static const bool ramp = [] { const char* e = std::getenv("TGO_MS_RAMP"); return e && std::atoi(e) != 0; }();
    // TGO_MS_COOP: lists longer than this are walked by the whole wave (64 default)
    static const int64_t coop = [] { const char* e = std::getenv("TGO_MS_COOP"); return e ? std::atoll(e) : kCoop; }();
    const dim3 grid(grid_for(n_active, 8192));
#define TGO_MS_PULL(S, D, LG, R) ms_pull<S, D, LG, R><<<grid, kBlock, 0, s>>>(pull, push, n_active, full, fr, fbm, vis, \
        nx, lvl, cnt, next_level, filter_from, dense, cand, cs, coop)
    if (diag) TGO_MS_PULL(8, true, 1, false);
    else if (ramp) TGO_MS_PULL(8, false, 4, true);
    else if (step == 4 && lng == 1) TGO_MS_PULL(4, false, 1, false);
    else if (step == 16 && lng == 1) TGO_MS_PULL(16, false, 1, false);
    else if (lng == 1) TGO_MS_PULL(8, false, 1, false);
    else if (lng == 2) TGO_MS_PULL(8, false, 2, false);
    else if (lng == 8) TGO_MS_PULL(8, false, 8, false);
    else if (step == 4) TGO_MS_PULL(4, false, 4, false);
    else if (step == 16) TGO_MS_PULL(16, false, 4, false);
    else TGO_MS_PULL(8, false, 4, false);
#undef TGO_MS_PULL
    return hipGetLastError();
}
hipError_t k_ms_cold(const int32_t* cadj, const int32_t* crow, int64_t C, const uint64_t* fr, const uint8_t* need,
                     uint64_t* acc, hipStream_t s) {
    if (C > 0) ms_cold<<<8 * 1024, kBlock, 0, s>>>(cadj, crow, C, fr, need, acc);
    return hipGetLastError();
}
hipError_t k_ms_finish(const View& push, int64_t n_active, uint64_t full, uint64_t* vis, uint64_t* nx,
                       const uint64_t* cand, LevelPlanes lvl, Counters* cnt, int32_t next_level, uint8_t* need,
                       const uint64_t* acc, hipStream_t s) {
    ms_finish<<<grid_for(n_active, 4096), kBlock, 0, s>>>(push, n_active, full, vis, nx, cand, lvl, cnt, next_level, need,
                                                         acc);
    return hipGetLastError();
}
hipError_t k_cold_flags(const int32_t* adj, int64_t m, int32_t hot, uint32_t* flag, hipStream_t s) {
    if (m > 0) cold_flags<<<grid_for(m, 65536), kBlock, 0, s>>>(adj, m, hot, flag);
    return hipGetLastError();
}
hipError_t k_cold_emit(const int64_t* off, int64_t n, const int32_t* adj, int64_t m, const uint32_t* flag,
                       const uint64_t* pos, int64_t base, int32_t hot, int64_t seg, uint64_t* key, int32_t* val,
                       hipStream_t s) {
    if (m > 0) cold_emit<<<grid_for(m, 65536), kBlock, 0, s>>>(off, n, adj, m, flag, pos, base, hot, seg, key, val);
    return hipGetLastError();
}
hipError_t k_low_rows(const uint64_t* key, int64_t m, int32_t* row, hipStream_t s) {
    if (m > 0) low_rows<<<grid_for(m, 65536), kBlock, 0, s>>>(key, m, row);
    return hipGetLastError();
}
// The pull diagnostics since the last call (zeroed after the read).
hipError_t k_ms_diag_take(unsigned long long* out, hipStream_t s) {  // kDiagWords (10) words
    hipError_t e = hipMemcpyFromSymbolAsync(out, HIP_SYMBOL(g_ms_diag), kDiagWords * sizeof(unsigned long long), 0,
                                            hipMemcpyDeviceToHost, s);
    if (e != hipSuccess) return e;
    static const unsigned long long zero[kDiagWords] = {};
    e = hipMemcpyToSymbolAsync(HIP_SYMBOL(g_ms_diag), zero, sizeof(zero), 0, hipMemcpyHostToDevice, s);
    if (e != hipSuccess) return e;
    return hipStreamSynchronize(s);
}
hipError_t k_ms_source_counts(const uint64_t* fr, int64_t n_active, unsigned long long* out64, hipStream_t s) {
    hipError_t e = hipMemsetAsync(out64, 0, 64 * sizeof(unsigned long long), s);
    if (e != hipSuccess) return e;
    // few blocks: each block ends in 64 atomics on the same 64 words (4096 blocks spent
    // ~50 us queueing on them)
    ms_source_counts<<<grid_for(n_active, 512), kBlock, 0, s>>>(fr, n_active, out64);
    return hipGetLastError();
}
hipError_t k_ms_source_entries(const View& push, const uint64_t* fr, int64_t n_active, uint64_t cand,
                               unsigned long long* out64, hipStream_t s) {
    hipError_t e = hipMemsetAsync(out64, 0, 64 * sizeof(unsigned long long), s);
    if (e != hipSuccess) return e;
    ms_source_entries<<<grid_for(n_active, 512), kBlock, 0, s>>>(push, fr, n_active, cand, out64);
    return hipGetLastError();
}
hipError_t k_ms_fbitmap(const uint64_t* fr, int64_t n, uint64_t* fbm, hipStream_t s) {
    const int64_t words = (n + 63) / 64;
    ms_fbitmap<<<grid_for(words * 64, 8192), kBlock, 0, s>>>(fr, n, fbm);
    return hipGetLastError();
}
hipError_t k_ms_queue(const View& push, int64_t n_active, const uint64_t* fr, int32_t* qn, int64_t* qdeg, Counters* cnt,
                      hipStream_t s, uint64_t mask) {
    ms_queue<<<extract_grid((n_active + 63) / 64), kBlock, 0, s>>>(push, n_active, fr, qn, qdeg, cnt, mask);
    return hipGetLastError();
}
hipError_t k_ms_push(const View& push, const int32_t* q, const int64_t* qpre, int64_t qlen, const uint64_t* fr,
                     const uint64_t* vis, uint64_t* nx, hipStream_t s, PackTouch touch, uint64_t mask, bool probe,
                     uint64_t* own_nx, int64_t own_lo) {
    static const bool e8 = [] { const char* e = std::getenv("TGO_MS_PUSH_E"); return e && std::atoi(e) == 8; }();
    if (e8) ms_push<8><<<256 * 8, kBlock, 0, s>>>(push, q, qpre, qlen, fr, vis, nx, touch, mask, probe, own_nx, own_lo);
    else ms_push<><<<256 * 8, kBlock, 0, s>>>(push, q, qpre, qlen, fr, vis, nx, touch, mask, probe, own_nx, own_lo);
    return hipGetLastError();
}
hipError_t k_ms_push_ranged(const View& push, const int32_t* q, int64_t qlen, int64_t n_active, int64_t S,
                            int64_t* P0, int64_t* P1, int64_t* cnt, int64_t* pre, void*& tmp, size_t& tmp_bytes,
                            const uint64_t* fr, const uint64_t* vis, uint64_t* nx, hipStream_t s, uint64_t mask) {
    if (S < 1 || qlen < 1) return hipErrorInvalidValue;
    const int64_t R = (n_active + S - 1) / S;
    if (R < 1) return hipErrorInvalidValue;
    ms_range_bounds<<<grid_for(qlen * (R + 1), 2048), kBlock, 0, s>>>(push, q, qlen, R, S, P0, P1);
    ms_range_counts<<<grid_for(R * qlen + 1, 2048), kBlock, 0, s>>>(push, qlen, R, P0, P1, cnt);
    hipError_t e = scan_exclusive_i64(tmp, tmp_bytes, cnt, pre, R * qlen + 1, s);
    if (e != hipSuccess) return e;
    ms_push_ranged<<<256 * 8, kBlock, 0, s>>>(push, q, qlen, R, P0, P1, pre, fr, vis, nx, mask);
    return hipGetLastError();
}
hipError_t k_ms_settle_count(const View& push, int64_t n_active, uint64_t* vis, uint64_t* nx, LevelPlanes lvl,
                            Counters* cnt, int32_t next_level, hipStream_t s, unsigned long long* srcent) {
    ms_settle_count<<<grid_for(n_active, 2048), kBlock, 0, s>>>(push, n_active, vis, nx, lvl, cnt, next_level, srcent);
    return hipGetLastError();
}
hipError_t k_ms_settle(const View& push, int64_t n_active, uint64_t* vis, uint64_t* nx, LevelPlanes lvl, int32_t* qn,
                       int64_t* qdeg, Counters* cnt, int32_t next_level, hipStream_t s, unsigned long long* srcent) {
    ms_settle<<<extract_grid((n_active + 63) / 64), kBlock, 0, s>>>(push, n_active, vis, nx, lvl, qn, qdeg, cnt,
                                                                    next_level, srcent);
    return hipGetLastError();
}
hipError_t k_ms_reach(const View& v, const uint64_t* vis, int64_t n_active, int nsrc, unsigned long long* reached,
                      unsigned long long* entries, hipStream_t s) {
    ms_reach<<<grid_for(n_active, 2048), kBlock, 0, s>>>(v, vis, n_active, nsrc, reached, entries);
    return hipGetLastError();
}
hipError_t k_ms_pack(bool write, uint64_t* cand, int64_t n_local, int64_t cps, int64_t nchunks, int64_t* cnt,
                     const int64_t* offs, int64_t* send, hipStream_t s, uint8_t* touched, int self) {
    const unsigned blocks = static_cast<unsigned>((nchunks * 64 + kBlock - 1) / kBlock);
    if (write) ms_pack<true><<<blocks, kBlock, 0, s>>>(cand, n_local, cps, nchunks, cnt, offs, send, touched, self);
    else ms_pack<false><<<blocks, kBlock, 0, s>>>(cand, n_local, cps, nchunks, cnt, offs, send, touched, self);
    return hipGetLastError();
}
hipError_t k_ms_or_local(uint64_t* cand_own, int64_t n_local, int64_t cps, uint8_t* touched_own, uint64_t* nx,
                         hipStream_t s) {
    ms_or_local<<<static_cast<unsigned>((cps * 64 + kBlock - 1) / kBlock), kBlock, 0, s>>>(cand_own, n_local, cps,
                                                                                           touched_own, nx);
    return hipGetLastError();
}
hipError_t k_slice_elems(const int64_t* off, int64_t cps, int nranks, int64_t* out, hipStream_t s) {
    slice_elems<<<1, kBlock, 0, s>>>(off, cps, nranks, out);
    return hipGetLastError();
}
hipError_t k_ms_pack_fixed(uint64_t* cand, int64_t n_local, int64_t cps, int64_t nchunks, const int64_t* offs,
                           int nranks, int64_t cap, int64_t* send, int* ovf, uint8_t* touched, hipStream_t s, int self) {
    const int64_t threads = nchunks * 64;
    ms_pack_fixed<<<static_cast<unsigned>((threads + kBlock - 1) / kBlock), kBlock, 0, s>>>(cand, n_local, cps, nchunks, offs,
                                                                                           cap, send, ovf, touched, self);
    fixed_headers<<<1, 64, 0, s>>>(offs, cps, nranks, cap, send);
    return hipGetLastError();
}
hipError_t k_ms_or_fixed(const int64_t* recv, int nslices, int64_t cap, uint64_t* nx, hipStream_t s) {
    const int64_t total = static_cast<int64_t>(nslices) * cap;
    int64_t g = (total + kBlock - 1) / kBlock;
    g = std::max<int64_t>(1, std::min<int64_t>(g, 65536));
    ms_or_fixed<<<static_cast<unsigned>(g), kBlock, 0, s>>>(recv, nslices, cap, nx);
    return hipGetLastError();
}
hipError_t k_ms_or_pairs(const int64_t* pairs, int64_t npairs, uint64_t* nx, hipStream_t s) {
    if (npairs > 0) ms_or_pairs<<<grid_for(npairs, 4096), kBlock, 0, s>>>(pairs, npairs, nx);
    return hipGetLastError();
}
hipError_t k_or_slices(const uint64_t* recv, int nslices, int64_t n_local, uint64_t* out, hipStream_t s) {
    or_slices<<<grid_for(n_local, 4096), kBlock, 0, s>>>(recv, nslices, n_local, out);
    return hipGetLastError();
}
hipError_t k_ms_extract(LevelPlanes lvl, int nplanes, const uint64_t* vis, const int32_t* perm, int r, int64_t* dist,
                        int64_t n, hipStream_t s) {
    ms_extract<<<grid_for(n, 4096), kBlock, 0, s>>>(lvl, nplanes, vis, perm, r, dist, n);
    return hipGetLastError();
}

}  // namespace tgo

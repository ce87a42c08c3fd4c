// delta.hip — delta-stepping SSSP (Meyer & Sanders, J. Algorithms 2003) on gfx950 for
// ShortestDistanceVertexProgram's converged distances (TGO_SSSP_DELTA), on one GPU or on a
// 1-D vertex partition of the graph over several.
//
// The reference program (ShortestDistanceVertexProgram.java:96-130) is a Jacobi
// Bellman-Ford: every superstep every reached vertex re-sends its distance, so a run of
// maxDepth supersteps relaxes every edge of the reached set up to maxDepth times.  With
// non-negative integer weights the converged result is unique, so any relaxation order
// reaches the same bit-exact distances; delta-stepping orders the work by distance buckets
// of width delta so that most vertices are relaxed once, with their final distance.
//
// Device state per run:
//   dist[v]   int64, atomicMin'd (global atomics execute at the memory side: coherent
//             across the 8 XCDs' L2s)
//   pend      bitmap: v improved and not yet relaxed with its current distance
//   msg[v]    snapshot of dist[v] taken when v enters a phase queue; the phase relaxes from
//             the snapshot, so a concurrent improvement of v (which sets pend again) never
//             leaks into the phase half-seen — it simply queues v once more.
// A phase relaxes the near queue (pending vertices with dist < thr) edge-balanced; a
// vertex improved below thr whose pend bit was clear joins the next near queue at once;
// the rest stay pending.  When the near queue runs dry, the host reads the minimum pending
// distance, moves thr to the end of that bucket and extracts the next near queue from the
// pending bitmap (a 2 MB scan at RMAT scale 24).
//
// Partitioned (titan_gpu_olap_part.h): the ctx holds the rows of global vertices
// [lo, lo + n_local).  A relaxation whose target is owned elsewhere is min-reduced per
// global target into rbest (int64 per global vertex) and marked in rmark (one bit per
// global vertex); after the phase the marks are packed per owner rank into (owner-local
// id, distance) pairs, the caller's all-to-all moves them, and the owner mins them into its
// dist with the same pending / near-queue rule (ds_apply).  rbest lives for the whole run:
// a target is re-sent only when this rank improves on what it sent before.
#include <cstdlib>
#include <hip/hip_runtime.h>
#include "frontier.hpp"

namespace tgo {
namespace {

constexpr long long kInfLL = 0x7FFFFFFFFFFFFFFFLL;

// min(cand) into dist[v] of an owned vertex; true when v has to join the near queue.  An
// improvement that leaves v pending outside the queue folds cand into tmin (the partitioned
// loop's running pending minimum, see ds_track_reset).
__device__ __forceinline__ bool relax_owned(int64_t* dist, uint64_t* pend, int64_t v, int64_t cand, int64_t thr,
                                            long long& tmin) {
    if (cand >= dist[v]) return false;                  // a stale (larger) read only costs an atomic
    const long long old = atomicMin(reinterpret_cast<long long*>(&dist[v]), static_cast<long long>(cand));
    if (cand >= old) return false;
    const uint64_t bit = 1ULL << (v & 63);
    const unsigned long long ob = atomicOr(reinterpret_cast<unsigned long long*>(&pend[v >> 6]), bit);
    const bool take = !(ob & bit) && cand < thr;
    if (!take && cand < tmin) tmin = cand;
    return take;
}

// Block minimum of x into *dst, one atomicMin per block (every thread of the block calls it).
__device__ __forceinline__ void block_fold_min(long long x, long long* dst) {
    __shared__ long long s_m[kWavesPerBlock];
    for (int o = 32; o > 0; o >>= 1) {
        const long long y = __shfl_xor(x, o, 64);
        x = y < x ? y : x;
    }
    __syncthreads();
    if (lane() == 0) s_m[threadIdx.x >> 6] = x;
    __syncthreads();
    if (threadIdx.x == 0) {
        for (int w = 1; w < kWavesPerBlock; ++w) x = s_m[w] < x ? s_m[w] : x;
        if (x != kInfLL) atomicMin(dst, x);
    }
}

__global__ void ds_seed(View push, int64_t* dist, int32_t* q, int64_t* qdeg, int64_t seed) {
    if (threadIdx.x == 0 && blockIdx.x == 0) {
        dist[seed] = 0;
        q[0] = static_cast<int32_t>(seed);
        qdeg[0] = push_degree(push, seed);
    }
}

// Phase prologue: snapshot the queue's distances, clear their pending bits.
__global__ void ds_commit(const int32_t* __restrict__ q, int64_t qlen, const int64_t* __restrict__ dist,
                          int64_t* __restrict__ msg, uint64_t* __restrict__ pend) {
    for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < qlen; i += (int64_t)gridDim.x * blockDim.x) {
        const int32_t v = q[i];
        msg[v] = dist[v];
        const uint64_t bit = 1ULL << (v & 63);
        if (pend[v >> 6] & bit) atomicAnd(reinterpret_cast<unsigned long long*>(&pend[v >> 6]), ~bit);
    }
}

// Relax every push entry of the near queue (load-balanced search over the exclusive scan
// of the queue's degrees, 2048 entries per 256-thread tile, queue slice staged in LDS).
// kPart: targets outside [lo, lo + n_local) go to rbest / rmark (see the header).
template <bool kPart>
__global__ void __launch_bounds__(kBlock) ds_relax(View push, const int32_t* __restrict__ q,
        const int64_t* __restrict__ qpre, int64_t qlen, const int64_t* __restrict__ msg,
        int64_t* __restrict__ dist, uint64_t* __restrict__ pend, int32_t* __restrict__ qn,
        int64_t* __restrict__ qdeg_n, Counters* cnt, int weighted, int64_t thr, int64_t lo, int64_t n_local,
        int64_t* __restrict__ rbest, uint64_t* __restrict__ rmark, long long* __restrict__ track) {
    __shared__ AppendLds sh;
    unsigned long long mf = 0;
    long long tmin = kInfLL;
    if (blockIdx.x == 0 && threadIdx.x == 0) cnt->red[1] = static_cast<unsigned long long>(qpre[qlen]);   // work done
    for_each_queue_edge(q, qpre, qlen, [&](bool valid, int32_t u, int64_t o) {
        bool take = false;
        int32_t v = 0;
        int64_t vdeg = 0;
        if (valid) {
            int32_t t, w;
            entry_at(push, u, o, t, w);
            if (!weighted) w = 1;
            const int64_t mu = msg[u];
            if (w == kMissingWeight) {
                atomicOr(&cnt->err, 1ULL);          // edge.value(weight) on a missing key
            } else if (dist[u] < mu) {
                // u improved during this phase: it is pending again and will relax every
                // entry with the better distance, so this relaxation is wasted work
            } else {
                const int64_t cand = mu + static_cast<int64_t>(w);
                const int64_t tl = kPart ? static_cast<int64_t>(t) - lo : static_cast<int64_t>(t);
                if (!kPart || (tl >= 0 && tl < n_local)) {
                    if (relax_owned(dist, pend, tl, cand, thr, tmin)) {
                        take = true;
                        v = static_cast<int32_t>(tl);
                        vdeg = push_degree(push, tl);
                    }
                } else if (cand < rbest[t]) {
                    const long long old = atomicMin(reinterpret_cast<long long*>(&rbest[t]), static_cast<long long>(cand));
                    if (cand < old) {
                        const uint64_t bit = 1ULL << (t & 63);
                        if (!(rmark[t >> 6] & bit)) atomicOr(reinterpret_cast<unsigned long long*>(&rmark[t >> 6]), bit);
                    }
                }
            }
        }
        block_append(take, v, vdeg, qn, qdeg_n, cnt, sh, mf);
    });
    block_flush(cnt, sh, mf);
    if (track) block_fold_min(tmin, track);
}

// ---- light/heavy split (one GPU, weighted): the push entries of every vertex sorted by
// weight (DevGraph::push_ws), light[u] = end of u's entries lighter than delta.  A bucket's
// phases relax LIGHT entries only; a vertex relaxed in the bucket is marked in `member`.  When
// the bucket's near queue runs dry its members' distances are final, and their HEAVY entries
// are relaxed once (Meyer & Sanders' light/heavy split) — in the same launches as the next
// bucket's first light phase: the extraction queues the next near queue and the members'
// heavy entries together (queue entry | kHeavyFlag), so the split costs no extra host round
// trip.  A heavy relaxation lands at >= the settled bucket's threshold: in the new bucket it
// simply joins the near queue, beyond it it stays pending (label-correcting: the converged
// distances do not depend on the order).
constexpr uint32_t kHeavyFlag = 0x80000000u;

__device__ __forceinline__ int64_t light_degree(const int64_t* off, const int64_t* light, int64_t u) {
    return light[u] - off[u];
}

__global__ void ds_light_end(const int64_t* __restrict__ off, const int32_t* __restrict__ w, int64_t delta,
                             int64_t n, int64_t* __restrict__ light) {
    for (int64_t v = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; v < n; v += (int64_t)gridDim.x * blockDim.x) {
        int64_t a = off[v], b = off[v + 1];               // first entry with w >= delta
        while (a < b) {
            const int64_t c = (a + b) >> 1;
            if (static_cast<int64_t>(w[c]) < delta) a = c + 1; else b = c;
        }
        light[v] = a;
    }
}

__global__ void ds_seed_ws(const int64_t* off, const int64_t* light, int64_t* dist, int32_t* q, int64_t* qdeg,
                           int64_t seed) {
    if (threadIdx.x == 0 && blockIdx.x == 0) {
        dist[seed] = 0;
        q[0] = static_cast<int32_t>(seed);
        qdeg[0] = light_degree(off, light, seed);
    }
}

// Light entries: snapshot, clear pending, mark the bucket member.  Heavy entries: the member's
// distance is final and msg already holds it.  Also zeroes the counters and the scan's tail
// degree for the phase (saves two memset launches per phase).
// track (partitioned): track[1] = 1 once a member is marked (members wait for their heavy pass).
__global__ void ds_commit_ws(const int32_t* __restrict__ q, int64_t qlen, const int64_t* __restrict__ dist,
                             int64_t* __restrict__ msg, uint64_t* __restrict__ pend, uint64_t* __restrict__ member,
                             int64_t* __restrict__ qdeg, Counters* cnt, long long* __restrict__ track) {
    if (blockIdx.x == 0) {
        constexpr int kWords = sizeof(Counters) / sizeof(unsigned long long);
        static_assert(kWords <= kBlock, "one thread per counter word");
        if (threadIdx.x < kWords) reinterpret_cast<unsigned long long*>(cnt)[threadIdx.x] = 0ULL;
        if (threadIdx.x == 0) qdeg[qlen] = 0;
    }
    for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < qlen; i += (int64_t)gridDim.x * blockDim.x) {
        const uint32_t e = static_cast<uint32_t>(q[i]);
        if (e & kHeavyFlag) continue;
        const int32_t v = static_cast<int32_t>(e);
        msg[v] = dist[v];
        const uint64_t bit = 1ULL << (v & 63);
        if (pend[v >> 6] & bit) atomicAnd(reinterpret_cast<unsigned long long*>(&pend[v >> 6]), ~bit);
        if (!(member[v >> 6] & bit)) {
            atomicOr(reinterpret_cast<unsigned long long*>(&member[v >> 6]), bit);
            if (track) track[1] = 1;
        }
    }
}

// ds_relax over one weight-sorted list: queue entry u relaxes [off[u], light[u]) or, flagged
// heavy, [light[u], off[u+1]); load-balanced as in ds_relax.
// kPart: targets outside [lo, lo + n_local) go to rbest / rmark as in ds_relax.
template <bool kPart>
__global__ void __launch_bounds__(kBlock) ds_relax_ws(const int64_t* __restrict__ off, const int32_t* __restrict__ adj,
        const int32_t* __restrict__ wt, const int64_t* __restrict__ light, const int32_t* __restrict__ q,
        const int64_t* __restrict__ qpre, int64_t qlen, const int64_t* __restrict__ msg, int64_t* __restrict__ dist,
        uint64_t* __restrict__ pend, int32_t* __restrict__ qn, int64_t* __restrict__ qdeg_n, Counters* cnt, int64_t thr,
        int64_t lo, int64_t n_local, int64_t* __restrict__ rbest, uint64_t* __restrict__ rmark,
        long long* __restrict__ track) {
    __shared__ AppendLds sh;
    unsigned long long mf = 0;
    long long tmin = kInfLL;
    if (blockIdx.x == 0 && threadIdx.x == 0) cnt->red[1] = static_cast<unsigned long long>(qpre[qlen]);   // work done
    for_each_queue_edge(q, qpre, qlen, [&](bool valid, int32_t qentry, int64_t o) {
        bool take = false;
        int32_t v = 0;
        int64_t vdeg = 0;
        if (valid) {
            const uint32_t qe = static_cast<uint32_t>(qentry);
            const int64_t u = static_cast<int64_t>(qe & ~kHeavyFlag);
            const int64_t e = ((qe & kHeavyFlag) ? light[u] : off[u]) + o;
            const int32_t t = adj[e], w = wt[e];
            const int64_t mu = msg[u];
            if (w == kMissingWeight) {
                atomicOr(&cnt->err, 1ULL);              // edge.value(weight) on a missing key
            } else if (dist[u] < mu) {
                // improved during this phase: pending again, relaxes with the better distance
            } else {
                const int64_t cand = mu + static_cast<int64_t>(w);
                const int64_t tl = kPart ? static_cast<int64_t>(t) - lo : static_cast<int64_t>(t);
                if (!kPart || (tl >= 0 && tl < n_local)) {
                    if (relax_owned(dist, pend, tl, cand, thr, tmin)) {
                        take = true;
                        v = static_cast<int32_t>(tl);
                        vdeg = light_degree(off, light, tl);
                    }
                } else if (cand < rbest[t]) {
                    const long long old = atomicMin(reinterpret_cast<long long*>(&rbest[t]), static_cast<long long>(cand));
                    if (cand < old) {
                        const uint64_t bit = 1ULL << (t & 63);
                        if (!(rmark[t >> 6] & bit)) atomicOr(reinterpret_cast<unsigned long long*>(&rmark[t >> 6]), bit);
                    }
                }
            }
        }
        block_append(take, v, vdeg, qn, qdeg_n, cnt, sh, mf);
    });
    block_flush(cnt, sh, mf);
    if (track) block_fold_min(tmin, track);
}

// ds_relax_ws<true> in stages (the structure of delta_loop.hip's ds_relax_dev): each thread's
// kEdgesPerThread entries go through the queue search, the list / snapshot loads, the target
// loads and the atomics stage by stage, so that each stage's loads are in flight together
// (one entry at a time left every thread waiting out the search -> list -> distance -> atomic
// chain once per entry).  The tile's takes are appended with one reservation per block; an
// owned target's improvement that stays pending outside the queue is folded into track[0],
// a remote target's goes to rbest / rmark.
__device__ __forceinline__ int64_t wave_incl_scan(int64_t x) {
    for (int o = 1; o < 64; o <<= 1) {
        const int64_t y = __shfl_up(x, o, 64);
        if (lane() >= o) x += y;
    }
    return x;
}

__global__ void __launch_bounds__(kBlock) ds_relax_ws_staged(const int64_t* __restrict__ off,
        const int32_t* __restrict__ adj, const int32_t* __restrict__ wt, const int64_t* __restrict__ light,
        const int32_t* __restrict__ q, const int64_t* __restrict__ qpre, int64_t qlen, const int64_t* __restrict__ msg,
        int64_t* __restrict__ dist, uint64_t* __restrict__ pend, int32_t* __restrict__ qn, int64_t* __restrict__ qdeg_n,
        Counters* cnt, int64_t thr, int64_t lo, int64_t n_local, int64_t* __restrict__ rbest,
        uint64_t* __restrict__ rmark, long long* __restrict__ track) {
    __shared__ int64_t s_pre[kLdsEntries];
    __shared__ int32_t s_q[kLdsEntries];
    __shared__ int64_t s_lo, s_hi;
    __shared__ int64_t s_c[kWavesPerBlock];
    __shared__ unsigned long long s_base;
    const int64_t total = qpre[qlen];
    if (blockIdx.x == 0 && threadIdx.x == 0) cnt->red[1] = static_cast<unsigned long long>(total);   // work done
    long long tmin = kInfLL;
    bool bad = false;
    unsigned long long mf = 0;
    const int wave = threadIdx.x >> 6;
    const int64_t ntiles = (total + kTileEdges - 1) / kTileEdges;
    for (int64_t tile = blockIdx.x; tile < ntiles; tile += gridDim.x) {
        const int64_t t0 = tile * kTileEdges;
        const int64_t t1 = min(total, t0 + kTileEdges);
        tile_bounds(qpre, qlen, t0, t1, s_lo, s_hi);   // lo = last i with qpre[i] <= t0; hi = last with <= t1-1
        __syncthreads();
        const int64_t qlo = s_lo, qhi = s_hi;
        const int64_t span = qhi - qlo + 1;
        const bool in_lds = span + 1 <= kLdsEntries;
        if (in_lds) {
            for (int64_t i = threadIdx.x; i <= span; i += kBlock) {
                s_pre[i] = qpre[qlo + i];
                if (i < span) s_q[i] = q[qlo + i];
            }
        }
        __syncthreads();
        int64_t u[kEdgesPerThread], e[kEdgesPerThread];
#pragma unroll
        for (int k = 0; k < kEdgesPerThread; ++k) {           // 1: owning queue entry
            const int64_t j = t0 + k * kBlock + threadIdx.x;
            u[k] = -1;
            e[k] = 0;
            if (j >= t1) continue;
            int32_t qe;
            int64_t start;
            if (in_lds) {
                int64_t a = 0, b = span;
                while (b - a > 1) { const int64_t m = (a + b) >> 1; if (s_pre[m] <= j) a = m; else b = m; }
                qe = s_q[a]; start = s_pre[a];
            } else {
                int64_t a = qlo, b = qhi + 1;
                while (b - a > 1) { const int64_t m = (a + b) >> 1; if (qpre[m] <= j) a = m; else b = m; }
                qe = q[a]; start = qpre[a];
            }
            const uint32_t ue = static_cast<uint32_t>(qe);
            u[k] = static_cast<int64_t>(ue & ~kHeavyFlag);
            e[k] = ((ue & kHeavyFlag) ? light[u[k]] : off[u[k]]) + (j - start);
        }
        int32_t t[kEdgesPerThread], w[kEdgesPerThread];
        int64_t mu[kEdgesPerThread], du[kEdgesPerThread];
#pragma unroll
        for (int k = 0; k < kEdgesPerThread; ++k) {           // 2: entry, the source's snapshot
            if (u[k] < 0) continue;
            t[k] = adj[e[k]];
            w[k] = wt[e[k]];
            mu[k] = msg[u[k]];
            du[k] = dist[u[k]];
        }
        int64_t cand[kEdgesPerThread], dt[kEdgesPerThread], tl[kEdgesPerThread];
#pragma unroll
        for (int k = 0; k < kEdgesPerThread; ++k) {           // 3: the targets' current bests
            cand[k] = -1;
            if (u[k] < 0) continue;
            if (w[k] == kMissingWeight) { bad = true; continue; }     // edge.value(weight) on a missing key
            if (du[k] < mu[k]) continue;     // u improved during this phase: pending again, relaxes later
            cand[k] = mu[k] + static_cast<int64_t>(w[k]);
            tl[k] = static_cast<int64_t>(t[k]) - lo;
            dt[k] = (tl[k] >= 0 && tl[k] < n_local) ? dist[tl[k]] : rbest[t[k]];
        }
        int32_t tv[kEdgesPerThread];
        int64_t td[kEdgesPerThread];
        int64_t ntake = 0, dtake = 0;
#pragma unroll
        for (int k = 0; k < kEdgesPerThread; ++k) {           // 4: min, pending bit, take
            tv[k] = -1;
            td[k] = 0;
            if (cand[k] < 0 || cand[k] >= dt[k]) continue;    // a stale (larger) read only costs an atomic
            if (tl[k] >= 0 && tl[k] < n_local) {
                const int64_t v = tl[k];
                const long long old = atomicMin(reinterpret_cast<long long*>(&dist[v]), static_cast<long long>(cand[k]));
                if (cand[k] >= old) continue;
                const uint64_t bit = 1ULL << (v & 63);
                const unsigned long long ob = atomicOr(reinterpret_cast<unsigned long long*>(&pend[v >> 6]), bit);
                if (!(ob & bit) && cand[k] < thr) {
                    tv[k] = static_cast<int32_t>(v);
                    td[k] = light_degree(off, light, v);
                    ++ntake;
                    dtake += td[k];
                } else if (cand[k] < tmin) {
                    tmin = cand[k];
                }
            } else {
                const int64_t g = t[k];
                const long long old = atomicMin(reinterpret_cast<long long*>(&rbest[g]), static_cast<long long>(cand[k]));
                if (cand[k] < old) {
                    const uint64_t bit = 1ULL << (g & 63);
                    if (!(rmark[g >> 6] & bit)) atomicOr(reinterpret_cast<unsigned long long*>(&rmark[g >> 6]), bit);
                }
            }
        }
        // the tile's takes: one reservation per block (block-uniform)
        const int64_t inc = wave_incl_scan(ntake);
        if (lane() == 63) s_c[wave] = inc;
        __syncthreads();
        if (threadIdx.x == 0) {
            int64_t tc = 0;
            for (int x = 0; x < kWavesPerBlock; ++x) { const int64_t c = s_c[x]; s_c[x] = tc; tc += c; }
            s_base = tc ? atomicAdd(&cnt->qlen, static_cast<unsigned long long>(tc)) : 0ULL;
        }
        __syncthreads();
        if (ntake) {
            unsigned long long slot = s_base + static_cast<unsigned long long>(s_c[wave] + inc - ntake);
#pragma unroll
            for (int k = 0; k < kEdgesPerThread; ++k)
                if (tv[k] >= 0) {
                    qn[slot] = tv[k];
                    qdeg_n[slot] = td[k];
                    ++slot;
                }
            mf += static_cast<unsigned long long>(dtake);
        }
        __syncthreads();
    }
    if (__ballot(bad) && lane() == 0) atomicOr(&cnt->err, 1ULL);
    count_flush(cnt, 0ULL, mf);
    if (track) block_fold_min(tmin, track);
}

// Next queue from the bitmaps (one wave per 64-vertex word), clearing what it takes: pending
// vertices with dist < thr (the new bucket's near queue, light degrees) and every member of
// the settled bucket with heavy entries (flagged, heavy degrees).
__global__ void __launch_bounds__(kBlock) ds_extract_ws(const int64_t* __restrict__ off,
        const int64_t* __restrict__ light, uint64_t* __restrict__ pend, uint64_t* __restrict__ member, int64_t n,
        const int64_t* __restrict__ dist, int64_t thr, int32_t* __restrict__ qn, int64_t* __restrict__ qdeg,
        Counters* cnt, long long* __restrict__ track) {
    const int64_t words = (n + 63) >> 6;
    long long rest = kInfLL;                    // smallest distance left pending (>= thr)
    auto probe = [&](int64_t wd, Take* t, bool commit) -> bool {
        const uint64_t pb = pend[wd];                            // uniform across the wave
        const uint64_t mb = member[wd];
        const int64_t v = (wd << 6) + lane();
        if (!(pb | mb)) {                                        // uniform: no loads for an empty word
            t[0] = {false, 0, 0};
            t[1] = {false, 0, 0};
            return false;
        }
        const bool pbit = (pb >> lane()) & 1ULL;
        const long long dv = pbit ? static_cast<long long>(dist[v]) : kInfLL;
        const bool lt = pbit && dv < thr;
        if (pbit && !lt && dv < rest) rest = dv;
        const bool mine = mb && ((mb >> lane()) & 1ULL);
        const int64_t hdeg = mine ? off[v + 1] - light[v] : 0;
        const unsigned long long tm = __ballot(lt);
        if (commit && lane() == 0) {
            if (tm) pend[wd] = pb & ~tm;
            if (mb) member[wd] = 0;
        }
        t[0] = {lt, static_cast<int32_t>(v), lt ? light_degree(off, light, v) : 0};
        t[1] = {hdeg > 0, static_cast<int32_t>(static_cast<uint32_t>(v) | kHeavyFlag), hdeg};
        return tm || mb;
    };
    chunk_extract<2>(words, probe, qn, qdeg, cnt);
    if (track) block_fold_min(rest, track);
}

// ---- light/heavy split of a partitioned load (device-assembled: no host lists to sort).
// The split only needs every row's light entries (w < delta) first, so instead of the one-GPU
// load's full weight sort, each row is stably partitioned at delta on the device, once per
// bucket width: off = the concatenated push lists' offsets, light[v] = end of v's light run.
__global__ void ds_ws_off(View push, int64_t n, int64_t* __restrict__ off) {
    for (int64_t v = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; v <= n; v += (int64_t)gridDim.x * blockDim.x)
        off[v] = push.off0[v] + (push.nlists > 1 ? push.off1[v] : 0);
}

// One wave per row: a counting pass (ballots) for the light total, then a writing pass with
// each entry's rank among its kind from the ballots (stable: list order kept on both sides).
__global__ void __launch_bounds__(kBlock) ds_split_rows(View push, const int64_t* __restrict__ off, int64_t n,
        int64_t delta, int32_t* __restrict__ adj, int32_t* __restrict__ wt, int64_t* __restrict__ light) {
    const int64_t waves = (static_cast<int64_t>(gridDim.x) * blockDim.x) >> 6;
    const unsigned long long below = (1ULL << lane()) - 1ULL;
    for (int64_t v = (blockIdx.x * (int64_t)blockDim.x + threadIdx.x) >> 6; v < n; v += waves) {
        const int64_t deg = push_degree(push, v);
        int64_t nl = 0;
        for (int64_t c = 0; c < deg; c += 64) {
            int32_t t = 0, w = 0;
            if (c + lane() < deg) entry_at(push, v, c + lane(), t, w);
            nl += __popcll(__ballot(c + lane() < deg && static_cast<int64_t>(w) < delta));
        }
        const int64_t base = off[v];
        int64_t li = 0, hi = 0;
        for (int64_t c = 0; c < deg; c += 64) {
            const bool in = c + lane() < deg;
            int32_t t = 0, w = 0;
            if (in) entry_at(push, v, c + lane(), t, w);
            const bool lt = in && static_cast<int64_t>(w) < delta;
            const unsigned long long bl = __ballot(lt), bh = __ballot(in && !lt);
            if (in) {
                const int64_t p = lt ? base + li + __popcll(bl & below) : base + nl + hi + __popcll(bh & below);
                adj[p] = t;
                wt[p] = w;
            }
            li += __popcll(bl);
            hi += __popcll(bh);
        }
        if (lane() == 0) light[v] = base + nl;
    }
}

// Pending minimum / count (red[0], red[1]) and the settled bucket's members left (red2).
__global__ void __launch_bounds__(kBlock) ds_pending_min_ws(const uint64_t* __restrict__ pend,
        const uint64_t* __restrict__ member, int64_t words, const int64_t* __restrict__ dist, Counters* cnt) {
    // one wave per 64-vertex word, lane = vertex: the pending vertices' distances load
    // coalesced and in parallel (a thread per word walked its set bits one dependent load at
    // a time); 4 words per trip keep their loads in flight together
    unsigned long long mn = ~0ULL >> 1, count = 0, mem = 0;
    const int64_t nw = (static_cast<int64_t>(gridDim.x) * blockDim.x) >> 6;
    const int64_t w0 = (blockIdx.x * (int64_t)blockDim.x + threadIdx.x) >> 6;
    for (int64_t wd = w0; wd < words; wd += 4 * nw) {
        uint64_t b[4], m[4];
#pragma unroll
        for (int u = 0; u < 4; ++u) {
            const int64_t w = wd + u * nw;
            b[u] = w < words ? pend[w] : 0;
            m[u] = w < words ? member[w] : 0;
        }
        unsigned long long d[4];
#pragma unroll
        for (int u = 0; u < 4; ++u) {
            // b[u] is wave-uniform: an empty word issues no load at all (without the branch the
            // compiler may load dist for every lane of every word, a full pass over dist)
            d[u] = ~0ULL >> 1;
            if (b[u] != 0 && ((b[u] >> lane()) & 1ULL)) d[u] = static_cast<unsigned long long>(dist[((wd + u * nw) << 6) + lane()]);
        }
#pragma unroll
        for (int u = 0; u < 4; ++u) {
            mn = d[u] < mn ? d[u] : mn;
            if (lane() == 0) { count += __popcll(b[u]); mem += __popcll(m[u]); }
        }
    }
    for (int off = 32; off > 0; off >>= 1) {
        const unsigned long long o = __shfl_xor(mn, off, 64);
        mn = o < mn ? o : mn;
        count += __shfl_xor(count, off, 64);
        mem += __shfl_xor(mem, off, 64);
    }
    __shared__ unsigned long long s_mn[kBlock / 64], s_ct[kBlock / 64], s_mb[kBlock / 64];
    if (lane() == 0) { s_mn[threadIdx.x >> 6] = mn; s_ct[threadIdx.x >> 6] = count; s_mb[threadIdx.x >> 6] = mem; }
    __syncthreads();
    if (threadIdx.x == 0) {
        for (int w = 1; w < kBlock / 64; ++w) { mn = s_mn[w] < mn ? s_mn[w] : mn; count += s_ct[w]; mem += s_mb[w]; }
        if (count) {
            atomicMin(&cnt->red[0], mn);
            atomicAdd(&cnt->red[1], count);
        }
        if (mem) atomicAdd(&cnt->red2, mem);
    }
}

// Minimum distance over the pending vertices (into cnt->red[0], pre-set to a large value)
// and their number (cnt->red[1]).
__global__ void __launch_bounds__(kBlock) ds_pending_min(const uint64_t* __restrict__ pend, int64_t words,
                                                         const int64_t* __restrict__ dist, Counters* cnt) {
    unsigned long long mn = ~0ULL >> 1, count = 0;
    for (int64_t wd = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; wd < words; wd += (int64_t)gridDim.x * blockDim.x) {
        uint64_t b = pend[wd];
        count += __popcll(b);
        while (b) {
            const int r = __ffsll(static_cast<long long>(b)) - 1;
            b &= b - 1;
            const unsigned long long d = static_cast<unsigned long long>(dist[(wd << 6) + r]);
            mn = d < mn ? d : mn;
        }
    }
    for (int off = 32; off > 0; off >>= 1) {
        const unsigned long long o = __shfl_xor(mn, off, 64);
        mn = o < mn ? o : mn;
        count += __shfl_xor(count, off, 64);
    }
    __shared__ unsigned long long s_mn[kBlock / 64], s_ct[kBlock / 64];
    if (lane() == 0) { s_mn[threadIdx.x >> 6] = mn; s_ct[threadIdx.x >> 6] = count; }
    __syncthreads();
    if (threadIdx.x == 0) {                              // one pair of atomics per block
        for (int w = 1; w < kBlock / 64; ++w) { mn = s_mn[w] < mn ? s_mn[w] : mn; count += s_ct[w]; }
        if (count) {
            atomicMin(&cnt->red[0], mn);
            atomicAdd(&cnt->red[1], count);
        }
    }
}

// Next near queue: pending vertices with dist < thr (one wave per 64-vertex word).
// track (partitioned): the smallest distance left pending is folded into track[0].
__global__ void __launch_bounds__(kBlock) ds_extract(View push, uint64_t* __restrict__ pend, int64_t n,
        const int64_t* __restrict__ dist, int64_t thr, int32_t* __restrict__ qn, int64_t* __restrict__ qdeg,
        Counters* cnt, long long* __restrict__ track) {
    const int64_t words = (n + 63) >> 6;
    long long rest = kInfLL;
    auto probe = [&](int64_t wd, Take* t, bool commit) -> bool {
        const uint64_t b = pend[wd];                             // uniform across the wave
        const int64_t v = (wd << 6) + lane();
        if (!b) {                                                // uniform: no loads for an empty word
            t[0] = {false, 0, 0};
            return false;
        }
        const bool pbit = (b >> lane()) & 1ULL;
        const long long dv = pbit ? static_cast<long long>(dist[v]) : kInfLL;
        const bool take = pbit && dv < thr;
        if (pbit && !take && dv < rest) rest = dv;
        const unsigned long long tm = __ballot(take);
        if (commit && lane() == 0 && tm) pend[wd] = b & ~tm;
        t[0] = {take, static_cast<int32_t>(v), take ? push_degree(push, v) : 0};
        return tm != 0;
    };
    chunk_extract<1>(words, probe, qn, qdeg, cnt);
    if (track) block_fold_min(rest, track);
}

// Partitioned: marked remote targets per owner rank (rank r owns words [r*wpr, (r+1)*wpr)).
__global__ void ds_mark_count(const uint64_t* __restrict__ rmark, int64_t words, int64_t wpr,
                              unsigned long long* __restrict__ counts) {
    for (int64_t w = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; w < words; w += (int64_t)gridDim.x * blockDim.x) {
        const uint64_t b = rmark[w];
        if (b) atomicAdd(&counts[w / wpr], static_cast<unsigned long long>(__popcll(b)));
    }
}

// Pack (owner-local id, distance) pairs rank-major from offs[r]; clears the marks.
__global__ void ds_mark_pack(uint64_t* __restrict__ rmark, int64_t words, int64_t wpr, int64_t n_local,
                             const int64_t* __restrict__ rbest, const unsigned long long* __restrict__ offs,
                             unsigned long long* __restrict__ cursor, int64_t* __restrict__ send) {
    for (int64_t w = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; w < words; w += (int64_t)gridDim.x * blockDim.x) {
        uint64_t b = rmark[w];
        if (!b) continue;
        rmark[w] = 0;
        const int64_t r = w / wpr;
        unsigned long long pos = offs[r] + atomicAdd(&cursor[r], static_cast<unsigned long long>(__popcll(b)));
        while (b) {
            const int k = __ffsll(static_cast<long long>(b)) - 1;
            b &= b - 1;
            const int64_t v = (w << 6) + k;
            send[2 * pos] = v - r * n_local;
            send[2 * pos + 1] = rbest[v];
            ++pos;
        }
    }
}

// Partitioned loop state without a bitmap scan (the idea of delta_loop.hip's decision):
//   track[0] <= the smallest distance of a pending vertex outside the near queue.  An
//            extraction sets it to the smallest distance it leaves pending; every later
//            improvement that leaves its vertex pending outside the queue mins its distance in.
//            It can be stale-low (that vertex was queued and committed since): then the next
//            extraction takes nothing, track[0] is exact again, and the loop goes on, one
//            extra exchange later, to the same converged distances.
//   track[1] = 1 once a bucket member was marked since the last extraction (light/heavy).
// Reset right before every extraction.
__global__ void ds_track_reset(long long* __restrict__ track) {
    if (threadIdx.x == 0) { track[0] = kInfLL; track[1] = 0; }
}

// After the header all-to-all: own[4r..4r+4) = this rank's header to r, recv[4r..) = r's
// header to this rank {pair elements, near-queue length, track[0], track[1]}.  out (2W + 3
// words, read by the host in one go): pair elements sent to / received from each rank, then
// the global near-queue length, pending minimum and -(ranks with members).
// host (may be null): the same words also go to the host-mapped counter page, then the sequence
// word (publish_words' protocol) — the fold and its publish in one launch.
__global__ void ds_header_fold(const int64_t* __restrict__ own, const int64_t* __restrict__ recv, int nranks,
                               int64_t* __restrict__ out, unsigned long long* host, unsigned long long seq) {
    if (threadIdx.x != 0) return;
    int64_t gq = 0, pm = INT64_MAX, mem = 0;
    for (int r = 0; r < nranks; ++r) {
        out[r] = own[4 * r];
        out[nranks + r] = recv[4 * r];
        gq += recv[4 * r + 1];
        pm = recv[4 * r + 2] < pm ? recv[4 * r + 2] : pm;
        mem -= recv[4 * r + 3];
    }
    out[2 * nranks] = gq;
    out[2 * nranks + 1] = pm;
    out[2 * nranks + 2] = mem;
    if (!host) return;
    for (int r = 0; r < nranks; ++r) {
        __hip_atomic_store(&host[r], static_cast<unsigned long long>(own[4 * r]), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        __hip_atomic_store(&host[nranks + r], static_cast<unsigned long long>(recv[4 * r]), __ATOMIC_RELAXED,
                           __HIP_MEMORY_SCOPE_SYSTEM);
    }
    __hip_atomic_store(&host[2 * nranks], static_cast<unsigned long long>(gq), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    __hip_atomic_store(&host[2 * nranks + 1], static_cast<unsigned long long>(pm), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    __hip_atomic_store(&host[2 * nranks + 2], static_cast<unsigned long long>(mem), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    __threadfence_system();
    __hip_atomic_store(&host[kCounterWords], seq, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
}

// The exchange header on the device (no host round trip): offs[r] = the pack offset of rank r's
// pairs; header to r = {pair elements sent to r, this rank's near-queue length, track[0],
// track[1]} (sizes[4r..4r+4)).
__global__ void ds_mark_sizes(unsigned long long* __restrict__ counts, int nranks, int64_t qlen,
                              unsigned long long* __restrict__ offs, unsigned long long* __restrict__ cursor,
                              const long long* __restrict__ track, int64_t* __restrict__ sizes) {
    if (threadIdx.x != 0) return;
    unsigned long long acc = 0;
    const int64_t pm = track[0], mem = track[1];
    for (int r = 0; r < nranks; ++r) {
        const unsigned long long c = counts[r];
        offs[r] = acc;
        acc += c;
        sizes[4 * r] = 2 * static_cast<int64_t>(c);
        sizes[4 * r + 1] = qlen;
        sizes[4 * r + 2] = pm;
        sizes[4 * r + 3] = mem;
        counts[r] = 0;              // ready for the next phase's count; the pack's cursors start at 0
        cursor[r] = 0;
    }
}

// Owner side of the exchange: min the received (local id, distance) pairs into dist with
// the pending / near-queue rule of ds_relax.
// ws_off / light set (light/heavy split): a queued vertex carries its light degree.
__global__ void __launch_bounds__(kBlock) ds_apply(View push, const int64_t* __restrict__ recv, int64_t npairs,
        int64_t* __restrict__ dist, uint64_t* __restrict__ pend, int32_t* __restrict__ qn,
        int64_t* __restrict__ qdeg_n, Counters* cnt, int64_t thr, const int64_t* __restrict__ ws_off,
        const int64_t* __restrict__ light, long long* __restrict__ track) {
    __shared__ AppendLds sh;
    unsigned long long mf = 0;
    long long tmin = kInfLL;
    const int64_t stride = (int64_t)gridDim.x * blockDim.x;
    for (int64_t base = (int64_t)blockIdx.x * blockDim.x; base < npairs; base += stride) {   // block-uniform trips
        const int64_t i = base + threadIdx.x;
        bool take = false;
        int32_t v = 0;
        int64_t vdeg = 0;
        if (i < npairs) {
            const int64_t vl = recv[2 * i];
            if (relax_owned(dist, pend, vl, recv[2 * i + 1], thr, tmin)) {
                take = true;
                v = static_cast<int32_t>(vl);
                vdeg = light ? light_degree(ws_off, light, vl) : push_degree(push, vl);
            }
        }
        block_append(take, v, vdeg, qn, qdeg_n, cnt, sh, mf);
    }
    block_flush(cnt, sh, mf);
    if (track) block_fold_min(tmin, track);
}

inline int grid_for(int64_t work, int cap) {
    int64_t g = (work + kBlock - 1) / kBlock;
    if (g < 1) g = 1;
    if (g > cap) g = cap;
    return static_cast<int>(g);
}

}  // namespace

static long long env_i64_d(const char* name, long long dflt) {
    const char* e = std::getenv(name);
    return e ? std::atoll(e) : dflt;
}

hipError_t k_ds_seed(const View& push, int64_t* dist, int32_t* q, int64_t* qdeg, int64_t seed, hipStream_t s) {
    ds_seed<<<1, 64, 0, s>>>(push, dist, q, qdeg, seed);
    return hipGetLastError();
}
hipError_t k_ds_commit(const int32_t* q, int64_t qlen, const int64_t* dist, int64_t* msg, uint64_t* pend, hipStream_t s) {
    ds_commit<<<grid_for(qlen, 2048), kBlock, 0, s>>>(q, qlen, dist, msg, pend);
    return hipGetLastError();
}
hipError_t k_ds_relax(const View& push, const int32_t* q, const int64_t* qpre, int64_t qlen, const int64_t* msg,
                      int64_t* dist, uint64_t* pend, int32_t* qn, int64_t* qdeg_n, Counters* cnt, int weighted,
                      int64_t thr, hipStream_t s) {
    ds_relax<false><<<256 * 8, kBlock, 0, s>>>(push, q, qpre, qlen, msg, dist, pend, qn, qdeg_n, cnt, weighted, thr,
                                              0, 0, nullptr, nullptr, nullptr);
    return hipGetLastError();
}
hipError_t k_ds_relax_part(const View& push, const int32_t* q, const int64_t* qpre, int64_t qlen, const int64_t* msg,
                           int64_t* dist, uint64_t* pend, int32_t* qn, int64_t* qdeg_n, Counters* cnt, int weighted,
                           int64_t thr, int64_t lo, int64_t n_local, int64_t* rbest, uint64_t* rmark, long long* track,
                           hipStream_t s) {
    ds_relax<true><<<256 * 8, kBlock, 0, s>>>(push, q, qpre, qlen, msg, dist, pend, qn, qdeg_n, cnt, weighted, thr,
                                             lo, n_local, rbest, rmark, track);
    return hipGetLastError();
}
hipError_t k_ds_light_end(const DevCsr& ws, int64_t delta, int64_t n, int64_t* light, hipStream_t s) {
    ds_light_end<<<grid_for(n, 8192), kBlock, 0, s>>>(ws.off, ws.w, delta, n, light);
    return hipGetLastError();
}
hipError_t k_ds_seed_ws(const DevCsr& ws, const int64_t* light, int64_t* dist, int32_t* q, int64_t* qdeg, int64_t seed,
                        hipStream_t s) {
    ds_seed_ws<<<1, 64, 0, s>>>(ws.off, light, dist, q, qdeg, seed);
    return hipGetLastError();
}
hipError_t k_ds_commit_ws(const int32_t* q, int64_t qlen, const int64_t* dist, int64_t* msg, uint64_t* pend,
                          uint64_t* member, int64_t* qdeg, Counters* cnt, hipStream_t s, long long* track) {
    ds_commit_ws<<<grid_for(qlen, 2048), kBlock, 0, s>>>(q, qlen, dist, msg, pend, member, qdeg, cnt, track);
    return hipGetLastError();
}
hipError_t k_ds_relax_ws(const DevCsr& ws, const int64_t* light, const int32_t* q, const int64_t* qpre, int64_t qlen,
                         const int64_t* msg, int64_t* dist, uint64_t* pend, int32_t* qn, int64_t* qdeg_n, Counters* cnt,
                         int64_t thr, hipStream_t s) {
    ds_relax_ws<false><<<256 * 8, kBlock, 0, s>>>(ws.off, ws.adj, ws.w, light, q, qpre, qlen, msg, dist, pend, qn, qdeg_n,
                                                  cnt, thr, 0, 0, nullptr, nullptr, nullptr);
    return hipGetLastError();
}
hipError_t k_ds_relax_ws_part(const DevCsr& ws, const int64_t* light, const int32_t* q, const int64_t* qpre, int64_t qlen,
                              const int64_t* msg, int64_t* dist, uint64_t* pend, int32_t* qn, int64_t* qdeg_n,
                              Counters* cnt, int64_t thr, int64_t lo, int64_t n_local, int64_t* rbest, uint64_t* rmark,
                              long long* track, hipStream_t s) {
    static const bool staged = env_i64_d("TGO_DS_PART_STAGED", 1) != 0;     // A/B: 0 = one entry at a time
    if (staged)
        ds_relax_ws_staged<<<256 * 8, kBlock, 0, s>>>(ws.off, ws.adj, ws.w, light, q, qpre, qlen, msg, dist, pend, qn,
                                                      qdeg_n, cnt, thr, lo, n_local, rbest, rmark, track);
    else
        ds_relax_ws<true><<<256 * 8, kBlock, 0, s>>>(ws.off, ws.adj, ws.w, light, q, qpre, qlen, msg, dist, pend, qn,
                                                     qdeg_n, cnt, thr, lo, n_local, rbest, rmark, track);
    return hipGetLastError();
}
hipError_t k_ds_split_rows(const View& push, int64_t n, int64_t delta, DevCsr& ws, int64_t* light, hipStream_t s) {
    ds_ws_off<<<grid_for(n + 1, 4096), kBlock, 0, s>>>(push, n, ws.off);
    ds_split_rows<<<grid_for(n * 64, 8192), kBlock, 0, s>>>(push, ws.off, n, delta, ws.adj, ws.w, light);
    return hipGetLastError();
}
hipError_t k_ds_extract_ws(const DevCsr& ws, const int64_t* light, uint64_t* pend, uint64_t* member, int64_t n,
                           const int64_t* dist, int64_t thr, int32_t* qn, int64_t* qdeg, Counters* cnt, hipStream_t s,
                           long long* track) {
    const int64_t words = (n + 63) / 64;
    ds_extract_ws<<<extract_grid(words), kBlock, 0, s>>>(ws.off, light, pend, member, n, dist, thr, qn, qdeg, cnt, track);
    return hipGetLastError();
}
hipError_t k_ds_pending_min_ws(const uint64_t* pend, const uint64_t* member, int64_t words, const int64_t* dist,
                               Counters* cnt, hipStream_t s) {
    ds_pending_min_ws<<<grid_for(words * 8, 2048), kBlock, 0, s>>>(pend, member, words, dist, cnt);
    return hipGetLastError();
}
hipError_t k_ds_pending_min(const uint64_t* pend, int64_t words, const int64_t* dist, Counters* cnt, hipStream_t s) {
    ds_pending_min<<<grid_for(words, 1024), kBlock, 0, s>>>(pend, words, dist, cnt);
    return hipGetLastError();
}
hipError_t k_ds_track_reset(long long* track, hipStream_t s) {
    ds_track_reset<<<1, 64, 0, s>>>(track);
    return hipGetLastError();
}
hipError_t k_ds_header_fold(const int64_t* own, const int64_t* recv, int nranks, int64_t* out, hipStream_t s,
                            unsigned long long* host, unsigned long long seq) {
    if (host && 2 * nranks + 3 > kCounterWords) return hipErrorInvalidValue;
    ds_header_fold<<<1, 64, 0, s>>>(own, recv, nranks, out, host, seq);
    return hipGetLastError();
}
hipError_t k_ds_extract(const View& push, uint64_t* pend, int64_t n, const int64_t* dist, int64_t thr, int32_t* qn,
                        int64_t* qdeg, Counters* cnt, hipStream_t s, long long* track) {
    const int64_t words = (n + 63) / 64;
    ds_extract<<<extract_grid(words), kBlock, 0, s>>>(push, pend, n, dist, thr, qn, qdeg, cnt, track);
    return hipGetLastError();
}
hipError_t k_ds_mark_count(const uint64_t* rmark, int64_t words, int64_t wpr, unsigned long long* counts, hipStream_t s) {
    ds_mark_count<<<grid_for(words, 4096), kBlock, 0, s>>>(rmark, words, wpr, counts);
    return hipGetLastError();
}
hipError_t k_ds_mark_pack(uint64_t* rmark, int64_t words, int64_t wpr, int64_t n_local, const int64_t* rbest,
                          const unsigned long long* offs, unsigned long long* cursor, int64_t* send, hipStream_t s) {
    ds_mark_pack<<<grid_for(words, 4096), kBlock, 0, s>>>(rmark, words, wpr, n_local, rbest, offs, cursor, send);
    return hipGetLastError();
}
hipError_t k_ds_mark_sizes(unsigned long long* counts, int nranks, int64_t qlen, unsigned long long* offs,
                           unsigned long long* cursor, const long long* track, int64_t* sizes, hipStream_t s) {
    ds_mark_sizes<<<1, 64, 0, s>>>(counts, nranks, qlen, offs, cursor, track, sizes);
    return hipGetLastError();
}
hipError_t k_ds_apply(const View& push, const int64_t* recv, int64_t npairs, int64_t* dist, uint64_t* pend, int32_t* qn,
                      int64_t* qdeg_n, Counters* cnt, int64_t thr, const int64_t* ws_off, const int64_t* light,
                      long long* track, hipStream_t s) {
    ds_apply<<<grid_for(npairs, 4096), kBlock, 0, s>>>(push, recv, npairs, dist, pend, qn, qdeg_n, cnt, thr, ws_off, light,
                                                       track);
    return hipGetLastError();
}

}  // namespace tgo

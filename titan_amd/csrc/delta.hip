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
#include <hip/hip_runtime.h>
#include "frontier.hpp"

namespace tgo {
namespace {

// min(cand) into dist[v] of an owned vertex; true when v has to join the near queue.
__device__ __forceinline__ bool relax_owned(int64_t* dist, uint64_t* pend, int64_t v, int64_t cand, int64_t thr) {
    if (cand >= dist[v]) return false;                  // a stale (larger) read only costs an atomic
    const long long old = atomicMin(reinterpret_cast<long long*>(&dist[v]), static_cast<long long>(cand));
    if (cand >= old) return false;
    const uint64_t bit = 1ULL << (v & 63);
    const unsigned long long ob = atomicOr(reinterpret_cast<unsigned long long*>(&pend[v >> 6]), bit);
    return !(ob & bit) && cand < thr;
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
        int64_t* __restrict__ rbest, uint64_t* __restrict__ rmark) {
    __shared__ AppendLds sh;
    unsigned long long mf = 0;
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
                    if (relax_owned(dist, pend, tl, cand, thr)) {
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
__global__ void ds_commit_ws(const int32_t* __restrict__ q, int64_t qlen, const int64_t* __restrict__ dist,
                             int64_t* __restrict__ msg, uint64_t* __restrict__ pend, uint64_t* __restrict__ member,
                             int64_t* __restrict__ qdeg, Counters* cnt) {
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
        if (!(member[v >> 6] & bit)) atomicOr(reinterpret_cast<unsigned long long*>(&member[v >> 6]), bit);
    }
}

// ds_relax over one weight-sorted list: queue entry u relaxes [off[u], light[u]) or, flagged
// heavy, [light[u], off[u+1]); load-balanced as in ds_relax.
__global__ void __launch_bounds__(kBlock) ds_relax_ws(const int64_t* __restrict__ off, const int32_t* __restrict__ adj,
        const int32_t* __restrict__ wt, const int64_t* __restrict__ light, const int32_t* __restrict__ q,
        const int64_t* __restrict__ qpre, int64_t qlen, const int64_t* __restrict__ msg, int64_t* __restrict__ dist,
        uint64_t* __restrict__ pend, int32_t* __restrict__ qn, int64_t* __restrict__ qdeg_n, Counters* cnt, int64_t thr) {
    __shared__ AppendLds sh;
    unsigned long long mf = 0;
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
            } else if (relax_owned(dist, pend, t, mu + static_cast<int64_t>(w), thr)) {
                take = true;
                v = t;
                vdeg = light_degree(off, light, t);
            }
        }
        block_append(take, v, vdeg, qn, qdeg_n, cnt, sh, mf);
    });
    block_flush(cnt, sh, mf);
}

// Next queue from the bitmaps (one wave per 64-vertex word), clearing what it takes: pending
// vertices with dist < thr (the new bucket's near queue, light degrees) and every member of
// the settled bucket with heavy entries (flagged, heavy degrees).
__global__ void __launch_bounds__(kBlock) ds_extract_ws(const int64_t* __restrict__ off,
        const int64_t* __restrict__ light, uint64_t* __restrict__ pend, uint64_t* __restrict__ member, int64_t n,
        const int64_t* __restrict__ dist, int64_t thr, int32_t* __restrict__ qn, int64_t* __restrict__ qdeg,
        Counters* cnt) {
    const int64_t words = (n + 63) >> 6;
    auto probe = [&](int64_t wd, Take* t, bool commit) -> bool {
        const uint64_t pb = pend[wd];                            // uniform across the wave
        const uint64_t mb = member[wd];
        const int64_t v = (wd << 6) + lane();
        const bool lt = pb && ((pb >> lane()) & 1ULL) && dist[v] < thr;
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
        for (int u = 0; u < 4; ++u)
            d[u] = ((b[u] >> lane()) & 1ULL) ? static_cast<unsigned long long>(dist[((wd + u * nw) << 6) + lane()]) : ~0ULL >> 1;
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
__global__ void __launch_bounds__(kBlock) ds_extract(View push, uint64_t* __restrict__ pend, int64_t n,
        const int64_t* __restrict__ dist, int64_t thr, int32_t* __restrict__ qn, int64_t* __restrict__ qdeg,
        Counters* cnt) {
    const int64_t words = (n + 63) >> 6;
    auto probe = [&](int64_t wd, Take* t, bool commit) -> bool {
        const uint64_t b = pend[wd];                             // uniform across the wave
        const int64_t v = (wd << 6) + lane();
        const bool take = b && ((b >> lane()) & 1ULL) && dist[v] < thr;
        const unsigned long long tm = __ballot(take);
        if (commit && lane() == 0 && tm) pend[wd] = b & ~tm;
        t[0] = {take, static_cast<int32_t>(v), take ? push_degree(push, v) : 0};
        return tm != 0;
    };
    chunk_extract<1>(words, probe, qn, qdeg, cnt);
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

// Owner side of the exchange: min the received (local id, distance) pairs into dist with
// the pending / near-queue rule of ds_relax.
__global__ void __launch_bounds__(kBlock) ds_apply(View push, const int64_t* __restrict__ recv, int64_t npairs,
        int64_t* __restrict__ dist, uint64_t* __restrict__ pend, int32_t* __restrict__ qn,
        int64_t* __restrict__ qdeg_n, Counters* cnt, int64_t thr) {
    __shared__ AppendLds sh;
    unsigned long long mf = 0;
    const int64_t stride = (int64_t)gridDim.x * blockDim.x;
    for (int64_t base = (int64_t)blockIdx.x * blockDim.x; base < npairs; base += stride) {   // block-uniform trips
        const int64_t i = base + threadIdx.x;
        bool take = false;
        int32_t v = 0;
        int64_t vdeg = 0;
        if (i < npairs) {
            const int64_t vl = recv[2 * i];
            if (relax_owned(dist, pend, vl, recv[2 * i + 1], thr)) {
                take = true;
                v = static_cast<int32_t>(vl);
                vdeg = push_degree(push, vl);
            }
        }
        block_append(take, v, vdeg, qn, qdeg_n, cnt, sh, mf);
    }
    block_flush(cnt, sh, mf);
}

inline int grid_for(int64_t work, int cap) {
    int64_t g = (work + kBlock - 1) / kBlock;
    if (g < 1) g = 1;
    if (g > cap) g = cap;
    return static_cast<int>(g);
}

}  // namespace

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
                                              0, 0, nullptr, nullptr);
    return hipGetLastError();
}
hipError_t k_ds_relax_part(const View& push, const int32_t* q, const int64_t* qpre, int64_t qlen, const int64_t* msg,
                           int64_t* dist, uint64_t* pend, int32_t* qn, int64_t* qdeg_n, Counters* cnt, int weighted,
                           int64_t thr, int64_t lo, int64_t n_local, int64_t* rbest, uint64_t* rmark, hipStream_t s) {
    ds_relax<true><<<256 * 8, kBlock, 0, s>>>(push, q, qpre, qlen, msg, dist, pend, qn, qdeg_n, cnt, weighted, thr,
                                             lo, n_local, rbest, rmark);
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
                          uint64_t* member, int64_t* qdeg, Counters* cnt, hipStream_t s) {
    ds_commit_ws<<<grid_for(qlen, 2048), kBlock, 0, s>>>(q, qlen, dist, msg, pend, member, qdeg, cnt);
    return hipGetLastError();
}
hipError_t k_ds_relax_ws(const DevCsr& ws, const int64_t* light, const int32_t* q, const int64_t* qpre, int64_t qlen,
                         const int64_t* msg, int64_t* dist, uint64_t* pend, int32_t* qn, int64_t* qdeg_n, Counters* cnt,
                         int64_t thr, hipStream_t s) {
    ds_relax_ws<<<256 * 8, kBlock, 0, s>>>(ws.off, ws.adj, ws.w, light, q, qpre, qlen, msg, dist, pend, qn, qdeg_n, cnt,
                                           thr);
    return hipGetLastError();
}
hipError_t k_ds_extract_ws(const DevCsr& ws, const int64_t* light, uint64_t* pend, uint64_t* member, int64_t n,
                           const int64_t* dist, int64_t thr, int32_t* qn, int64_t* qdeg, Counters* cnt, hipStream_t s) {
    const int64_t words = (n + 63) / 64;
    ds_extract_ws<<<extract_grid(words), kBlock, 0, s>>>(ws.off, light, pend, member, n, dist, thr, qn, qdeg, cnt);
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
hipError_t k_ds_extract(const View& push, uint64_t* pend, int64_t n, const int64_t* dist, int64_t thr, int32_t* qn,
                        int64_t* qdeg, Counters* cnt, hipStream_t s) {
    const int64_t words = (n + 63) / 64;
    ds_extract<<<extract_grid(words), kBlock, 0, s>>>(push, pend, n, dist, thr, qn, qdeg, cnt);
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
hipError_t k_ds_apply(const View& push, const int64_t* recv, int64_t npairs, int64_t* dist, uint64_t* pend, int32_t* qn,
                      int64_t* qdeg_n, Counters* cnt, int64_t thr, hipStream_t s) {
    ds_apply<<<grid_for(npairs, 4096), kBlock, 0, s>>>(push, recv, npairs, dist, pend, qn, qdeg_n, cnt, thr);
    return hipGetLastError();
}

}  // namespace tgo

// delta_loop.hip — the light/heavy delta-stepping loop of one GPU (delta.hip's
// run_delta_split protocol) driven from the device: no host round trip per phase.
//
// The host-driven loop pays, per phase, a scan launch sized on the host and a host read of
// the next queue's length, and per bucket a pending-minimum pass plus a second read; on
// RMAT-24 that is ~170 host round trips and ~45 full bitmap passes per source, a third of
// the run.  Here every launch reads its sizes from device memory (DsLoop), so the host
// enqueues steps in batches and reads the state once per batch:
//   step = decide (1 thread: is the near queue empty? then the next threshold, or done)
//        + extract (only if decided: next near queue + the settled members' heavy entries)
//        + commit  (snapshot the queue's distances, clear their pending bits, mark members)
//        + relax   (the queue's entries, edge-balanced; appends the next near queue)
// Two changes make this possible:
//   * queue counters are packed (count << kDsCountShift | entries), so ONE atomicAdd per block reserves
//     both the queue slots and the entry range: the appender writes the exclusive prefix of
//     the entries directly (qpre), and no scan pass is needed before the next relax;
//   * the minimum pending distance is never scanned for: it is min(tm, lo), where tm is the
//     smallest improvement since the last extraction that queued nothing (block-reduced in
//     the relax) and lo the smallest distance the last extraction left pending.  tm can be
//     stale-low (its vertex may have been queued since); then the extraction takes nothing,
//     lo becomes exact and the next step's decision is exact — one extra step, same result.
// The converged distances are unique (ShortestDistanceVertexProgram.java:96-130 is a
// Jacobi Bellman-Ford with a min combiner), so this order of the same relaxations reaches
// the same bit-exact result as the host loop and the oracle.
#include <algorithm>
#include <cstdlib>
#include <hip/hip_runtime.h>
#include "frontier.hpp"

namespace tgo {
namespace {

constexpr unsigned long long kEntryMask = (1ULL << kDsCountShift) - 1ULL;
constexpr long long kInf = 0x7FFFFFFFFFFFFFFFLL;
constexpr uint32_t kHeavy = 0x80000000u;

__device__ __forceinline__ int64_t qcount(unsigned long long c) { return static_cast<int64_t>(c >> kDsCountShift); }
__device__ __forceinline__ int64_t qentries(unsigned long long c) { return static_cast<int64_t>(c & kEntryMask); }
__device__ __forceinline__ int64_t light_deg(const int64_t* off, const int64_t* light, int64_t u) { return light[u] - off[u]; }

__device__ __forceinline__ int64_t wave_incl_scan(int64_t x) {
    for (int o = 1; o < 64; o <<= 1) {
        const int64_t y = __shfl_up(x, o, 64);
        if (lane() >= o) x += y;
    }
    return x;
}

__device__ __forceinline__ long long block_min(long long x) {
    __shared__ long long s_min[kWavesPerBlock];
    for (int o = 32; o > 0; o >>= 1) {
        const long long y = __shfl_xor(x, o, 64);
        x = y < x ? y : x;
    }
    if (lane() == 0) s_min[threadIdx.x >> 6] = x;
    __syncthreads();
    long long m = s_min[0];
    for (int w = 1; w < kWavesPerBlock; ++w) m = s_min[w] < m ? s_min[w] : m;
    return m;
}

// Reserve `cnt` queue slots and `deg` entries with one packed atomic; every thread of the
// block calls it with its own (cnt, deg) and gets its first slot and entry offset, in thread
// order.  `qc` is the queue's packed counter.
__device__ __forceinline__ void block_reserve(unsigned long long* qc, int64_t cnt, int64_t deg, int64_t& slot,
                                              int64_t& doff) {
    __shared__ int64_t s_c[kWavesPerBlock], s_d[kWavesPerBlock];
    __shared__ unsigned long long s_base;
    const int wave = threadIdx.x >> 6;
    const int64_t ic = wave_incl_scan(cnt), id = wave_incl_scan(deg);
    if (lane() == 63) { s_c[wave] = ic; s_d[wave] = id; }
    __syncthreads();
    if (threadIdx.x == 0) {
        int64_t tc = 0, td = 0;
        for (int w = 0; w < kWavesPerBlock; ++w) {
            const int64_t c = s_c[w], d = s_d[w];
            s_c[w] = tc; s_d[w] = td;
            tc += c; td += d;
        }
        s_base = tc ? atomicAdd(qc, (static_cast<unsigned long long>(tc) << kDsCountShift) |
                                        static_cast<unsigned long long>(td))
                    : 0ULL;
    }
    __syncthreads();
    slot = qcount(s_base) + s_c[wave] + ic - cnt;
    doff = qentries(s_base) + s_d[wave] + id - deg;
}

// ---------------------------------------------------------------- seed / decide
__global__ void ds_loop_seed(const int64_t* off, const int64_t* light, int64_t* dist, int32_t* q, int64_t* qpre,
                             DsLoop* L, int64_t seed, int64_t delta) {
    if (blockIdx.x != 0) return;
    if (threadIdx.x < kDsMaxBins) L->bc[threadIdx.x] = 0;
    if (threadIdx.x != 0) return;
    if (seed >= 0) {                        // (a partitioned run's rank without the seed: empty queue)
        dist[seed] = 0;
        q[0] = static_cast<int32_t>(seed);
        qpre[0] = 0;
        L->qc[0] = (1ULL << kDsCountShift) | static_cast<unsigned long long>(light_deg(off, light, seed));
    } else {
        L->qc[0] = 0;
    }
    L->qc[1] = 0;
    L->tm = kInf;
    L->lo = kInf;
    L->thr = delta;
    L->extract = 0;
    L->members = 0;
    L->done = 0;
    L->err = 0;
    L->phases = 0;
    L->relaxed = 0;
    L->buckets = 0;
    L->extractions = 0;
    L->bucket = 0;
    L->xbin = -1;
    L->xcount = 0;
    L->xm = 0;
    L->mcount = 0;
    L->overflow = 0;
    L->spill = 0;
    L->full_scans = 0;
    L->xfin = 0;
    L->mlo = 0;
    L->xpull = 0;
    L->pulls = 0;
    L->pbucket = 0;
    L->pcount[0] = L->pcount[1] = 0;
    L->xprev = 0;
    L->cur = 0;
    L->big = 0;
    L->small_steps = 0;
    L->lo_next = kInf;
    L->xnew = 0;
}

__device__ __forceinline__ unsigned long long load_agent(const unsigned long long* p) {
    return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ long long load_agent(const long long* p) {
    return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// The decision at the start of a step: if the near queue `cur` ran dry, the next threshold from min(tm, lo)
// (the host loop's pending minimum), or done when nothing is pending and no settled member
// has heavy entries left to relax.
__device__ void decide_next(DsLoop* L, int cur, int64_t delta) {
    L->extract = 0;
    if (L->done || qcount(load_agent(&L->qc[cur])) != 0) return;
    const long long tm = load_agent(&L->tm);
    const long long mn = tm < L->lo ? tm : L->lo;
    if (mn == kInf && !L->members) { L->done = 1; return; }
    if (mn != kInf) {
        if (mn >= L->thr) L->thr = (mn / delta + 1) * delta;
        L->buckets += 1;
    }
    L->tm = kInf;
    L->lo = kInf;
    L->members = 0;
    L->extract = 1;
    L->extractions += 1;
}

// The binned decision: when the near queue ran dry, the current bucket's pile if it holds
// entries (improvements into the current bucket of vertices that were already pending).
// Otherwise the bucket is finished: its members' distances are final, so their heavy entries
// are taken now, once (a heavy entry cannot reach back into its own bucket), and the members
// become `done`; the threshold moves to the nearest later bucket whose pile holds entries and
// that pile is extracted in the same step; with no such pile only the heavy entries, and with
// no members either the run is done.  A pile that dropped entries is extracted by the bitmap
// scan instead (extract = 1: it takes every member from the member bitmap, none becomes done).
__device__ void decide_bins(DsLoop* L, int cur, int64_t delta, int nbins, int64_t cap, int64_t scan_above,
                            int64_t pull_min) {
    L->extract = 0;
    L->xpull = 0;
    if (L->done || qcount(load_agent(&L->qc[cur])) != 0) return;
    long long k = L->bucket;
    const long long kfin = k;
    int b = static_cast<int>(k % nbins);
    unsigned long long c = load_agent(&L->bc[b]);
    const bool finished = c == 0;
    // the finished range [mlo, kfin] is one bucket: its members are final (done, pull floor)
    const bool single = finished && L->mlo == kfin;
    if (finished) {
        int j = 1;
        while (j < nbins && load_agent(&L->bc[(k + j) % nbins]) == 0) ++j;
        if (j < nbins) {
            k += j;
            // the members' heavy entries pushed in this step reach buckets >= kfin + 1 and are
            // taken into the near queue below the new threshold: buckets kfin+1 .. k merge
            L->mlo = L->mcount > 0 ? kfin + 1 : k;
            L->bucket = k;
            L->thr = (k + 1) * delta;
            L->buckets += 1;
            b = static_cast<int>(k % nbins);
            c = load_agent(&L->bc[b]);
        } else if (L->mcount == 0) {
            L->done = 1;
            return;
        } else {
            b = -1;
        }
    }
    L->extractions += 1;
    L->xbin = b;
    L->xcount = b >= 0 ? (c < static_cast<unsigned long long>(cap) ? c : static_cast<unsigned long long>(cap)) : 0;
    L->xm = finished ? L->mcount : 0;
    if (finished) L->mcount = 0;
    L->xfin = single ? 1 : 0;
    L->extract = 2;
    if (b >= 0) {
        L->bc[b] = 0;
        const bool over = (L->overflow >> b) & 1ULL;
        L->overflow &= ~(1ULL << b);
        // a pile past scan_above entries (random reads per entry) costs more than the scan's
        // sequential pass over the bitmaps
        if (over || c > static_cast<unsigned long long>(scan_above)) {
            L->extract = 1;
            L->xm = 0;
            L->mcount = 0;                   // the scan takes every member from the bitmap
            L->full_scans += 1;
        }
    }
    // A large finished bucket pulls its heavy entries (ds_pull_heavy) instead of pushing them;
    // its members go to pull list j & 1 and the previous pull's list is cleared on the way.
    if (L->extract == 2 && single && pull_min > 0 && L->xm >= static_cast<unsigned long long>(pull_min)) {
        const unsigned long long j = L->pulls;
        L->xpull = 1;
        L->pbucket = kfin;
        L->xprev = L->pcount[(j + 1) & 1];
        L->pcount[(j + 1) & 1] = 0;
        L->pcount[j & 1] = L->xm;
    }
}

// ---------------------------------------------------------------- extract
// chunk_extract (frontier.hpp) with the packed counter: pass 1 counts (slots and entries),
// one packed atomic per block, pass 2 writes the queue and its entry offsets.
template <int kStreams, class Probe>
__device__ __forceinline__ void chunk_extract_packed(int64_t words, const Probe& probe, int32_t* __restrict__ qn,
                                                     int64_t* __restrict__ qpre, unsigned long long* qc) {
    const int64_t per = ((words + gridDim.x - 1) / gridDim.x + kWavesPerBlock - 1) / kWavesPerBlock * kWavesPerBlock;
    const int64_t w0 = static_cast<int64_t>(blockIdx.x) * per;
    const int64_t w1 = min(words, w0 + per);
    const int wave = threadIdx.x >> 6;
    const unsigned long long below = (1ULL << lane()) - 1ULL;
    int64_t count = 0, dsum = 0;             // this lane's takes
    unsigned long long mask = 0;
    bool touch = false;
    extract_count<kStreams>(w0 + wave, w1, probe, count, dsum, mask, touch);
    // per-wave totals: the pass-2 order is word by word inside a wave, so only the wave's
    // first slot / offset come from the reservation
    const int64_t wc = wave_incl_scan(count), wdg = wave_incl_scan(dsum);
    int64_t slot0, doff0;
    block_reserve(qc, lane() == 63 ? wc : 0, lane() == 63 ? wdg : 0, slot0, doff0);
    int64_t cursor = __shfl(slot0, 63, 64), dcur = __shfl(doff0, 63, 64);
    if (!touch) return;                                      // wave-uniform
    extract_write<kStreams>(w0 + wave, w1, mask, probe, [&](const Take* t) {
        for (int k = 0; k < kStreams; ++k) {
            const unsigned long long bm = __ballot(t[k].take);
            if (!bm) continue;
            const int64_t d = t[k].take ? t[k].deg : 0;
            const int64_t id = wave_incl_scan(d);
            if (t[k].take) {
                const int64_t slot = cursor + __popcll(bm & below);
                qn[slot] = t[k].entry;
                qpre[slot] = dcur + id - d;
            }
            cursor += __popcll(bm);
            dcur += __shfl(id, 63, 64);
        }
    });
}

// chunk_extract_packed over a staged probe (frontier.hpp extract_count_staged)
template <int kStreams, class Probe, int kU = kExtractUnroll>
__device__ __forceinline__ void chunk_extract_packed_staged(int64_t words, const Probe& probe, int32_t* __restrict__ qn,
                                                            int64_t* __restrict__ qpre, unsigned long long* qc) {
    const int64_t per = ((words + gridDim.x - 1) / gridDim.x + kWavesPerBlock - 1) / kWavesPerBlock * kWavesPerBlock;
    const int64_t w0 = static_cast<int64_t>(blockIdx.x) * per;
    const int64_t w1 = min(words, w0 + per);
    const int wave = threadIdx.x >> 6;
    const unsigned long long below = (1ULL << lane()) - 1ULL;
    int64_t count = 0, dsum = 0;
    unsigned long long mask = 0;
    bool touch = false;
    if (w0 + wave < w1) extract_count_staged<kStreams, Probe, kU>(w0 + wave, w1, probe, count, dsum, mask, touch);
    const int64_t wc = wave_incl_scan(count), wdg = wave_incl_scan(dsum);
    int64_t slot0, doff0;
    block_reserve(qc, lane() == 63 ? wc : 0, lane() == 63 ? wdg : 0, slot0, doff0);
    int64_t cursor = __shfl(slot0, 63, 64), dcur = __shfl(doff0, 63, 64);
    if (!touch) return;                                      // wave-uniform
    const auto emit = [&](const Take* t) {
        for (int k = 0; k < kStreams; ++k) {
            const unsigned long long bm = __ballot(t[k].take);
            if (!bm) continue;
            const int64_t d = t[k].take ? t[k].deg : 0;
            const int64_t id = wave_incl_scan(d);
            if (t[k].take) {
                const int64_t slot = cursor + __popcll(bm & below);
                qn[slot] = t[k].entry;
                qpre[slot] = dcur + id - d;
            }
            cursor += __popcll(bm);
            dcur += __shfl(id, 63, 64);
        }
    };
    extract_write_staged<kStreams, Probe, decltype(emit), kU>(w0 + wave, w1, mask, probe, emit);
}

// The bitmap-scan extraction's probe in stages: the pending / member words, then each lane's
// distance and list bounds (only where its bit is set), then the takes.
struct ScanProbe {
    const int64_t* off; const int64_t* light; uint64_t* pend; uint64_t* member; const int64_t* dist;
    uint64_t* fin; int64_t thr; long long* left;
    struct State { uint64_t pb, mb; long long d; int64_t o0, o1, lt; };
    // a word with no pending and no member bit takes nothing and leaves nothing pending
    __device__ __forceinline__ bool live(int64_t wd) const { return (pend[wd] | member[wd]) != 0; }
    __device__ __forceinline__ void stage1(int64_t wd, State& s) const {
        s.pb = pend[wd];                                      // uniform across the wave
        s.mb = member[wd];
    }
    __device__ __forceinline__ void stage2(int64_t wd, State& s) const {
        const int64_t v = (wd << 6) + lane();
        const bool p = (s.pb >> lane()) & 1ULL, mine = (s.mb >> lane()) & 1ULL;
        s.d = p ? static_cast<long long>(dist[v]) : kInf;
        s.o0 = p ? off[v] : 0;
        s.o1 = mine ? off[v + 1] : 0;
        s.lt = p || mine ? light[v] : 0;
    }
    __device__ __forceinline__ bool finish(int64_t wd, const State& s, Take* t, bool commit) const {
        const int64_t v = (wd << 6) + lane();
        const bool p = (s.pb >> lane()) & 1ULL, mine = (s.mb >> lane()) & 1ULL;
        const bool lt = p && s.d < thr;
        if (!commit && p && !lt && s.d < *left) *left = s.d;
        const int64_t hdeg = mine ? s.o1 - s.lt : 0;
        const unsigned long long tm = __ballot(lt);
        if (commit && lane() == 0) {
            if (tm) pend[wd] = s.pb & ~tm;
            if (s.mb) {
                member[wd] = 0;
                if (fin) fin[wd] |= s.mb;
            }
        }
        t[0] = {lt, static_cast<int32_t>(v), lt ? s.lt - s.o0 : 0};
        t[1] = {hdeg > 0, static_cast<int32_t>(static_cast<uint32_t>(v) | kHeavy), hdeg};
        return tm || s.mb;
    }
};

// done (binned loop, may be null): when the decision found the bucket finished (L->xfin), the
// members taken here are final and become done.  The smallest distance left pending is
// min-reduced into *lo (L->lo, or L->lo_next for the partitioned loop).
template <int kU = kExtractUnroll>
__device__ __forceinline__ void extract_scan(const int64_t* __restrict__ off, const int64_t* __restrict__ light,
        uint64_t* __restrict__ pend, uint64_t* __restrict__ member, int64_t n, const int64_t* __restrict__ dist,
        DsLoop* L, int cur, int32_t* __restrict__ qn, int64_t* __restrict__ qpre, uint64_t* __restrict__ done,
        int64_t thr, long long* lo) {
    uint64_t* const fin = (done && L->xfin) ? done : nullptr;
    const int64_t words = (n + 63) >> 6;
    long long left = kInf;                                   // smallest distance left pending
    const ScanProbe probe{off, light, pend, member, dist, fin, thr, &left};
    chunk_extract_packed_staged<2, ScanProbe, kU>(words, probe, qn, qpre, &L->qc[cur]);
    const long long m = block_min(left);
    if (threadIdx.x == 0 && m != kInf) atomicMin(lo, m);
}

__global__ void __launch_bounds__(kBlock) ds_extract_dev(const int64_t* __restrict__ off,
        const int64_t* __restrict__ light, uint64_t* __restrict__ pend, uint64_t* __restrict__ member, int64_t n,
        const int64_t* __restrict__ dist, DsLoop* L, int cur, int32_t* __restrict__ qn, int64_t* __restrict__ qpre) {
    if (L->extract != 1) return;                             // grid-uniform
    extract_scan(off, light, pend, member, n, dist, L, cur, qn, qpre, nullptr, L->thr, &L->lo);
}

// The binned extraction (extract == 2): the decided pile's entries — a vertex is taken when it
// is still pending and below the threshold, the pending bit cleared by the taking atomic, so a
// vertex appended several times is taken once — then, when a bucket finished, its member
// list's heavy entries (member words reset: every set bit of the member bitmap is on the list;
// the members marked done).  Work proportional to the pile, not to n.
// Body of the pile extraction (mode 2) for block `bid` of `nb` (ds_small_steps runs it as one
// block).
__device__ __forceinline__ void extract_bins_body(int64_t bid, int64_t nb, const int64_t* __restrict__ off,
        const int64_t* __restrict__ light, uint64_t* __restrict__ pend, uint64_t* __restrict__ member,
        const int64_t* __restrict__ dist, DsLoop* L, int cur, const int32_t* __restrict__ pile, int64_t cap,
        const int32_t* __restrict__ mlist, uint64_t* __restrict__ done, int32_t* __restrict__ qn,
        int64_t* __restrict__ qpre, const DsPull& pull) {
    const int64_t thr = L->thr;
    const bool xpull = L->xpull != 0;
    const bool xfin = L->xfin != 0;
    const unsigned long long j = L->pulls;
    uint64_t* __restrict__ pm = pull.pm[j & 1];
    int32_t* __restrict__ pl_now = pull.pl[j & 1];
    uint64_t* __restrict__ pm_prev = pull.pm[(j + 1) & 1];
    const int32_t* __restrict__ pl_prev = pull.pl[(j + 1) & 1];
    const int64_t xc = static_cast<int64_t>(L->xcount), xme = xc + static_cast<int64_t>(L->xm);
    const int64_t total = xme + (xpull ? static_cast<int64_t>(L->xprev) : 0);
    const int32_t* __restrict__ pl = pile + (L->xbin >= 0 ? L->xbin : 0) * cap;
    for (int64_t base = bid * kBlock; base < total; base += nb * kBlock) {   // block-uniform trips
        const int64_t i = base + threadIdx.x;
        bool take = false;
        int32_t entry = 0;
        int64_t deg = 0;
        if (i < xc) {
            const int32_t v = pl[i];
            const uint64_t bit = 1ULL << (v & 63);
            if ((pend[v >> 6] & bit) && dist[v] < thr) {
                const unsigned long long old = atomicAnd(reinterpret_cast<unsigned long long*>(&pend[v >> 6]), ~bit);
                if (old & bit) {
                    take = true;
                    entry = v;
                    deg = light_deg(off, light, v);
                }
            }
        } else if (i < xme) {                                 // a finished bucket's member
            const int32_t v = mlist[i - xc];
            member[v >> 6] = 0;
            if (xfin)                                         // final only after a single bucket
                atomicOr(reinterpret_cast<unsigned long long*>(&done[v >> 6]), 1ULL << (v & 63));
            if (xpull) {                                      // its heavy entries are pulled
                atomicOr(reinterpret_cast<unsigned long long*>(&pm[v >> 6]), 1ULL << (v & 63));
                pl_now[i - xc] = v;
            } else {
                const int64_t hdeg = off[v + 1] - light[v];
                if (hdeg > 0) {
                    take = true;
                    entry = static_cast<int32_t>(static_cast<uint32_t>(v) | kHeavy);
                    deg = hdeg;
                }
            }
        } else if (i < total) {                               // the previous pull's bitmap words
            pm_prev[pl_prev[i - xme] >> 6] = 0;
        }
        int64_t slot, doff;
        block_reserve(&L->qc[cur], take ? 1 : 0, deg, slot, doff);
        if (take) {
            qn[slot] = entry;
            qpre[slot] = doff;
        }
    }
}

__global__ void __launch_bounds__(kBlock) ds_extract_bins(const int64_t* __restrict__ off,
        const int64_t* __restrict__ light, uint64_t* __restrict__ pend, uint64_t* __restrict__ member,
        const int64_t* __restrict__ dist, DsLoop* L, int cur, const int32_t* __restrict__ pile, int64_t cap,
        const int32_t* __restrict__ mlist, uint64_t* __restrict__ done, int32_t* __restrict__ qn,
        int64_t* __restrict__ qpre, int64_t n, DsPull pull) {
    const unsigned long long mode = L->extract;             // grid-uniform
    if (mode == 1) {                                         // a large or overflowed pile: the bitmap scan
        extract_scan(off, light, pend, member, n, dist, L, cur, qn, qpre, done, L->thr, &L->lo);
        return;
    }
    if (mode != 2) return;
    extract_bins_body(blockIdx.x, gridDim.x, off, light, pend, member, dist, L, cur, pile, cap, mlist, done, qn, qpre,
                      pull);
}

// ---------------------------------------------------------------- commit
// kList (binned loop): a newly marked member is also appended to the member list (one
// reservation per wave), so the extraction visits the members without scanning the bitmap.
template <bool kList>
__device__ __forceinline__ void commit_body(int64_t bid, int64_t nb, const int32_t* __restrict__ q,
        const int64_t* __restrict__ dist, int64_t* __restrict__ msg, uint64_t* __restrict__ pend,
        uint64_t* __restrict__ member, DsLoop* L, int cur, int32_t* __restrict__ mlist) {
    const int64_t qlen = qcount(L->qc[cur]);
    if (bid == 0 && threadIdx.x == 0) L->qc[cur ^ 1] = 0;           // the relax appends there next
    bool marked = false;
    __shared__ unsigned int s_wc[kWavesPerBlock];
    __shared__ unsigned long long s_mb;
    const int64_t stride = nb * kBlock;
    for (int64_t base = bid * kBlock; base < qlen; base += stride) {                // block-uniform
        const int64_t i = base + threadIdx.x;
        bool nm = false;
        int32_t v = -1;
        if (i < qlen) {
            const uint32_t e = static_cast<uint32_t>(q[i]);
            if (!(e & kHeavy)) {
                v = static_cast<int32_t>(e);
                msg[v] = dist[v];
                const uint64_t bit = 1ULL << (v & 63);
                if (pend[v >> 6] & bit) atomicAnd(reinterpret_cast<unsigned long long*>(&pend[v >> 6]), ~bit);
                if (!(member[v >> 6] & bit)) {
                    const unsigned long long ob = atomicOr(reinterpret_cast<unsigned long long*>(&member[v >> 6]), bit);
                    nm = !(ob & bit);
                    marked = true;
                }
            }
        }
        if (kList) {                                          // one reservation per block and trip
            const unsigned long long bm = __ballot(nm);
            const int wave = threadIdx.x >> 6;
            if (lane() == 0) s_wc[wave] = static_cast<unsigned int>(__popcll(bm));
            __syncthreads();
            if (threadIdx.x == 0) {
                unsigned int tot = 0;
                for (int w = 0; w < kWavesPerBlock; ++w) { const unsigned int x = s_wc[w]; s_wc[w] = tot; tot += x; }
                s_mb = tot ? atomicAdd(&L->mcount, static_cast<unsigned long long>(tot)) : 0ULL;
            }
            __syncthreads();
            if (nm) mlist[s_mb + s_wc[wave] + __popcll(bm & ((1ULL << lane()) - 1ULL))] = v;
            __syncthreads();
        }
    }
    if (__ballot(marked) && lane() == 0) L->members = 1;
}
template <bool kList>
__global__ void __launch_bounds__(kBlock) ds_commit_dev(const int32_t* __restrict__ q, const int64_t* __restrict__ dist,
        int64_t* __restrict__ msg, uint64_t* __restrict__ pend, uint64_t* __restrict__ member, DsLoop* L, int cur,
        int32_t* __restrict__ mlist) {
    commit_body<kList>(blockIdx.x, gridDim.x, q, dist, msg, pend, member, L, cur, mlist);
}

// ---------------------------------------------------------------- relax
// ds_relax_ws over the packed queue: the load-balanced search of frontier.hpp
// (for_each_queue_edge) with the total from the counter, and the takes of a whole tile
// appended with one packed reservation (the per-trip block_append cost 8 reservations and
// 16 barriers per tile).
// kBins (binned loop): an improvement that is not taken into the near queue — a later bucket,
// or the current bucket for a vertex already pending — is appended to its bucket's pile
// (bucket / nbins ring), the appends of a tile aggregated per pile in LDS (one atomic per
// pile and tile).
// kPart (1-D partition, not with kBins): the lists hold global ids; a target outside
// [plo, plo + n_local) is min-reduced into rbest and marked in rmark for the owner (delta.hip).
// kDone (binned loop with the done filter, TGO_DS_DONE): the done-word stage is compiled only
// when it runs (its 8 words per thread cost the occupancy of the filter-off kernel).
// kE: entries per thread of a tile (kBlock * kE per tile).  8 (round 6, with the branch-free
// stages below): 127 VGPRs, 4 waves per SIMD — the RMAT-24 sum over 4 roots 47.0 ms (round-5
// code, kE 5) -> 45.7 (kE 5, 97 VGPRs) -> 44.0 (kE 8); 6: 45.2, 12 (174 VGPRs): 55.6, 16: 56.3
// (profiles/r06ds1_sssp_branchfree_ab.log, r06ds2_sssp_relax_e_ab.log).  Round 5 measured 5 best
// when every stage's loads were serialised (125 VGPRs then).
constexpr int kDsRelaxE = 8;
template <bool kBins, bool kPart, bool kDone, int kE>
__device__ __forceinline__ void relax_body(int64_t bid, int64_t nb, const int64_t* __restrict__ off,
        const int32_t* __restrict__ adj, const int32_t* __restrict__ wt, const int64_t* __restrict__ light,
        const int32_t* __restrict__ q, const int64_t* __restrict__ qpre, const int64_t* __restrict__ msg,
        int64_t* __restrict__ dist, uint64_t* __restrict__ pend, int32_t* __restrict__ qn,
        int64_t* __restrict__ qpre_n, DsLoop* L, int cur, int64_t delta, int nbins, int32_t* __restrict__ pile,
        int64_t cap, const uint64_t* __restrict__ done, int64_t plo, int64_t n_local, int64_t* __restrict__ rbest,
        uint64_t* __restrict__ rmark) {
    static_assert(!(kBins && kPart), "the partitioned loop has no piles");
    const unsigned long long c = L->qc[cur];
    const int64_t qlen = qcount(c), total = qentries(c);
    if (qlen == 0) return;                                   // grid-uniform
    const int64_t thr = L->thr;
    const int64_t bucket = kBins ? L->bucket : 0;
    __shared__ unsigned int s_bn[kDsMaxBins];
    __shared__ unsigned long long s_bb[kDsMaxBins];
    bool spill = false;
    if (bid == 0 && threadIdx.x == 0) {
        L->phases += 1;
        L->relaxed += static_cast<unsigned long long>(total);
    }
    __shared__ int64_t s_pre[(kBlock * kE + 2)];
    __shared__ int32_t s_q[(kBlock * kE + 2)];
    __shared__ int64_t s_lo, s_hi;
    long long tmin = kInf;                                   // improvements that queued nothing
    bool bad = false;
    const int64_t ntiles = (total + (kBlock * kE) - 1) / (kBlock * kE);
    auto pre = [&](int64_t i) -> int64_t { return i < qlen ? qpre[i] : total; };
    for (int64_t tile = bid; tile < ntiles; tile += nb) {
        const int64_t t0 = tile * (kBlock * kE);
        const int64_t t1 = min(total, t0 + (kBlock * kE));
        if (kBins && threadIdx.x < kDsMaxBins) s_bn[threadIdx.x] = 0;
        tile_bounds(qpre, qlen, t0, t1, s_lo, s_hi);   // lo = last i with pre(i) <= t0; hi = last with <= t1-1
        __syncthreads();
        const int64_t lo = s_lo, hi = s_hi;
        const int64_t span = hi - lo + 1;
        const bool in_lds = span + 1 <= (kBlock * kE + 2);
        if (in_lds) {
            for (int64_t i = threadIdx.x; i <= span; i += kBlock) {
                s_pre[i] = pre(lo + i);
                if (i < span) s_q[i] = q[lo + i];
            }
        }
        __syncthreads();
        // the tile's kE entries per thread in stages, so each stage's loads are
        // independent and in flight together (one entry at a time left every thread waiting
        // out the whole search -> list -> distance -> atomic chain once per entry)
        int64_t u[kE], e[kE];
        bool hv[kE];
#pragma unroll
        for (int k = 0; k < kE; ++k) {           // 1: owning queue entry (LDS search)
            const int64_t j = t0 + k * kBlock + threadIdx.x;
            u[k] = -1;
            e[k] = 0;
            hv[k] = false;
            if (j >= t1) continue;
            int32_t qe;
            int64_t start;
            if (in_lds) {
                int64_t a = 0, b = span;
                while (b - a > 1) { const int64_t m = (a + b) >> 1; if (s_pre[m] <= j) a = m; else b = m; }
                qe = s_q[a]; start = s_pre[a];
            } else {
                int64_t a = lo, b = hi + 1;
                while (b - a > 1) { const int64_t m = (a + b) >> 1; if (qpre[m] <= j) a = m; else b = m; }
                qe = q[a]; start = qpre[a];
            }
            const uint32_t ue = static_cast<uint32_t>(qe);
            u[k] = static_cast<int64_t>(ue & ~kHeavy);
            e[k] = j - start;
            hv[k] = (ue & kHeavy) != 0;
        }
#pragma unroll
        for (int k = 0; k < kE; ++k) {           // 1b: the list starts, loads issued together
            const int64_t* base = hv[k] ? light : off;
            e[k] += base[u[k] >= 0 ? u[k] : 0];
        }
        // Stages 2-4 issue each stage's memory operations for all kE entries together, without a
        // branch around a load: a conditional load per entry made the compiler wait for every
        // outstanding load before the next (one load, then one atomic, in flight per lane).
        // Lanes without an entry read entry 0 / vertex 0 (valid: the tile exists, n >= 1) and
        // drop the values.
        int32_t t[kE], w[kE];
        int64_t mu[kE], du[kE];
#pragma unroll
        for (int k = 0; k < kE; ++k) {           // 2: entry, the source's snapshot
            const bool ok = u[k] >= 0;
            const int64_t ek = ok ? e[k] : 0, uk = ok ? u[k] : 0;
            t[k] = adj[ek];
            w[k] = wt[ek];
            mu[k] = msg[uk];
            du[k] = dist[uk];
        }
        int64_t cand[kE], dt[kE], tl[kE];
        uint64_t dw[kE];
        if (kBins && kDone) {
#pragma unroll
            for (int k = 0; k < kE; ++k)         // 3a: done words (L2-resident bitmap)
                dw[k] = done ? done[(u[k] >= 0 ? t[k] : 0) >> 6] : 0ULL;
        }
#pragma unroll
        for (int k = 0; k < kE; ++k) {           // 3: the targets' distances
            const bool ok = u[k] >= 0;
            bad |= ok && w[k] == kMissingWeight;                   // edge.value(weight) on a missing key
            // u improved during this phase (du < mu): pending again, relaxes later
            bool live = ok && w[k] != kMissingWeight && !(du[k] < mu[k]);
            // a done target's distance is below every candidate of a later bucket: no read
            if (kBins && kDone) live = live && !((dw[k] >> (t[k] & 63)) & 1ULL);
            cand[k] = live ? mu[k] + static_cast<int64_t>(w[k]) : -1;
            if constexpr (kPart) {
                tl[k] = static_cast<int64_t>(t[k]) - plo;
                const bool local = tl[k] >= 0 && tl[k] < n_local;
                dt[k] = local ? dist[live ? tl[k] : 0] : rbest[live ? t[k] : 0];
            } else {
                dt[k] = dist[live ? t[k] : 0];
            }
        }
        int32_t tv[kE];
        int64_t td[kE];
        int32_t fb[kE];                          // kBins: pile of a far append, or -1
        unsigned int fl[kE];                     // and its slot among the tile's appends
        int ntake = 0;
        int64_t dtake = 0;
        bool imp[kE];                            // 4: min, pending bit, take
#pragma unroll
        for (int k = 0; k < kE; ++k) imp[k] = cand[k] >= 0 && cand[k] < dt[k];   // a stale (larger) read only costs an atomic
        if constexpr (kPart) {                   // a remote target: best sent so far
            long long rold[kE];
#pragma unroll
            for (int k = 0; k < kE; ++k) {
                rold[k] = kInf;
                if (imp[k] && !(tl[k] >= 0 && tl[k] < n_local))
                    rold[k] = atomicMin(reinterpret_cast<long long*>(&rbest[t[k]]), static_cast<long long>(cand[k]));
            }
#pragma unroll
            for (int k = 0; k < kE; ++k) {
                if (!imp[k] || (tl[k] >= 0 && tl[k] < n_local)) continue;
                imp[k] = false;
                if (cand[k] < rold[k]) {
                    const int64_t g = t[k];
                    const uint64_t rbit = 1ULL << (g & 63);
                    if (!(rmark[g >> 6] & rbit)) atomicOr(reinterpret_cast<unsigned long long*>(&rmark[g >> 6]), rbit);
                }
            }
        }
        int32_t tk[kE];
        long long old[kE];
#pragma unroll
        for (int k = 0; k < kE; ++k) {           // 4a: every improving entry's atomicMin in flight together
            tk[k] = t[k];
            if constexpr (kPart) tk[k] = static_cast<int32_t>(tl[k]);
            old[k] = kInf;
            if (imp[k]) old[k] = atomicMin(reinterpret_cast<long long*>(&dist[tk[k]]), static_cast<long long>(cand[k]));
        }
        unsigned long long ob[kE];
#pragma unroll
        for (int k = 0; k < kE; ++k) {           // 4b: then every improved entry's pending bit
            imp[k] = imp[k] && cand[k] < old[k];
            ob[k] = 0;
            if (imp[k]) ob[k] = atomicOr(reinterpret_cast<unsigned long long*>(&pend[tk[k] >> 6]), 1ULL << (tk[k] & 63));
        }
#pragma unroll
        for (int k = 0; k < kE; ++k) {           // 4c: take, or a pile / the pending minimum
            tv[k] = -1;
            td[k] = 0;
            fb[k] = -1;
            if (!imp[k]) continue;
            const uint64_t bit = 1ULL << (tk[k] & 63);
            if (!(ob[k] & bit) && cand[k] < thr) {
                tv[k] = tk[k];
                td[k] = light_deg(off, light, tk[k]);
                ++ntake;
                dtake += td[k];
            } else if (kBins) {
                const int64_t ahead = cand[k] / delta - bucket;
                if (ahead >= nbins) {
                    spill = true;
                } else {
                    fb[k] = static_cast<int32_t>((bucket + ahead) % nbins);
                    fl[k] = atomicAdd(&s_bn[fb[k]], 1u);
                }
            } else if (cand[k] < tmin) {
                tmin = cand[k];
            }
        }
        if (kBins) {                                          // the tile's far appends, per pile
            __syncthreads();
            if (threadIdx.x < nbins) {
                const unsigned int cnt = s_bn[threadIdx.x];
                s_bb[threadIdx.x] = cnt ? atomicAdd(&L->bc[threadIdx.x], static_cast<unsigned long long>(cnt)) : 0ULL;
                if (cnt && s_bb[threadIdx.x] + cnt > static_cast<unsigned long long>(cap))
                    atomicOr(&L->overflow, 1ULL << threadIdx.x);
            }
            __syncthreads();
#pragma unroll
            for (int k = 0; k < kE; ++k)
                if (fb[k] >= 0) {
                    const unsigned long long slot = s_bb[fb[k]] + fl[k];
                    if (slot < static_cast<unsigned long long>(cap)) pile[fb[k] * cap + static_cast<int64_t>(slot)] = t[k];
                }
        }
        // the tile's takes: one packed reservation (block-uniform call)
        int64_t slot, doff;
        block_reserve(&L->qc[cur ^ 1], ntake, dtake, slot, doff);
        if (ntake) {
#pragma unroll
            for (int k = 0; k < kE; ++k)
                if (tv[k] >= 0) {
                    qn[slot] = tv[k];
                    qpre_n[slot] = doff;
                    ++slot;
                    doff += td[k];
                }
        }
        __syncthreads();
    }
    if (__ballot(bad) && lane() == 0) L->err = 1;
    if (kBins) {
        if (__ballot(spill) && lane() == 0) L->spill = 1;
        return;
    }
    const long long m = block_min(tmin);
    if (threadIdx.x == 0 && m != kInf) atomicMin(&L->tm, m);
}
template <bool kBins, bool kPart = false, bool kDone = false, int kE = kDsRelaxE>
__global__ void __launch_bounds__(kBlock) ds_relax_dev(const int64_t* __restrict__ off, const int32_t* __restrict__ adj,
        const int32_t* __restrict__ wt, const int64_t* __restrict__ light, const int32_t* __restrict__ q,
        const int64_t* __restrict__ qpre, const int64_t* __restrict__ msg, int64_t* __restrict__ dist,
        uint64_t* __restrict__ pend, int32_t* __restrict__ qn, int64_t* __restrict__ qpre_n, DsLoop* L, int cur,
        int64_t delta, int nbins, int32_t* __restrict__ pile, int64_t cap, const uint64_t* __restrict__ done,
        int64_t plo = 0, int64_t n_local = 0, int64_t* __restrict__ rbest = nullptr,
        uint64_t* __restrict__ rmark = nullptr) {
    relax_body<kBins, kPart, kDone, kE>(blockIdx.x, gridDim.x, off, adj, wt, light, q, qpre, msg, dist, pend, qn,
                                        qpre_n, L, cur, delta, nbins, pile, cap, done, plo, n_local, rbest, rmark);
}

// ---------------------------------------------------------------- 1-D partition
// The partitioned loop (part_driver.cpp tgo_part_sssp_run over api.cpp's part_sssp_dev_*) runs
// this file's commit / relax / extraction on each rank's rows; the decisions are global, so
// they come from the host after the per-phase header exchange instead of ds_decide.
//
// Owner side of the exchange: min the received (local id, distance) pairs into dist; a newly
// pending one below the threshold joins the next near queue (packed reservation), any other
// improvement folds into tm.
__global__ void __launch_bounds__(kBlock) ds_part_apply(const int64_t* __restrict__ recv, int64_t npairs,
        const int64_t* __restrict__ off, const int64_t* __restrict__ light, int64_t* __restrict__ dist,
        uint64_t* __restrict__ pend, int32_t* __restrict__ qn, int64_t* __restrict__ qpre_n, DsLoop* L, int cur) {
    const int64_t thr = L->thr;
    long long tmin = kInf;
    for (int64_t base = static_cast<int64_t>(blockIdx.x) * kBlock; base < npairs;
         base += static_cast<int64_t>(gridDim.x) * kBlock) {                 // block-uniform trips
        const int64_t i = base + threadIdx.x;
        bool take = false;
        int64_t v = 0, deg = 0;
        if (i < npairs) {
            v = recv[2 * i];
            const long long cand = recv[2 * i + 1];
            if (cand < dist[v]) {
                const long long old = atomicMin(reinterpret_cast<long long*>(&dist[v]), cand);
                if (cand < old) {
                    const uint64_t bit = 1ULL << (v & 63);
                    const unsigned long long ob = atomicOr(reinterpret_cast<unsigned long long*>(&pend[v >> 6]), bit);
                    if (!(ob & bit) && cand < thr) {
                        take = true;
                        deg = light_deg(off, light, v);
                    } else if (cand < tmin) {
                        tmin = cand;
                    }
                }
            }
        }
        int64_t slot, doff;
        block_reserve(&L->qc[cur ^ 1], take ? 1 : 0, deg, slot, doff);
        if (take) {
            qn[slot] = static_cast<int32_t>(v);
            qpre_n[slot] = doff;
        }
    }
    const long long m = block_min(tmin);
    if (threadIdx.x == 0 && m != kInf) atomicMin(&L->tm, m);
}

// The global decision of an empty phase (host: every near queue empty) and its extraction below
// thr, in one launch: block 0 books the decision (none of it is read by the extraction, which
// takes thr as an argument), the blocks min their pending distances into lo_next, and the next
// header (ds_part_header, after every block has finished) moves it into lo.  (A separate
// one-thread decision launch cost ~10 us a bucket.)
template <int kU>
__global__ void __launch_bounds__(kBlock) ds_part_extract(const int64_t* __restrict__ off,
        const int64_t* __restrict__ light, uint64_t* __restrict__ pend, uint64_t* __restrict__ member, int64_t n,
        const int64_t* __restrict__ dist, DsLoop* L, int cur, int32_t* __restrict__ qn, int64_t* __restrict__ qpre,
        int64_t thr) {
    if (blockIdx.x == 0 && threadIdx.x == 0) {
        if (thr > L->thr) L->buckets += 1;
        L->thr = thr;
        L->tm = kInf;
        L->members = 0;
        L->extract = 1;
        L->extractions += 1;
        L->xnew = 1;
    }
    extract_scan<kU>(off, light, pend, member, n, dist, L, cur, qn, qpre, nullptr, thr, &L->lo_next);
}

// The exchange header (delta.hip ds_mark_sizes for this loop): offs[r] = the pack offset of
// rank r's pairs; to r {pair elements, near-queue length, min(tm, lo), members}.  Zeroes the
// counts for the next phase and the pack's cursors.
// host (one rank only, may be null): the header all-to-all of one rank is the identity, so the
// fold (delta.hip ds_header_fold: sent / received elements, queue length, pending minimum,
// -members) goes straight to the host-mapped counter page with its sequence word — one launch
// where the exchange takes three (header, all-to-all copy, fold + publish).
__global__ void ds_part_header(unsigned long long* __restrict__ counts, int nranks, DsLoop* L, int cur,
                               unsigned long long* __restrict__ offs, unsigned long long* __restrict__ cursor,
                               int64_t* __restrict__ sizes, unsigned long long* host, unsigned long long seq) {
    if (threadIdx.x != 0) return;
    if (L->xnew) {                       // the pending minimum of the extraction since the last header
        L->lo = L->lo_next;
        L->lo_next = kInf;
        L->xnew = 0;
    }
    const int64_t qlen = qcount(L->qc[cur]);
    const long long pm = L->tm < L->lo ? L->tm : L->lo;
    const int64_t mem = L->members ? 1 : 0;
    unsigned long long acc = 0;
    for (int r = 0; r < nranks; ++r) {
        const unsigned long long c = counts[r];
        offs[r] = acc;
        acc += c;
        sizes[4 * r] = 2 * static_cast<int64_t>(c);
        sizes[4 * r + 1] = qlen;
        sizes[4 * r + 2] = pm;
        sizes[4 * r + 3] = mem;
        counts[r] = 0;
        cursor[r] = 0;
    }
    if (!host || nranks != 1) return;
    const unsigned long long w[5] = {static_cast<unsigned long long>(sizes[0]), static_cast<unsigned long long>(sizes[0]),
                                     static_cast<unsigned long long>(qlen), static_cast<unsigned long long>(pm),
                                     static_cast<unsigned long long>(-mem)};
    for (int i = 0; i < 5; ++i) __hip_atomic_store(&host[i], w[i], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    __threadfence_system();
    __hip_atomic_store(&host[kCounterWords], seq, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
}

// The pull form of a large finished bucket's heavy entries: a vertex that can still improve
// (dist > (finished bucket + 1) * delta: every heavy candidate is at least that) reads its pull
// list for heavy entries (w >= delta) from the bucket's members (bitmap pm) and takes the
// minimum over msg[u] + w; an improvement is settled as the relax settles one (near queue below
// the threshold when newly pending, else the pile of its bucket).  Same relaxations as the
// members' push, so the same converged distances.
__global__ void __launch_bounds__(kBlock) ds_pull_heavy(const int64_t* __restrict__ ws_off,
        const int64_t* __restrict__ light, const int64_t* __restrict__ msg, int64_t* __restrict__ dist,
        uint64_t* __restrict__ pend, int32_t* __restrict__ qn, int64_t* __restrict__ qpre_n, DsLoop* L, int cur,
        int64_t delta, int nbins, int32_t* __restrict__ pile, int64_t cap, DsPull pull) {
    if (!L->xpull) return;                                   // grid-uniform
    const uint64_t* __restrict__ pm = pull.pm[L->pulls & 1];
    const int64_t thr = L->thr, bucket = L->bucket;
    const int64_t floor_c = (L->pbucket + 1) * delta;        // no heavy candidate is below this
    const View& pv = pull.view;
    __shared__ unsigned int s_bn[kDsMaxBins];
    __shared__ unsigned long long s_bb[kDsMaxBins];
    bool bad = false, spill = false;
    for (int64_t base = static_cast<int64_t>(blockIdx.x) * kBlock; base < pull.n_active;
         base += static_cast<int64_t>(gridDim.x) * kBlock) {                 // block-uniform trips
        if (threadIdx.x < kDsMaxBins) s_bn[threadIdx.x] = 0;
        __syncthreads();
        const int64_t v = base + threadIdx.x;
        long long best = kInf;
        long long dv = kInf;
        if (v < pull.n_active) {
            dv = static_cast<long long>(dist[v]);
            if (dv > floor_c) {
                for (int l = 0; l < pv.nlists; ++l) {
                    const int64_t* off = l == 0 ? pv.off0 : pv.off1;
                    const int32_t* adj = l == 0 ? pv.adj0 : pv.adj1;
                    const int32_t* wt = l == 0 ? pv.w0 : pv.w1;
                    const int64_t e1 = off[v + 1];
                    for (int64_t e = off[v]; e < e1; e += 4) {
                        int32_t u[4], w[4];
                        uint64_t mw[4];
#pragma unroll
                        for (int q = 0; q < 4; ++q) {
                            u[q] = e + q < e1 ? adj[e + q] : -1;
                            w[q] = e + q < e1 ? wt[e + q] : 0;
                        }
#pragma unroll
                        for (int q = 0; q < 4; ++q) mw[q] = u[q] >= 0 ? pm[u[q] >> 6] : 0ULL;
#pragma unroll
                        for (int q = 0; q < 4; ++q) {
                            if (u[q] < 0 || !((mw[q] >> (u[q] & 63)) & 1ULL)) continue;
                            if (w[q] == kMissingWeight) { bad = true; continue; }
                            if (w[q] < delta) continue;               // light: relaxed in its bucket
                            const long long c = static_cast<long long>(msg[u[q]] + static_cast<int64_t>(w[q]));
                            best = c < best ? c : best;
                        }
                    }
                }
            }
        }
        int take = 0, fb = -1;
        unsigned int fl = 0;
        int64_t td = 0;
        if (best < dv) {
            const long long old = atomicMin(reinterpret_cast<long long*>(&dist[v]), best);
            if (best < old) {
                const uint64_t bit = 1ULL << (v & 63);
                const unsigned long long ob = atomicOr(reinterpret_cast<unsigned long long*>(&pend[v >> 6]), bit);
                if (!(ob & bit) && best < thr) {
                    take = 1;
                    td = light_deg(ws_off, light, v);
                } else {
                    const int64_t ahead = best / delta - bucket;
                    if (ahead >= nbins || ahead < 0) {
                        spill = true;
                    } else {
                        fb = static_cast<int>((bucket + ahead) % nbins);
                        fl = atomicAdd(&s_bn[fb], 1u);
                    }
                }
            }
        }
        int64_t slot, doff;
        block_reserve(&L->qc[cur ^ 1], take, td, slot, doff);
        if (take) {
            qn[slot] = static_cast<int32_t>(v);
            qpre_n[slot] = doff;
        }
        __syncthreads();
        if (threadIdx.x < nbins) {
            const unsigned int cnt = s_bn[threadIdx.x];
            s_bb[threadIdx.x] = cnt ? atomicAdd(&L->bc[threadIdx.x], static_cast<unsigned long long>(cnt)) : 0ULL;
            if (cnt && s_bb[threadIdx.x] + cnt > static_cast<unsigned long long>(cap))
                atomicOr(&L->overflow, 1ULL << threadIdx.x);
        }
        __syncthreads();
        if (fb >= 0) {
            const unsigned long long sl = s_bb[fb] + fl;
            if (sl < static_cast<unsigned long long>(cap)) pile[fb * cap + static_cast<int64_t>(sl)] = static_cast<int32_t>(v);
        }
        __syncthreads();
    }
    if (__ballot(bad) && lane() == 0) L->err = 1;
    if (__ballot(spill) && lane() == 0) L->spill = 1;
}

// One thread, at the start of a step: the decision of decide_next.  (Folding it into the
// relax's last block — a ticket counter — measured 13.3 -> 24.8 ms per source, most likely
// the agent-scope fence every block issues before taking its ticket.)
__global__ void ds_decide(DsLoop* L, int cur, int64_t delta) {
    if (threadIdx.x == 0 && blockIdx.x == 0) decide_next(L, cur, delta);
}
__global__ void ds_decide_bins(DsLoop* L, int cur, int64_t delta, int nbins, int64_t cap, int64_t scan_above,
                               int64_t pull_min) {
    if (threadIdx.x == 0 && blockIdx.x == 0) decide_bins(L, cur, delta, nbins, cap, scan_above, pull_min);
}
// The loop's stop flags (done, err, spill) to host-mapped words, then the sequence number
// (publish_counters' protocol): the host checks a batch while the next one runs.
__global__ void ds_publish(const DsLoop* L, unsigned long long* host, unsigned long long seq) {
    if (threadIdx.x != 0 || blockIdx.x != 0) return;
    __hip_atomic_store(&host[0], L->done, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    __hip_atomic_store(&host[1], L->err, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    __hip_atomic_store(&host[2], L->spill, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    __threadfence_system();
    __hip_atomic_store(&host[kCounterWords], seq, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
}
// After a pull step: the next pull uses the other bitmap / list.
__global__ void ds_pull_flip(DsLoop* L) {
    if (threadIdx.x == 0 && blockIdx.x == 0 && L->xpull) L->pulls += 1;
}

// ---------------------------------------------------------------- small steps
// Most of a run's ~90 steps are tiny: the tail of every bucket (a few queue entries, a few
// hundred edges) and the run's end.  As four launches each, such a step costs ~20-30 us of
// dispatch and host enqueue (profiles/r05t_sssp_timeline.txt: ~5 us per launch back to back,
// ~7.5 us when the host is behind), for microseconds of work.  ds_small_steps runs them in ONE
// block, looping decide -> extract -> commit -> relax with a barrier and an agent-scope acquire
// (L1 invalidate: the other waves' atomics are performed in L2) between the phases — the same
// bodies the grid kernels run, with one block.  It stops at the first step that is not small —
// the queue or the extraction above small_q entries, or the committed queue above small_e
// edges — leaving that step, already decided (and committed when big == 2), to the grid
// kernels launched behind it (ds_*_dc: each returns at once unless big says it has work).
// The queue buffer in use lives in DsLoop::cur, since the host does not know how many steps a
// launch ran.  Not with the done filter or the pull form (the host keeps the four-launch step).
struct DsQ {
    int32_t* q0;
    int32_t* q1;
    int64_t* p0;
    int64_t* p1;
    // selects, not an indexed array: a runtime index into a kernel argument array is a
    // private-memory (scratch) copy
    __device__ int32_t* q(int c) const { return c ? q1 : q0; }
    __device__ int64_t* qp(int c) const { return c ? p1 : p0; }
};

__device__ __forceinline__ void acquire_agent() { __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent"); }

template <int kE>
__global__ void __launch_bounds__(kBlock) ds_small_steps(const int64_t* __restrict__ off,
        const int32_t* __restrict__ adj, const int32_t* __restrict__ wt, const int64_t* __restrict__ light,
        uint64_t* __restrict__ pend, uint64_t* __restrict__ member, int64_t* __restrict__ dist,
        int64_t* __restrict__ msg, DsQ qs, DsLoop* L, int64_t delta, int nbins, int32_t* __restrict__ pile,
        int64_t cap, int32_t* __restrict__ mlist, uint64_t* __restrict__ done, int64_t scan_above, int max_steps,
        int64_t small_q, int64_t small_e, DsPull nopull) {   // nopull: empty (a kernel argument: no scratch copy)
    __shared__ int s_go, s_cur, s_mode;
    if (threadIdx.x == 0 && L->big) {        // the grid kernels ran the previous launch's last step
        L->cur ^= 1ULL;
        L->big = 0;
    }
    for (int step = 0;; ++step) {
        __syncthreads();
        if (threadIdx.x == 0) {
            acquire_agent();
            const int cur = static_cast<int>(L->cur);
            int go = 0;
            if (step < max_steps) {
                decide_bins(L, cur, delta, nbins, cap, scan_above, 0);
                if (!L->done) {
                    const unsigned long long m = L->extract;
                    if (m == 0) {
                        const unsigned long long c = load_agent(&L->qc[cur]);
                        go = qcount(c) <= small_q && qentries(c) <= small_e;
                    } else if (m == 2) {
                        go = static_cast<int64_t>(L->xcount + L->xm) <= small_q;
                    }
                    if (!go) L->big = 1;
                }
            }
            s_go = go;
            s_cur = cur;
            s_mode = static_cast<int>(L->extract);
        }
        __syncthreads();
        if (!s_go) break;                                    // block-uniform
        const int cur = s_cur;
        acquire_agent();
        if (s_mode == 2)
            extract_bins_body(0, 1, off, light, pend, member, dist, L, cur, pile, cap, mlist, done, qs.q(cur),
                              qs.qp(cur), nopull);
        __syncthreads();
        acquire_agent();
        commit_body<true>(0, 1, qs.q(cur), dist, msg, pend, member, L, cur, mlist);
        __syncthreads();
        if (threadIdx.x == 0) {
            acquire_agent();
            s_go = qentries(load_agent(&L->qc[cur])) <= small_e;
            if (!s_go) L->big = 2;                           // committed: the grid relaxes it
        }
        __syncthreads();
        if (!s_go) break;
        acquire_agent();
        relax_body<true, false, false, kE>(0, 1, off, adj, wt, light, qs.q(cur), qs.qp(cur), msg, dist, pend,
                                           qs.q(cur ^ 1), qs.qp(cur ^ 1), L, cur, delta, nbins, pile, cap, nullptr,
                                           0, 0, nullptr, nullptr);
        __syncthreads();
        if (threadIdx.x == 0) {
            L->cur = static_cast<unsigned long long>(cur ^ 1);
            L->small_steps += 1;
        }
    }
}

// The grid kernels behind ds_small_steps, on the step it left (buffer from DsLoop::cur).
__global__ void __launch_bounds__(kBlock) ds_extract_dc(const int64_t* __restrict__ off,
        const int64_t* __restrict__ light, uint64_t* __restrict__ pend, uint64_t* __restrict__ member,
        const int64_t* __restrict__ dist, DsLoop* L, const int32_t* __restrict__ pile, int64_t cap,
        const int32_t* __restrict__ mlist, uint64_t* __restrict__ done, DsQ qs, int64_t n, DsPull nopull) {
    if (L->big != 1) return;                                 // grid-uniform
    const int cur = static_cast<int>(L->cur);
    const unsigned long long mode = L->extract;
    if (mode == 1) {
        extract_scan(off, light, pend, member, n, dist, L, cur, qs.q(cur), qs.qp(cur), done, L->thr, &L->lo);
        return;
    }
    if (mode != 2) return;
    extract_bins_body(blockIdx.x, gridDim.x, off, light, pend, member, dist, L, cur, pile, cap, mlist, done,
                      qs.q(cur), qs.qp(cur), nopull);
}
__global__ void __launch_bounds__(kBlock) ds_commit_dc(DsQ qs, const int64_t* __restrict__ dist,
        int64_t* __restrict__ msg, uint64_t* __restrict__ pend, uint64_t* __restrict__ member, DsLoop* L,
        int32_t* __restrict__ mlist) {
    if (L->big != 1) return;
    const int cur = static_cast<int>(L->cur);
    commit_body<true>(blockIdx.x, gridDim.x, qs.q(cur), dist, msg, pend, member, L, cur, mlist);
}
template <int kE>
__global__ void __launch_bounds__(kBlock) ds_relax_dc(const int64_t* __restrict__ off, const int32_t* __restrict__ adj,
        const int32_t* __restrict__ wt, const int64_t* __restrict__ light, DsQ qs, const int64_t* __restrict__ msg,
        int64_t* __restrict__ dist, uint64_t* __restrict__ pend, DsLoop* L, int64_t delta, int nbins,
        int32_t* __restrict__ pile, int64_t cap) {
    if (L->big == 0) return;
    const int cur = static_cast<int>(L->cur);
    relax_body<true, false, false, kE>(blockIdx.x, gridDim.x, off, adj, wt, light, qs.q(cur), qs.qp(cur), msg, dist,
                                       pend, qs.q(cur ^ 1), qs.qp(cur ^ 1), L, cur, delta, nbins, pile, cap, nullptr,
                                       0, 0, nullptr, nullptr);
}

}  // namespace

static long long env_i64_dl(const char* name, long long dflt) {
    const char* e = std::getenv(name);
    return e ? std::atoll(e) : dflt;
}

hipError_t k_ds_loop_seed(const DevCsr& ws, const int64_t* light, int64_t* dist, int32_t* q, int64_t* qpre, DsLoop* L,
                          int64_t seed, int64_t delta, hipStream_t s) {
    ds_loop_seed<<<1, 64, 0, s>>>(ws.off, light, dist, q, qpre, L, seed, delta);
    return hipGetLastError();
}

// One step (decide, extract if decided, commit, relax) of the device-driven loop, queue
// buffer `cur` in.
hipError_t k_ds_loop_step(const DevCsr& ws, const int64_t* light, uint64_t* pend, uint64_t* member, int64_t n,
                          int64_t* dist, int64_t* msg, int32_t* const q[2], int64_t* const qpre[2], DsLoop* L, int cur,
                          int64_t delta, hipStream_t s) {
    ds_decide<<<1, 64, 0, s>>>(L, cur, delta);
    const int64_t words = (n + 63) / 64;
    ds_extract_dev<<<extract_grid(words), kBlock, 0, s>>>(ws.off, light, pend, member, n, dist, L, cur, q[cur], qpre[cur]);
    ds_commit_dev<false><<<1024, kBlock, 0, s>>>(q[cur], dist, msg, pend, member, L, cur, nullptr);
    ds_relax_dev<false><<<256 * 8, kBlock, 0, s>>>(ws.off, ws.adj, ws.w, light, q[cur], qpre[cur], msg, dist, pend,
                                                   q[cur ^ 1], qpre[cur ^ 1], L, cur, delta, 0, nullptr, 0, nullptr);
    return hipGetLastError();
}

hipError_t k_ds_part_relax(const DevCsr& ws, const int64_t* light, uint64_t* pend, uint64_t* member, int64_t* dist,
                           int64_t* msg, int32_t* const q[2], int64_t* const qpre[2], DsLoop* L, int cur, int64_t delta,
                           int64_t lo, int64_t n_local, int64_t* rbest, uint64_t* rmark, hipStream_t s) {
    static const int cg = static_cast<int>(env_i64_dl("TGO_DS_CGRID", 1024));
    ds_commit_dev<false><<<cg, kBlock, 0, s>>>(q[cur], dist, msg, pend, member, L, cur, nullptr);
    ds_relax_dev<false, true><<<256 * 8, kBlock, 0, s>>>(ws.off, ws.adj, ws.w, light, q[cur], qpre[cur], msg, dist, pend,
                                                         q[cur ^ 1], qpre[cur ^ 1], L, cur, delta, 0, nullptr, 0,
                                                         nullptr, lo, n_local, rbest, rmark);
    return hipGetLastError();
}
hipError_t k_ds_part_header(unsigned long long* counts, int nranks, DsLoop* L, int cur, unsigned long long* offs,
                            unsigned long long* cursor, int64_t* sizes, hipStream_t s, unsigned long long* host,
                            unsigned long long seq) {
    if (host && nranks != 1) return hipErrorInvalidValue;
    ds_part_header<<<1, 64, 0, s>>>(counts, nranks, L, cur, offs, cursor, sizes, host, seq);
    return hipGetLastError();
}
hipError_t k_ds_part_apply(const int64_t* recv, int64_t npairs, const DevCsr& ws, const int64_t* light, int64_t* dist,
                           uint64_t* pend, int32_t* const q[2], int64_t* const qpre[2], DsLoop* L, int cur, hipStream_t s) {
    if (npairs <= 0) return hipSuccess;
    const int64_t g = std::min<int64_t>(4096, (npairs + kBlock - 1) / kBlock);
    ds_part_apply<<<static_cast<int>(g), kBlock, 0, s>>>(recv, npairs, ws.off, light, dist, pend, q[cur ^ 1],
                                                         qpre[cur ^ 1], L, cur);
    return hipGetLastError();
}
hipError_t k_ds_part_extract(const DevCsr& ws, const int64_t* light, uint64_t* pend, uint64_t* member, int64_t n,
                             int64_t* dist, int32_t* const q[2], int64_t* const qpre[2], DsLoop* L, int cur, int64_t thr,
                             hipStream_t s) {
    const int64_t words = (n + 63) / 64;
    // two words a wave in flight (profiles/r06pq_part_sssp_scan_ab.log, r06pr_*: summed over 3
    // roots at world 1, 1 / 2 / 4 / 8 words 35.9 / 34.2-34.5 / 34.8-35.0 / 38.0 ms; grid 1024 / 4096 with 2
    // words 38.4 / 35.2: extract_grid's 2048 kept)
    ds_part_extract<2><<<extract_grid(words), kBlock, 0, s>>>(ws.off, light, pend, member, n, dist, L, cur, q[cur],
                                                              qpre[cur], thr);
    return hipGetLastError();
}

// One step of the binned loop: decide, extract (piles, or the bitmap scan for a pile that
// overflowed — each kernel returns at once unless its mode was decided), commit, relax.
hipError_t k_ds_publish(const DsLoop* L, unsigned long long* host, unsigned long long seq, hipStream_t s) {
    ds_publish<<<1, 64, 0, s>>>(L, host, seq);
    return hipGetLastError();
}
// TGO_DS_SMALL_Q / _E / _STEPS: a small step has at most small_q queue (or extraction)
// entries and small_e edges; one launch runs at most _STEPS steps
hipError_t k_ds_loop_step_small(const DevCsr& ws, const int64_t* light, uint64_t* pend, uint64_t* member, int64_t n,
                                int64_t* dist, int64_t* msg, int32_t* const q[2], int64_t* const qpre[2], DsLoop* L,
                                int64_t delta, int nbins, int32_t* pile, int64_t cap, int32_t* mlist, uint64_t* done,
                                int64_t scan_above, hipStream_t s) {
    if (nbins < 2 || nbins > kDsMaxBins || nbins > kBlock || cap < 1) return hipErrorInvalidValue;
    static const int64_t sq = env_i64_dl("TGO_DS_SMALL_Q", 1024);
    static const int64_t se = env_i64_dl("TGO_DS_SMALL_E", 4096);
    static const int ss = static_cast<int>(env_i64_dl("TGO_DS_SMALL_STEPS", 64));
    static const int cg = static_cast<int>(env_i64_dl("TGO_DS_CGRID", 1024));
    static const int rg = static_cast<int>(env_i64_dl("TGO_DS_RGRID", 256 * 8));
    const DsQ qs{q[0], q[1], qpre[0], qpre[1]};
    ds_small_steps<kDsRelaxE><<<1, kBlock, 0, s>>>(ws.off, ws.adj, ws.w, light, pend, member, dist, msg, qs, L, delta,
                                                   nbins, pile, cap, mlist, done, scan_above, ss, sq, se, DsPull{});
    const int64_t words = (n + 63) / 64;
    ds_extract_dc<<<extract_grid(words), kBlock, 0, s>>>(ws.off, light, pend, member, dist, L, pile, cap, mlist, done,
                                                         qs, n, DsPull{});
    ds_commit_dc<<<cg, kBlock, 0, s>>>(qs, dist, msg, pend, member, L, mlist);
    ds_relax_dc<kDsRelaxE><<<rg, kBlock, 0, s>>>(ws.off, ws.adj, ws.w, light, qs, msg, dist, pend, L, delta, nbins,
                                                 pile, cap);
    return hipGetLastError();
}

hipError_t k_ds_loop_step_bins(const DevCsr& ws, const int64_t* light, uint64_t* pend, uint64_t* member, int64_t n,
                               int64_t* dist, int64_t* msg, int32_t* const q[2], int64_t* const qpre[2], DsLoop* L,
                               int cur, int64_t delta, int nbins, int32_t* pile, int64_t cap, int32_t* mlist,
                               uint64_t* done, bool done_filter, int64_t scan_above, const DsPull& pull,
                               hipStream_t s) {
    if (nbins < 2 || nbins > kDsMaxBins || nbins > kBlock || cap < 1) return hipErrorInvalidValue;
    const bool pulls = pull.min_members > 0 && pull.pm[0] && pull.pm[1] && pull.pl[0] && pull.pl[1];
    if (pulls && pull.n_active > n) return hipErrorInvalidValue;
    ds_decide_bins<<<1, 64, 0, s>>>(L, cur, delta, nbins, cap, scan_above, pulls ? pull.min_members : 0);
    const int64_t words = (n + 63) / 64;
    // grids (TGO_DS_XGRID / _CGRID / _RGRID, A/B): most of a run's ~100 steps have tiny queues
    // and no extraction, and a launch of thousands of blocks that exit at once still costs
    // ~10-15 us; the grid-stride loops take any grid
    static const int xg = static_cast<int>(env_i64_dl("TGO_DS_XGRID", 0));
    static const int cg = static_cast<int>(env_i64_dl("TGO_DS_CGRID", 1024));
    static const int rg = static_cast<int>(env_i64_dl("TGO_DS_RGRID", 256 * 8));
    ds_extract_bins<<<xg > 0 ? std::min(xg, extract_grid(words)) : extract_grid(words), kBlock, 0, s>>>(ws.off, light, pend, member, dist, L, cur, pile, cap, mlist,
                                                           done, q[cur], qpre[cur], n, pull);
    ds_commit_dev<true><<<cg, kBlock, 0, s>>>(q[cur], dist, msg, pend, member, L, cur, mlist);
    if (pulls) {
        ds_pull_heavy<<<256 * 8, kBlock, 0, s>>>(ws.off, light, msg, dist, pend, q[cur ^ 1], qpre[cur ^ 1], L, cur, delta,
                                                 nbins, pile, cap, pull);
        ds_pull_flip<<<1, 64, 0, s>>>(L);
    }
    // TGO_DS_RELAX_E=5 (A/B): the round-5 entries per thread of the binned relax (default kDsRelaxE)
    static const int re = static_cast<int>(env_i64_dl("TGO_DS_RELAX_E", kDsRelaxE));
    if (!done_filter && re == 5) {
        ds_relax_dev<true, false, false, 5><<<rg, kBlock, 0, s>>>(ws.off, ws.adj, ws.w, light, q[cur], qpre[cur], msg,
                                                                  dist, pend, q[cur ^ 1], qpre[cur ^ 1], L, cur, delta,
                                                                  nbins, pile, cap, nullptr);
    } else if (done_filter)
        ds_relax_dev<true, false, true><<<rg, kBlock, 0, s>>>(ws.off, ws.adj, ws.w, light, q[cur], qpre[cur], msg, dist,
                                                              pend, q[cur ^ 1], qpre[cur ^ 1], L, cur, delta, nbins, pile,
                                                              cap, done);
    else
        ds_relax_dev<true><<<rg, kBlock, 0, s>>>(ws.off, ws.adj, ws.w, light, q[cur], qpre[cur], msg, dist, pend,
                                                 q[cur ^ 1], qpre[cur ^ 1], L, cur, delta, nbins, pile, cap, nullptr);
    return hipGetLastError();
}

}  // namespace tgo

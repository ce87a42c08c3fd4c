// frontier.hpp — device building blocks shared by the frontier kernels (bfs.hip, delta.hip,
// msbfs.hip): edge-balanced load-balanced search over a vertex queue, block-aggregated
// queue appends, and two-pass bitmap extraction.  Include from exactly those .hip files
// (everything here is in an anonymous namespace, one copy per translation unit).
#pragma once
#include <hip/hip_runtime.h>
#include "engine.hpp"

namespace tgo {
namespace {

constexpr int kBlock = 256;
constexpr int kWavesPerBlock = kBlock / 64;
constexpr int kEdgesPerThread = 8;
constexpr int kTileEdges = kBlock * kEdgesPerThread;   // 2048 queue entries' edges per block tile
constexpr int kLdsEntries = kTileEdges + 2;

__device__ __forceinline__ int lane() { return static_cast<int>(threadIdx.x & 63); }

// Entries of u over the one or two lists of a view.
__device__ __forceinline__ int64_t push_degree(const View& v, int64_t u) {
    int64_t d = v.off0[u + 1] - v.off0[u];
    if (v.nlists > 1) d += v.off1[u + 1] - v.off1[u];
    return d;
}

// Entry `o` (0 <= o < push_degree(u)) of u's list(s): neighbour and weight (1 if unweighted).
__device__ __forceinline__ void entry_at(const View& v, int64_t u, int64_t o, int32_t& nbr, int32_t& w) {
    const int64_t b0 = v.off0[u];
    const int64_t d0 = v.off0[u + 1] - b0;
    if (o < d0) {
        nbr = v.adj0[b0 + o];
        w = v.w0 ? v.w0[b0 + o] : 1;
    } else {
        const int64_t b1 = v.off1[u] + (o - d0);
        nbr = v.adj1[b1];
        w = v.w1 ? v.w1[b1] : 1;
    }
}

// A tile's queue bounds, by one whole wave: the last i in [a, b) with pre[i] <= key, given
// pre[a] <= key and pre nondecreasing — 64 probes a round (log64 rounds) instead of a lane-0
// binary search (~20 dependent loads a tile while the block waits at its barrier).  Every lane
// of the calling wave gets the result.
__device__ __forceinline__ int64_t wave_last_le(const int64_t* __restrict__ pre, int64_t a, int64_t b, int64_t key) {
    while (b - a > 1) {                                   // wave-uniform
        const int64_t step = (b - a + 63) >> 6;
        const int64_t pos = a + static_cast<int64_t>(threadIdx.x & 63) * step;
        const bool le = pos < b && pre[pos < b ? pos : a] <= key;
        const unsigned long long m = __ballot(le);       // a prefix of the lanes; lane 0 always
        const int k = 63 - __clzll(static_cast<long long>(m));
        a += static_cast<int64_t>(k) * step;
        b = min(b, a + step);
    }
    return a;
}
// lo = last i with pre[i] <= t0, hi = last i with pre[i] <= t1 - 1, by the block's first wave
__device__ __forceinline__ void tile_bounds(const int64_t* __restrict__ pre, int64_t n, int64_t t0, int64_t t1,
                                            int64_t& s_lo, int64_t& s_hi) {
    if (threadIdx.x < 64) {
        const int64_t lo = wave_last_le(pre, 0, n, t0);
        const int64_t hi = wave_last_le(pre, lo, n, t1 - 1);
        if (threadIdx.x == 0) { s_lo = lo; s_hi = hi; }
    }
}

// Edge-balanced load-balanced search (Merrill et al., PPoPP'12) over a queue q[0..qlen) whose
// entries' edge counts have the exclusive scan qpre[0..qlen] (qpre[qlen] = total).  The edge
// space is cut into kTileEdges tiles; a block stages the scan entries its tile touches in
// LDS (when they fit) and every thread binary-searches the queue entry of each of its
// kEdgesPerThread edges.  body(valid, entry, offset) is called by EVERY thread of the block
// for every k in the same trip (block-uniform, so it may synchronise the block, e.g. via
// block_append); valid = the edge exists, entry = q[i] of the owning queue slot, offset = the
// edge's position inside that entry's list.
template <class Body>
__device__ __forceinline__ void for_each_queue_edge(const int32_t* __restrict__ q, const int64_t* __restrict__ qpre,
                                                    int64_t qlen, Body&& body) {
    __shared__ int64_t s_pre[kLdsEntries];
    __shared__ int32_t s_q[kLdsEntries];
    __shared__ int64_t s_lo, s_hi;
    const int64_t total = qpre[qlen];
    const int64_t ntiles = (total + kTileEdges - 1) / kTileEdges;
    for (int64_t tile = blockIdx.x; tile < ntiles; tile += gridDim.x) {
        const int64_t t0 = tile * kTileEdges;
        const int64_t t1 = min(total, t0 + kTileEdges);
        tile_bounds(qpre, qlen, t0, t1, s_lo, s_hi);   // lo = last i with qpre[i] <= t0; hi = last with <= t1-1
        __syncthreads();
        const int64_t lo = s_lo, hi = s_hi;
        const int64_t span = hi - lo + 1;   // queue entries touching this tile
        const bool in_lds = span + 1 <= kLdsEntries;
        if (in_lds) {
            for (int64_t i = threadIdx.x; i <= span; i += kBlock) {
                s_pre[i] = qpre[lo + i];
                if (i < span) s_q[i] = q[lo + i];
            }
        }
        __syncthreads();
        for (int k = 0; k < kEdgesPerThread; ++k) {
            const int64_t j = t0 + k * kBlock + threadIdx.x;
            int32_t entry = 0;
            int64_t start = j;
            const bool valid = j < t1;
            if (valid) {
                if (in_lds) {
                    int64_t a = 0, b = span;
                    while (b - a > 1) { const int64_t c = (a + b) >> 1; if (s_pre[c] <= j) a = c; else b = c; }
                    entry = s_q[a]; start = s_pre[a];
                } else {
                    int64_t a = lo, b = hi + 1;
                    while (b - a > 1) { const int64_t c = (a + b) >> 1; if (qpre[c] <= j) a = c; else b = c; }
                    entry = q[a]; start = qpre[a];
                }
            }
            body(valid, entry, j - start);
        }
        __syncthreads();
    }
}

// Block-aggregated append (all threads of the block call it in the same trip): the block
// reserves its queue slots with ONE atomicAdd on cnt->qlen; the appended degrees stay in
// registers (mf) until block_flush.  A single contended counter word serves ~88 atomics/us
// (MI355X_MICROARCH.md, dequeue), so per-wave counter atomics dominated the dense levels.
struct AppendLds { unsigned long long off[kWavesPerBlock]; unsigned long long base; unsigned long long mf[kWavesPerBlock]; };
__device__ __forceinline__ void block_append(bool take, int32_t v, int64_t deg, int32_t* qn, int64_t* qdeg,
                                             Counters* cnt, AppendLds& sh, unsigned long long& mf) {
    const unsigned long long mask = __ballot(take);
    const int wave = threadIdx.x >> 6;
    if (mask) {
        int64_t dsum = take ? deg : 0;
        for (int off = 32; off > 0; off >>= 1) dsum += __shfl_xor(dsum, off, 64);
        mf += static_cast<unsigned long long>(dsum);
    }
    if (lane() == 0) sh.off[wave] = static_cast<unsigned long long>(__popcll(mask));
    __syncthreads();
    if (threadIdx.x == 0) {
        unsigned long long t = 0;
        for (int w = 0; w < kWavesPerBlock; ++w) { const unsigned long long c = sh.off[w]; sh.off[w] = t; t += c; }
        sh.base = t ? atomicAdd(&cnt->qlen, t) : 0ULL;
    }
    __syncthreads();
    if (take) {
        const unsigned long long slot = sh.base + sh.off[wave] + static_cast<unsigned long long>(__popcll(mask & ((1ULL << lane()) - 1ULL)));
        qn[slot] = v;
        qdeg[slot] = deg;
    }
}
__device__ __forceinline__ void block_flush(Counters* cnt, AppendLds& sh, unsigned long long mf) {
    __syncthreads();
    if (lane() == 0) sh.mf[threadIdx.x >> 6] = mf;
    __syncthreads();
    if (threadIdx.x == 0) {
        unsigned long long a = 0;
        for (int w = 0; w < kWavesPerBlock; ++w) a += sh.mf[w];
        if (a) atomicAdd(&cnt->mf, a);
    }
}

// End of a counting kernel: per-thread sums of the next frontier (vertices, push entries)
// reduced over the block, one atomicAdd per block and counter (no per-trip barrier).
__device__ __forceinline__ void count_flush(Counters* cnt, unsigned long long nv, unsigned long long mf) {
    __shared__ unsigned long long s_nv[kWavesPerBlock], s_mf[kWavesPerBlock];
    for (int off = 32; off > 0; off >>= 1) {
        nv += __shfl_xor(nv, off, 64);
        mf += __shfl_xor(mf, off, 64);
    }
    if (lane() == 0) { s_nv[threadIdx.x >> 6] = nv; s_mf[threadIdx.x >> 6] = mf; }
    __syncthreads();
    if (threadIdx.x == 0) {
        unsigned long long a = 0, m = 0;
        for (int w = 0; w < kWavesPerBlock; ++w) { a += s_nv[w]; m += s_mf[w]; }
        if (a) atomicAdd(&cnt->qlen, a);
        if (m) atomicAdd(&cnt->mf, m);
    }
}

// Bitmap extraction into a queue, two passes over a contiguous chunk of 64-vertex words per
// block (one wave per word): pass 1 counts what the chunk takes, one atomicAdd per block
// reserves its slots, pass 2 re-reads (L2-warm) and writes.  No per-trip block barriers or
// counter atomics, which dominated the one-pass form (~200 us per extraction at 16M
// vertices).  probe(wd, takes, commit) fills up to kStreams (take, entry, degree) per lane and
// returns whether the word needs pass 2 (it takes something or, with commit, writes
// something); with commit it also applies its writes (one writer per word) — pass 1 never
// writes, so both passes see the same state.  Both passes keep kUnroll words in flight per
// wave (one word per trip left each wave waiting a memory latency per word), and pass 2
// visits only the words pass 1 flagged (a wave's first 64 words by a bit mask; a longer
// chunk visits all).
struct Take { bool take; int32_t entry; int64_t deg; };
constexpr int kExtractUnroll = 4;
// Pass 1 of a wave's words [first, end) step kWavesPerBlock: per-lane take counts and degree
// sums, the flagged-word mask (bit i = i-th word of the wave), and whether any word was flagged.
template <int kStreams, class Probe>
__device__ __forceinline__ void extract_count(int64_t first, int64_t end, const Probe& probe, int64_t& count,
                                              int64_t& dsum, unsigned long long& mask, bool& touch) {
    int64_t wd = first;
    int idx = 0;
    for (; wd + (kExtractUnroll - 1) * kWavesPerBlock < end; wd += kExtractUnroll * kWavesPerBlock, idx += kExtractUnroll) {
        Take t[kExtractUnroll][kStreams];
        bool r[kExtractUnroll];
#pragma unroll
        for (int u = 0; u < kExtractUnroll; ++u) r[u] = probe(wd + u * kWavesPerBlock, t[u], false);
#pragma unroll
        for (int u = 0; u < kExtractUnroll; ++u) {
            if (r[u]) { touch = true; if (idx + u < 64) mask |= 1ULL << (idx + u); }
            for (int k = 0; k < kStreams; ++k)
                if (t[u][k].take) { ++count; dsum += t[u][k].deg; }
        }
    }
    for (; wd < end; wd += kWavesPerBlock, ++idx) {
        Take t[kStreams];
        if (probe(wd, t, false)) { touch = true; if (idx < 64) mask |= 1ULL << idx; }
        for (int k = 0; k < kStreams; ++k)
            if (t[k].take) { ++count; dsum += t[k].deg; }
    }
}
// Pass 2: the flagged words in order (all words when the wave has more than 64), kUnroll
// probes in flight, then emit(takes) per word in order.
template <int kStreams, class Probe, class Emit>
__device__ __forceinline__ void extract_write(int64_t first, int64_t end, unsigned long long mask, const Probe& probe,
                                              const Emit& emit) {
    const int64_t nwords = end > first ? (end - first + kWavesPerBlock - 1) / kWavesPerBlock : 0;
    const bool all = nwords > 64;
    int64_t next = 0;                        // (all) next word index to visit
    for (;;) {
        int64_t wl[kExtractUnroll];
        bool any = false;
#pragma unroll
        for (int u = 0; u < kExtractUnroll; ++u) {
            wl[u] = -1;
            if (all) {
                if (next < nwords) wl[u] = first + (next++) * kWavesPerBlock;
            } else if (mask) {
                const int b = __ffsll(static_cast<long long>(mask)) - 1;
                mask &= mask - 1;
                wl[u] = first + static_cast<int64_t>(b) * kWavesPerBlock;
            }
            any |= wl[u] >= 0;
        }
        if (!any) break;                      // wave-uniform
        Take t[kExtractUnroll][kStreams];
#pragma unroll
        for (int u = 0; u < kExtractUnroll; ++u)
            if (wl[u] >= 0) probe(wl[u], t[u], true);
#pragma unroll
        for (int u = 0; u < kExtractUnroll; ++u)
            if (wl[u] >= 0) emit(t[u]);
    }
}
// Staged probes (Probe::State, stage1 / stage2 / finish): the kExtractUnroll words' loads
// issued stage by stage — stage 1 (word loads) for all of them, then stage 2 (per-lane loads
// that depend on the words, under a per-lane condition) for all of them, then the uses.  A
// conditional load whose value is used right away made the compiler wait for every load in
// flight, so the unrolled words of a plain probe ran one dependent chain after the other.
// The wave's words in windows of 64: one word a lane asks which can take anything
// (Probe::live, one load round trip a window), and the stages run on those only — a sparse
// scan (the tail of a run: a few pending vertices in 16 M) costs a round trip a window instead
// of one per kU words.  live_words calls visit(wl, bi, st) per kU live words with their
// stages 1 and 2 issued (live_words_plain below: bi = index within the wave's words, -1 for an
// unused slot, whose wl is `first`).
template <int kU, class Live, class Visit>
__device__ __forceinline__ void live_words_plain(int64_t first, int64_t nwords, const Live& live, const Visit& visit);
template <class Probe, int kU, class Visit>
__device__ __forceinline__ void live_words(int64_t first, int64_t nwords, const Probe& probe, const Visit& visit) {
    live_words_plain<kU>(first, nwords, [&](int64_t wd) { return probe.live(wd); }, [&](const int64_t* wl, const int* bi) {
        typename Probe::State st[kU];
#pragma unroll
        for (int u = 0; u < kU; ++u) probe.stage1(wl[u], st[u]);
#pragma unroll
        for (int u = 0; u < kU; ++u) probe.stage2(wl[u], st[u]);
        visit(wl, bi, st);
    });
}
// Pass 1 over the live words: the takes counted, the touched words of a wave of <= 64 words
// flagged for pass 2.
template <int kStreams, class Probe, int kU = kExtractUnroll>
__device__ __forceinline__ void extract_count_staged(int64_t first, int64_t end, const Probe& probe, int64_t& count,
                                                     int64_t& dsum, unsigned long long& mask, bool& touch) {
    const int64_t nwords = end > first ? (end - first + kWavesPerBlock - 1) / kWavesPerBlock : 0;
    live_words<Probe, kU>(first, nwords, probe, [&](const int64_t* wl, const int* bi, const typename Probe::State* st) {
#pragma unroll
        for (int u = 0; u < kU; ++u) {
            if (bi[u] < 0) continue;
            Take t[kStreams];
            if (probe.finish(wl[u], st[u], t, false)) { touch = true; if (bi[u] < 64) mask |= 1ULL << bi[u]; }
            for (int k = 0; k < kStreams; ++k)
                if (t[k].take) { ++count; dsum += t[k].deg; }
        }
    });
}
// Pass 2: the flagged words in order (a wave of <= 64 words), else the live words again.
template <int kStreams, class Probe, class Emit, int kU = kExtractUnroll>
__device__ __forceinline__ void extract_write_staged(int64_t first, int64_t end, unsigned long long mask, const Probe& probe,
                                                     const Emit& emit) {
    const int64_t nwords = end > first ? (end - first + kWavesPerBlock - 1) / kWavesPerBlock : 0;
    if (nwords > 64) {
        live_words<Probe, kU>(first, nwords, probe, [&](const int64_t* wl, const int* bi, const typename Probe::State* st) {
            Take t[kU][kStreams];
#pragma unroll
            for (int u = 0; u < kU; ++u)
                if (bi[u] >= 0) probe.finish(wl[u], st[u], t[u], true);
#pragma unroll
            for (int u = 0; u < kU; ++u)
                if (bi[u] >= 0) emit(t[u]);
        });
        return;
    }
    while (mask) {                            // wave-uniform
        int64_t wl[kU];
#pragma unroll
        for (int u = 0; u < kU; ++u) {
            wl[u] = -1;
            if (mask) {
                const int b = __ffsll(static_cast<long long>(mask)) - 1;
                mask &= mask - 1;
                wl[u] = first + static_cast<int64_t>(b) * kWavesPerBlock;
            }
        }
        typename Probe::State st[kU];
#pragma unroll
        for (int u = 0; u < kU; ++u) probe.stage1(wl[u] >= 0 ? wl[u] : first, st[u]);
#pragma unroll
        for (int u = 0; u < kU; ++u) probe.stage2(wl[u] >= 0 ? wl[u] : first, st[u]);
        Take t[kU][kStreams];
#pragma unroll
        for (int u = 0; u < kU; ++u)
            if (wl[u] >= 0) probe.finish(wl[u], st[u], t[u], true);
#pragma unroll
        for (int u = 0; u < kU; ++u)
            if (wl[u] >= 0) emit(t[u]);
    }
}

template <int kStreams, class Probe>
__device__ __forceinline__ void chunk_extract(int64_t words, const Probe& probe, int32_t* __restrict__ qn,
                                              int64_t* __restrict__ qdeg, Counters* cnt) {
    __shared__ unsigned long long s_cnt[kWavesPerBlock], s_mf[kWavesPerBlock], s_base;
    const int64_t per = ((words + gridDim.x - 1) / gridDim.x + kWavesPerBlock - 1) / kWavesPerBlock * kWavesPerBlock;
    const int64_t w0 = static_cast<int64_t>(blockIdx.x) * per;
    const int64_t w1 = min(words, w0 + per);
    const int wave = threadIdx.x >> 6;
    const unsigned long long below = (1ULL << lane()) - 1ULL;
    int64_t count = 0, dsum = 0;
    unsigned long long mask = 0;
    bool touch = false;
    extract_count<kStreams>(w0 + wave, w1, probe, count, dsum, mask, touch);
    unsigned long long c = static_cast<unsigned long long>(count), m = static_cast<unsigned long long>(dsum);
    for (int o = 32; o > 0; o >>= 1) { c += __shfl_xor(c, o, 64); m += __shfl_xor(m, o, 64); }
    if (lane() == 0) { s_cnt[wave] = c; s_mf[wave] = m; }
    __syncthreads();
    if (threadIdx.x == 0) {
        unsigned long long t = 0, mm = 0;
        for (int w = 0; w < kWavesPerBlock; ++w) { const unsigned long long x = s_cnt[w]; s_cnt[w] = t; t += x; mm += s_mf[w]; }
        s_base = t ? atomicAdd(&cnt->qlen, t) : 0ULL;
        if (mm) atomicAdd(&cnt->mf, mm);
    }
    __syncthreads();
    if (!touch) return;                                      // wave-uniform
    unsigned long long cursor = s_base + s_cnt[wave];
    extract_write<kStreams>(w0 + wave, w1, mask, probe, [&](const Take* t) {
        for (int k = 0; k < kStreams; ++k) {
            const unsigned long long bm = __ballot(t[k].take);
            if (t[k].take) {
                const unsigned long long slot = cursor + __popcll(bm & below);
                qn[slot] = t[k].entry;
                qdeg[slot] = t[k].deg;
            }
            cursor += __popcll(bm);
        }
    });
}

// The live words of a wave, kU at a time (see live_words).
template <int kU, class Live, class Visit>
__device__ __forceinline__ void live_words_plain(int64_t first, int64_t nwords, const Live& live, const Visit& visit) {
    for (int64_t w0 = 0; w0 < nwords; w0 += 64) {                // wave-uniform
        const int64_t base = first + w0 * kWavesPerBlock;
        const int64_t nw = nwords - w0 < 64 ? nwords - w0 : 64;
        const bool in = lane() < nw;
        unsigned long long lv = __ballot(in && live(in ? base + static_cast<int64_t>(lane()) * kWavesPerBlock : first));
        while (lv) {                                              // wave-uniform
            int64_t wl[kU];
            int bi[kU];
#pragma unroll
            for (int u = 0; u < kU; ++u) {
                bi[u] = -1;
                wl[u] = first;
                if (lv) {
                    const int b = __ffsll(static_cast<long long>(lv)) - 1;
                    lv &= lv - 1;
                    bi[u] = static_cast<int>(w0) + b;
                    wl[u] = base + static_cast<int64_t>(b) * kWavesPerBlock;
                }
            }
            visit(wl, bi);
        }
    }
}
// chunk_extract for a sparse bitmap: live(wd) says whether word wd can take anything (a
// cheap load), one word a lane per 64-word window, and both passes probe the live words only
// (the queue after a bottom-up level: the frontier is a few thousand vertices in 16 M, and a
// wave's 32 words cost 8 dependent round trips a pass at 4 in flight).
template <int kStreams, class Live, class Probe>
__device__ __forceinline__ void chunk_extract_live(int64_t words, const Live& live, const Probe& probe,
                                                   int32_t* __restrict__ qn, int64_t* __restrict__ qdeg, Counters* cnt) {
    __shared__ unsigned long long s_cnt[kWavesPerBlock], s_mf[kWavesPerBlock], s_base;
    const int64_t per = ((words + gridDim.x - 1) / gridDim.x + kWavesPerBlock - 1) / kWavesPerBlock * kWavesPerBlock;
    const int64_t w0 = static_cast<int64_t>(blockIdx.x) * per;
    const int64_t w1 = min(words, w0 + per);
    const int wave = threadIdx.x >> 6;
    const unsigned long long below = (1ULL << lane()) - 1ULL;
    const int64_t first = w0 + wave;
    const int64_t nwords = w1 > first ? (w1 - first + kWavesPerBlock - 1) / kWavesPerBlock : 0;
    int64_t count = 0, dsum = 0;
    unsigned long long mask = 0;
    bool touch = false;
    live_words_plain<kExtractUnroll>(first, nwords, live, [&](const int64_t* wl, const int* bi) {
        Take t[kExtractUnroll][kStreams];
        bool r[kExtractUnroll];
#pragma unroll
        for (int u = 0; u < kExtractUnroll; ++u) r[u] = bi[u] >= 0 && probe(wl[u], t[u], false);
#pragma unroll
        for (int u = 0; u < kExtractUnroll; ++u) {
            if (bi[u] < 0) continue;
            if (r[u]) { touch = true; if (bi[u] < 64) mask |= 1ULL << bi[u]; }
            for (int k = 0; k < kStreams; ++k)
                if (t[u][k].take) { ++count; dsum += t[u][k].deg; }
        }
    });
    unsigned long long c = static_cast<unsigned long long>(count), m = static_cast<unsigned long long>(dsum);
    for (int o = 32; o > 0; o >>= 1) { c += __shfl_xor(c, o, 64); m += __shfl_xor(m, o, 64); }
    if (lane() == 0) { s_cnt[wave] = c; s_mf[wave] = m; }
    __syncthreads();
    if (threadIdx.x == 0) {
        unsigned long long t = 0, mm = 0;
        for (int w = 0; w < kWavesPerBlock; ++w) { const unsigned long long x = s_cnt[w]; s_cnt[w] = t; t += x; mm += s_mf[w]; }
        s_base = t ? atomicAdd(&cnt->qlen, t) : 0ULL;
        if (mm) atomicAdd(&cnt->mf, mm);
    }
    __syncthreads();
    if (!touch) return;                                      // wave-uniform
    unsigned long long cursor = s_base + s_cnt[wave];
    const auto emit = [&](const Take* t) {
        for (int k = 0; k < kStreams; ++k) {
            const unsigned long long bm = __ballot(t[k].take);
            if (t[k].take) {
                const unsigned long long slot = cursor + __popcll(bm & below);
                qn[slot] = t[k].entry;
                qdeg[slot] = t[k].deg;
            }
            cursor += __popcll(bm);
        }
    };
    if (nwords <= 64) {
        extract_write<kStreams>(first, w1, mask, probe, emit);
        return;
    }
    live_words_plain<kExtractUnroll>(first, nwords, live, [&](const int64_t* wl, const int* bi) {
        Take t[kExtractUnroll][kStreams];
#pragma unroll
        for (int u = 0; u < kExtractUnroll; ++u)
            if (bi[u] >= 0) probe(wl[u], t[u], true);
#pragma unroll
        for (int u = 0; u < kExtractUnroll; ++u)
            if (bi[u] >= 0) emit(t[u]);
    });
}

// Grid for chunk_extract: >= 64 words per block, at most 2048 blocks.
inline int extract_grid(int64_t words) {
    const int64_t g = (words + 63) / 64;
    return static_cast<int>(g < 1 ? 1 : (g > 2048 ? 2048 : g));
}

}  // namespace
}  // namespace tgo

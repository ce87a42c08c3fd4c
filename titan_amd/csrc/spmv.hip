// spmv.hip — pull gathers for PageRankVertexProgram and OLAPTest.DegreeCounter on gfx950.
//
// Both programs gather, for every vertex, a sum over its reversed-scope list of the
// neighbours' previous-superstep messages (VertexMemoryHandler.receiveMessages,
// VertexMemoryHandler.java:77-103):
//   PageRank  (PageRankVertexProgram.java:84-89): PR'(v) = a * sum_{u in IN(v)} c(u) + (1-a)/N,
//             c'(v) = PR'(v) / edgeCount(v)  — fp64 SpMV over the in-CSR.
//   DegreeCounter (OLAPTest.java:357-364): d'(v) = sum_{w in OUT(v)} d(w), Java int wrap.
//
// CSR-Adaptive (Greathouse & Daga, SC'14): rows are cut on the host into blocks of at
// most kTile entries; a 256-thread workgroup stages its block's gathered messages in LDS
// with coalesced index reads, then reduces rows from LDS — thread-per-row when the block
// has many short rows, wave-per-row (fixed shuffle tree) when it has few.  Rows longer
// than kTile are split into kTile chunks reduced by separate workgroups and summed in chunk
// order by a finalize kernel.
//
// PageRank on one GPU is cache-blocked (ColdBlocks, engine.hpp): cold sources are gathered
// segment by segment by workgroups pinned to the XCD that caches the segment (cold_gather),
// their per-(row, segment) sums land in partial[], and the hot pass adds them to each row.
// Every sum has a fixed order: results are bitwise reproducible run to run.
#include <algorithm>
#include <cstdlib>
#include <mutex>
#include <vector>
#include <hip/hip_runtime.h>
#include "engine.hpp"

namespace tgo {
namespace {

constexpr int kBlock = 256;

__device__ __forceinline__ int lane() { return static_cast<int>(threadIdx.x & 63); }

struct PrOp {
    using T = double;
    const double* msg;
    __device__ __forceinline__ double load(int32_t u) const { return msg[u]; }
    __device__ __forceinline__ static double add(double a, double b) { return a + b; }
    __device__ __forceinline__ static double zero() { return 0.0; }
};
// Diagnostic only (TGO_PR_DIAG=lo:hi): gathers of sources outside [lo, hi) are skipped (read
// as 0), so the time attributable to a source range can be measured.  Results are wrong.
struct PrDiagOp {
    using T = double;
    const double* msg; int32_t lo, hi;
    __device__ __forceinline__ double load(int32_t u) const { return (u >= lo && u < hi) ? msg[u] : 0.0; }
    __device__ __forceinline__ static double add(double a, double b) { return a + b; }
    __device__ __forceinline__ static double zero() { return 0.0; }
};
struct WalkOp {
    using T = uint32_t;                     // Java int arithmetic wraps: use unsigned adds
    const int32_t* msg;
    __device__ __forceinline__ uint32_t load(int32_t u) const { return static_cast<uint32_t>(msg[u]); }
    __device__ __forceinline__ static uint32_t add(uint32_t a, uint32_t b) { return a + b; }
    __device__ __forceinline__ static uint32_t zero() { return 0u; }
};

template <class T>
__device__ __forceinline__ T wave_sum(T x) {
    for (int off = 32; off > 0; off >>= 1) x = x + __shfl_xor(x, off, 64);
    return x;
}

// Finalisers: what a vertex does with its gathered sum.
struct PrFinal {
    const double* edge_count; double* pr; double* contrib_next; double alpha; double base;
    // fixed-point layouts: a contribution outside [2^(elo-1023), 2^(ehi-1023)) sets *bad (FxGuard)
    unsigned* bad = nullptr;
    unsigned elo = 0, ehi = 0x800;
    __device__ __forceinline__ void operator()(int64_t r, double sum) const {
        const double p = (alpha * sum) + base;      // PageRankVertexProgram.java:86
        if (pr) pr[r] = p;                          // the PAGE_RANK property: read after the last update only
        // :88, edgeCount 0 => +inf.  It IS read when a row cut (QueryContainer.java:28,122) left
        // the vertex no OUT entry but a neighbour's row still holds its IN entry: the fixed-point
        // passes' first-update entry check flags it (FxGuard; edgeCount never changes), and the
        // program re-runs on the plain fp64 gather.  Every other contribution is checked here.
        const double ec = __builtin_nontemporal_load(edge_count + r);
        const double c = p / ec;
        contrib_next[r] = c;
        if (bad && ec != 0.0) {
            const unsigned long long b = static_cast<unsigned long long>(__double_as_longlong(c));
            const unsigned e = static_cast<unsigned>(b >> 52) & 0x7FFu;
            if ((b << 1) != 0 && e - elo >= ehi - elo) *bad = 1u;
        }
    }
};
// Cache-blocked form: the row's cold sum (its pieces in segment order, cold_fold) is added
// after its hot sum — one coalesced load, no dependent chain in the reduce loop.
struct PrColdFinal {
    PrFinal f; const double* csum;
    __device__ __forceinline__ void operator()(int64_t r, double sum) const { f(r, sum + csum[r]); }
};
struct WalkFinal {
    int32_t* next;
    __device__ __forceinline__ void operator()(int64_t r, uint32_t sum) const { next[r] = static_cast<int32_t>(sum); }
};

// The index stream is read exactly once per superstep: load it non-temporally so it does
// not evict the message vector from L2 / the Infinity Cache, which every gather re-reads.
__device__ __forceinline__ int32_t stream_idx(const int32_t* p) { return __builtin_nontemporal_load(p); }

constexpr int kPer = static_cast<int>(kTile / kBlock);   // entries per thread per tile (16)



// Gather up to kTile messages of the entries [s0, s0+nnz) into registers: all kPer index
// loads are issued first, then all kPer message loads, so every thread keeps kPer
// independent gathers in flight (a dependent load per loop trip leaves the wave waiting
// one memory latency per entry).
template <class Op>
__device__ __forceinline__ void gather_tile(const int32_t* __restrict__ adj, int64_t s0, int64_t nnz, const Op& op,
                                            typename Op::T (&val)[kPer]) {
    int32_t idx[kPer];
#pragma unroll
    for (int j = 0; j < kPer; ++j) {
        const int64_t k = threadIdx.x + static_cast<int64_t>(j) * kBlock;
        idx[j] = k < nnz ? stream_idx(adj + s0 + k) : 0;
    }
    // validity by position: a packed word of a wide slot space may have its top bit set
#pragma unroll
    for (int j = 0; j < kPer; ++j)
        val[j] = threadIdx.x + static_cast<int64_t>(j) * kBlock < nnz ? op.load(idx[j]) : Op::zero();
}

// Stage a tile's gathered messages in LDS.
template <class Op>
__device__ __forceinline__ void stage_tile(const int32_t* __restrict__ adj, int64_t s0, int64_t nnz, const Op& op,
                                           typename Op::T* s_val) {
    typename Op::T val[kPer];
    gather_tile(adj, s0, nnz, op, val);
#pragma unroll
    for (int j = 0; j < kPer; ++j) {
        const int k = threadIdx.x + j * kBlock;
        if (k < nnz) s_val[k] = val[j];
    }
    __syncthreads();
}

// Reduce the runs [off[i], off[i+1]) of items i in [i0, i1) from the staged tile (base s0):
// thread-per-run for many runs, wave-per-run with a fixed shuffle tree for few.
template <class Op, class Emit>
__device__ __forceinline__ void reduce_runs(const int64_t* __restrict__ off, int64_t i0, int64_t i1, int64_t s0,
                                            const typename Op::T* s_val, const Emit& emit) {
    using T = typename Op::T;
    if (i1 - i0 > 64) {
        for (int64_t i = i0 + threadIdx.x; i < i1; i += kBlock) {
            T sum = Op::zero();
            const int64_t e = off[i + 1] - s0;
            for (int64_t k = off[i] - s0; k < e; ++k) sum = Op::add(sum, s_val[k]);
            emit(i, sum);
        }
    } else {
        const int wave = threadIdx.x >> 6;
        for (int64_t i = i0 + wave; i < i1; i += kBlock / 64) {
            T sum = Op::zero();
            const int64_t e = off[i + 1] - s0;
            for (int64_t k = off[i] - s0 + lane(); k < e; k += 64) sum = Op::add(sum, s_val[k]);
            sum = wave_sum(sum);
            if (lane() == 0) emit(i, sum);
        }
    }
}

template <class Op, class Fin>
__global__ void __launch_bounds__(kBlock) gather_short(const int64_t* __restrict__ off,
        const int32_t* __restrict__ adj, const int64_t* __restrict__ blk, Op op, Fin fin) {
    __shared__ typename Op::T s_val[kTile];
    const int64_t r0 = blk[blockIdx.x], r1 = blk[blockIdx.x + 1];
    const int64_t s0 = off[r0];
    const int64_t nnz = off[r1] - s0;
    if (nnz > kTile) return;                          // long row: handled by chunks
    stage_tile(adj, s0, nnz, op, s_val);
    reduce_runs<Op>(off, r0, r1, s0, s_val, fin);
}

// Packed, source-sorted tiles (pack_tiles): entry = source << kPackShift | slot.  The
// gathered message goes back to its slot, so the row reduce is unchanged.
template <class Fin>
__global__ void __launch_bounds__(kBlock) gather_short_packed(const int64_t* __restrict__ off,
        const int32_t* __restrict__ padj, const int64_t* __restrict__ blk, const double* __restrict__ msg, Fin fin) {
    __shared__ double s_val[kTile];
    const int64_t r0 = blk[blockIdx.x], r1 = blk[blockIdx.x + 1];
    const int64_t s0 = off[r0];
    const int64_t nnz = off[r1] - s0;
    if (nnz > kTile) return;                          // long row: handled by chunks
    {
        int32_t v[kPer];
#pragma unroll
        for (int j = 0; j < kPer; ++j) {
            const int64_t k = threadIdx.x + static_cast<int64_t>(j) * kBlock;
            v[j] = k < nnz ? stream_idx(padj + s0 + k) : -1;
        }
        double val[kPer];
#pragma unroll
        for (int j = 0; j < kPer; ++j) val[j] = v[j] >= 0 ? msg[v[j] >> kPackShift] : 0.0;
#pragma unroll
        for (int j = 0; j < kPer; ++j)
            if (v[j] >= 0) s_val[v[j] & ((1 << kPackShift) - 1)] = val[j];
    }
    __syncthreads();
    reduce_runs<PrOp>(off, r0, r1, s0, s_val, fin);
}
// gather_short_packed with the row data prefetched.  A tile's chain of dependent memory
// trips is blk -> off -> indices -> messages -> (barrier) -> row offsets -> csum/edge_count
// -> stores; here every thread issues its first row's offsets, cold sum and edge count
// together with the index loads, so the reduce starts from registers instead of waiting one
// more memory latency after the barrier.  Thread-per-row tiles prefetch row r0 + tid;
// wave-per-row tiles (<= 64 rows) prefetch row r0 + wave + 4 * lane, handed to the row's
// wave by a shuffle.  Same sums in the same order as gather_short_packed: bitwise equal.
template <bool kSkip = false>
__global__ void __launch_bounds__(kBlock) gather_hot_pf(const int64_t* __restrict__ off,
        const int32_t* __restrict__ padj, const int64_t* __restrict__ bdesc, const double* __restrict__ msg,
        PrColdFinal fin, int32_t skip_below = 0) {
    __shared__ double s_val[kTile];
    // block bounds and first entries in one descriptor pair (RowBlocks::bdesc)
    const int64_t r0 = bdesc[2 * blockIdx.x], s0 = bdesc[2 * blockIdx.x + 1];
    const int64_t r1 = bdesc[2 * blockIdx.x + 2], nnz = bdesc[2 * blockIdx.x + 3] - s0;
    const bool tpr = r1 - r0 > 64;
    const int wave = threadIdx.x >> 6;
    const int64_t pr = tpr ? r0 + threadIdx.x : r0 + wave + 4 * lane();
    int64_t pb = 0, pe = 0;
    double pcs = 0.0, pec = 1.0;
    if (pr < r1) {
        pb = off[pr];
        pe = off[pr + 1];
        pcs = fin.csum[pr];
        pec = __builtin_nontemporal_load(fin.f.edge_count + pr);
    }
    if (nnz > kTile) return;                          // long row: handled by chunks
    {
        int32_t v[kPer];
#pragma unroll
        for (int j = 0; j < kPer; ++j) {
            const int64_t k = threadIdx.x + static_cast<int64_t>(j) * kBlock;
            v[j] = k < nnz ? stream_idx(padj + s0 + k) : -1;
        }
        double val[kPer];
        // kSkip (diagnostic, TGO_PR_SKIP_BELOW): sources below skip_below read as 0 without a
        // load — the time the top sources' gathers cost in this pass; results are wrong
#pragma unroll
        for (int j = 0; j < kPer; ++j)
            val[j] = v[j] >= 0 && (!kSkip || (v[j] >> kPackShift) >= skip_below) ? msg[v[j] >> kPackShift] : 0.0;
#pragma unroll
        for (int j = 0; j < kPer; ++j)
            if (v[j] >= 0) s_val[v[j] & ((1 << kPackShift) - 1)] = val[j];
    }
    __syncthreads();
    const PrFinal& f = fin.f;
    auto emit = [&](int64_t r, double sum, double cs, double ec) {
        const double p = (f.alpha * (sum + cs)) + f.base;   // PrColdFinal: f(r, sum + csum[r])
        if (f.pr) f.pr[r] = p;
        f.contrib_next[r] = p / ec;
    };
    if (tpr) {
        bool first = true;
        for (int64_t i = r0 + threadIdx.x; i < r1; i += kBlock) {
            int64_t b = pb, e = pe;
            double cs = pcs, ec = pec;
            if (!first) {
                b = off[i]; e = off[i + 1]; cs = fin.csum[i];
                ec = __builtin_nontemporal_load(f.edge_count + i);
            }
            first = false;
            double sum = 0.0;
            for (int64_t k = b - s0; k < e - s0; ++k) sum = sum + s_val[k];
            emit(i, sum, cs, ec);
        }
    } else {
        for (int t = 0; r0 + wave + 4 * t < r1; ++t) {
            const int64_t i = r0 + wave + 4 * t;
            const int64_t b = __shfl(pb, t, 64), e = __shfl(pe, t, 64);
            const double cs = __shfl(pcs, t, 64), ec = __shfl(pec, t, 64);
            double sum = 0.0;
            for (int64_t k = b - s0 + lane(); k < e - s0; k += 64) sum = sum + s_val[k];
            sum = wave_sum(sum);
            if (lane() == 0) emit(i, sum, cs, ec);
        }
    }
}

// gather_hot_pf with larger tiles: kT entries (kT / kThreads = 16 per thread) staged in kT * 8
// bytes of LDS, entries packed as uint32 source << kShift | slot.  A larger tile holds more
// entries of the same 128-byte lines, and a tile is source-sorted, so more lanes of one gather
// instruction share a line: at RMAT-24, 0.70 line requests per hot entry at 4096 entries,
// 0.60 at 8192 and 0.48 at 16384 (host count over the bench graph).  Same sums in the same
// order as the 4096 form's reduce for the same tile boundaries (fixed association).
template <int kT, int kThreads, int kShift>
__global__ void __launch_bounds__(kThreads) gather_hot_big(const int64_t* __restrict__ off,
        const uint32_t* __restrict__ padj, const int64_t* __restrict__ bdesc, const double* __restrict__ msg,
        PrColdFinal fin) {
    constexpr int kP = kT / kThreads;
    constexpr int kWaves = kThreads / 64;
    static_assert(kP * kThreads == kT && (1 << kShift) == kT, "tile shape");
    __shared__ double s_val[kT];
    const int64_t r0 = bdesc[2 * blockIdx.x], s0 = bdesc[2 * blockIdx.x + 1];
    const int64_t r1 = bdesc[2 * blockIdx.x + 2], nnz = bdesc[2 * blockIdx.x + 3] - s0;
    const bool tpr = r1 - r0 > 64;
    const int wave = threadIdx.x >> 6;
    const int64_t pr = tpr ? r0 + threadIdx.x : r0 + wave + kWaves * lane();
    int64_t pb = 0, pe = 0;
    double pcs = 0.0, pec = 1.0;
    if (pr < r1) {
        pb = off[pr];
        pe = off[pr + 1];
        pcs = fin.csum[pr];
        pec = __builtin_nontemporal_load(fin.f.edge_count + pr);
    }
    if (nnz > kT) return;                             // long row: handled by chunks
    {
        uint32_t v[kP];
#pragma unroll
        for (int j = 0; j < kP; ++j) {
            const int64_t k = threadIdx.x + static_cast<int64_t>(j) * kThreads;
            v[j] = k < nnz ? __builtin_nontemporal_load(padj + s0 + k) : 0u;
        }
        double val[kP];
#pragma unroll
        for (int j = 0; j < kP; ++j) {
            const int64_t k = threadIdx.x + static_cast<int64_t>(j) * kThreads;
            val[j] = k < nnz ? msg[v[j] >> kShift] : 0.0;
        }
#pragma unroll
        for (int j = 0; j < kP; ++j) {
            const int64_t k = threadIdx.x + static_cast<int64_t>(j) * kThreads;
            if (k < nnz) s_val[v[j] & (kT - 1)] = val[j];
        }
    }
    __syncthreads();
    const PrFinal& f = fin.f;
    auto emit = [&](int64_t r, double sum, double cs, double ec) {
        const double p = (f.alpha * (sum + cs)) + f.base;   // PrColdFinal: f(r, sum + csum[r])
        if (f.pr) f.pr[r] = p;
        f.contrib_next[r] = p / ec;
    };
    if (tpr) {
        bool first = true;
        for (int64_t i = r0 + threadIdx.x; i < r1; i += kThreads) {
            int64_t b = pb, e = pe;
            double cs = pcs, ec = pec;
            if (!first) {
                b = off[i]; e = off[i + 1]; cs = fin.csum[i];
                ec = __builtin_nontemporal_load(f.edge_count + i);
            }
            first = false;
            double sum = 0.0;
            for (int64_t k = b - s0; k < e - s0; ++k) sum = sum + s_val[k];
            emit(i, sum, cs, ec);
        }
    } else {
        for (int t = 0; r0 + wave + kWaves * t < r1; ++t) {
            const int64_t i = r0 + wave + kWaves * t;
            const int64_t b = __shfl(pb, t, 64), e = __shfl(pe, t, 64);
            const double cs = __shfl(pcs, t, 64), ec = __shfl(pec, t, 64);
            double sum = 0.0;
            for (int64_t k = b - s0 + lane(); k < e - s0; k += 64) sum = sum + s_val[k];
            sum = wave_sum(sum);
            if (lane() == 0) emit(i, sum, cs, ec);
        }
    }
}

// gather_hot_big as persistent workgroups (grid = CUs x workgroups per CU) that walk the
// tiles t = blockIdx.x, + gridDim.x, ... and software-pipeline them: tile t+1's gathers and
// tile t+2's index loads are in flight while tile t is reduced from LDS.  A large tile leaves
// one (16384) or two (8192) workgroups per CU, too few for the hardware to hide a tile's
// load -> gather -> barrier -> reduce chain by switching workgroups; here each workgroup
// overlaps it itself.  Issue order keeps the counted waits short: a tile's row data is
// loaded before the next tile's gathers, so the reduce waits only for loads older than them.
// Same sums in the same order as gather_hot_big (bitwise equal for the same tiles).
template <int kT, int kThreads, int kShift>
__global__ void __launch_bounds__(kThreads, 4) gather_hot_pipe(const int64_t* __restrict__ off,
        const uint32_t* __restrict__ padj, const int64_t* __restrict__ bdesc, int64_t nblocks,
        const double* __restrict__ msg, PrColdFinal fin) {
    constexpr int kP = kT / kThreads;
    constexpr int kWaves = kThreads / 64;
    static_assert(kP * kThreads == kT && (1 << kShift) == kT && kP % 2 == 0, "tile shape");
    __shared__ double s_val[kT + 1];                     // [kT]: the sink of lanes past the tile's entries
    const int wave = threadIdx.x >> 6;
    const PrFinal& f = fin.f;
    struct Desc { int64_t r0, s0, r1; int nnz; };
    auto desc = [&](int64_t t) {
        Desc d{0, 0, 0, 0};
        if (t < nblocks) {
            d.r0 = bdesc[2 * t]; d.s0 = bdesc[2 * t + 1];
            d.r1 = bdesc[2 * t + 2];
            const int64_t nnz = bdesc[2 * t + 3] - d.s0;
            d.nnz = nnz > kT ? -1 : static_cast<int>(nnz);   // -1: a long row, handled by chunks
        }
        return d;
    };
    typedef unsigned int v2u __attribute__((ext_vector_type(2)));
    uint32_t idx[kP];
    uint32_t slot2[kP / 2];                              // two 16-bit LDS slots per register
    double val[kP];
    // buffer loads: 32-bit per-lane offsets against wave-uniform descriptors, and their range
    // check instead of branches — a lane past the tile's entries reads index 0 (records end
    // at the tile) and gathers from an offset past the vector's records, i.e. reads 0.0
    // without touching memory; its value goes to the sink slot kT
    const __amdgpu_buffer_rsrc_t rmsg = __builtin_amdgcn_make_buffer_rsrc(const_cast<double*>(msg), (short)0,
                                                                          0x7FFFFFF0, 0x00020000);
    auto load_idx = [&](const Desc& d) {
        const __amdgpu_buffer_rsrc_t ri = __builtin_amdgcn_make_buffer_rsrc(
            const_cast<uint32_t*>(padj + d.s0), (short)0, d.nnz > 0 ? d.nnz * 4 : 0, 0x00020000);
#pragma unroll
        for (int j = 0; j < kP; ++j)
            idx[j] = __builtin_amdgcn_raw_buffer_load_b32(ri, (threadIdx.x + j * kThreads) * 4, 0, 2);  // aux 2: nt
    };
    auto gather = [&](const Desc& d) {
#pragma unroll
        for (int j = 0; j < kP; ++j) {
            const bool ok = static_cast<int>(threadIdx.x + j * kThreads) < d.nnz;
            const v2u x = __builtin_amdgcn_raw_buffer_load_b64(rmsg, ok ? (idx[j] >> kShift) * 8u : 0x7FFFFFF8u, 0, 0);
            val[j] = __longlong_as_double(static_cast<long long>((static_cast<unsigned long long>(x.y) << 32) | x.x));
        }
#pragma unroll
        for (int j = 0; j < kP; j += 2) {
            const int k = threadIdx.x + j * kThreads;
            const uint32_t a = k < d.nnz ? (idx[j] & (kT - 1)) : kT;
            const uint32_t b = k + kThreads < d.nnz ? (idx[j + 1] & (kT - 1)) : kT;
            slot2[j / 2] = a | (b << 16);
        }
    };
    int64_t t = blockIdx.x;
    Desc cur = desc(t), nxt = desc(t + gridDim.x);
    load_idx(cur);
    gather(cur);
    load_idx(nxt);
    for (; t < nblocks; t += gridDim.x) {
        const Desc nx2 = desc(t + 2 * static_cast<int64_t>(gridDim.x));
        // row data of this tile first (older than the next tile's loads)
        const bool tpr = cur.r1 - cur.r0 > 64;
        const int64_t pr = tpr ? cur.r0 + threadIdx.x : cur.r0 + wave + kWaves * lane();
        int64_t pb = 0, pe = 0;
        double pcs = 0.0, pec = 1.0;
        if (cur.nnz >= 0 && pr < cur.r1) {
            pb = off[pr];
            pe = off[pr + 1];
            pcs = fin.csum[pr];
            pec = __builtin_nontemporal_load(f.edge_count + pr);
        }
#pragma unroll
        for (int j = 0; j < kP; ++j) s_val[(slot2[j / 2] >> (16 * (j & 1))) & 0xFFFFu] = val[j];
        __syncthreads();
        gather(nxt);                                     // tile t+1 in flight during the reduce
        load_idx(nx2);                                   // tile t+2's indices behind it
        if (cur.nnz >= 0) {
            auto emit = [&](int64_t r, double sum, double cs, double ec) {
                const double p = (f.alpha * (sum + cs)) + f.base;
                if (f.pr) f.pr[r] = p;
                f.contrib_next[r] = p / ec;
            };
            const int64_t s0 = cur.s0;
            if (tpr) {
                bool first = true;
                for (int64_t i = cur.r0 + threadIdx.x; i < cur.r1; i += kThreads) {
                    int64_t b = pb, e = pe;
                    double cs = pcs, ec = pec;
                    if (!first) {
                        b = off[i]; e = off[i + 1]; cs = fin.csum[i];
                        ec = __builtin_nontemporal_load(f.edge_count + i);
                    }
                    first = false;
                    double sum = 0.0;
                    for (int k = static_cast<int>(b - s0); k < static_cast<int>(e - s0); ++k) sum = sum + s_val[k];
                    emit(i, sum, cs, ec);
                }
            } else {
                for (int q = 0; cur.r0 + wave + kWaves * q < cur.r1; ++q) {
                    const int64_t i = cur.r0 + wave + kWaves * q;
                    const int b = static_cast<int>(__shfl(pb, q, 64) - s0), e = static_cast<int>(__shfl(pe, q, 64) - s0);
                    const double cs = __shfl(pcs, q, 64), ec = __shfl(pec, q, 64);
                    double sum = 0.0;
                    for (int k = b + lane(); k < e; k += 64) sum = sum + s_val[k];
                    sum = wave_sum(sum);
                    if (lane() == 0) emit(i, sum, cs, ec);
                }
            }
        }
        __syncthreads();                                 // every read of s_val done before the next store
        cur = nxt;
        nxt = nx2;
    }
}

// ---------------------------------------------------------------- fixed-point hot pass
// The slot form above stages one double per entry in LDS so that every row can add its
// entries in a fixed order; LDS then caps a tile at 4096 - 16384 entries, and a tile's sorted
// sources share few 128-byte lines (0.70 L2 requests per hot entry at 4096 at RMAT-24, the
// request rate being the hot pass's bound — DESIGN.md §4.1).  Here a row's sum is an exact
// 128-bit fixed-point integer (binary point at bit kFxPoint: resolution 2^-80, range 2^47), so
// the entries of a tile may be added in ANY order and the result is still bit-for-bit the same:
// a tile needs one LDS accumulator per row, not one slot per entry, and grows to 64 K entries
// (super-tiles, pack_supertiles_device) — its source-sorted entries then share lines: 0.29 L2
// requests per hot entry at RMAT-24 (host count over the bench graph, 64 K entries / 4096 rows).
// The conversion of the exact sum back to a double rounds once (fx_to_double, nearest-even);
// the reference's fp64 sum (PageRankVertexProgram.java:84-89, VertexMemoryHandler.java:97-102)
// rounds once per entry.
//
// The form is exact only inside a range: a nonzero |v| below 2^-53 loses more than 2^-27 of
// itself to the 2^-80 resolution, and a row of D entries overflows the 2^47 range unless every
// |v| < 2^47 / D; the split LDS accumulators (below) narrow that to |v| < 2^23 / min(D, 2^22),
// and the entry conversion (fx_hl) to |v| < 2^11.
// Infinities and NaN — the +inf contribution of a vertex whose row cut left it no OUT entry
// (PageRankVertexProgram.java:80-88 divides by edgeCount 0) — have no fixed-point form at all.
// Every entry is checked against the layout's range (FxGuard: biased exponents [elo, ehi), from
// the longest row); one outside it sets *bad, and the caller re-runs the whole program on the
// plain fp64 gather, whose sums follow Java double arithmetic (+inf + x = +inf, +inf + -inf =
// NaN).  Inside the range the check costs two integer compares per entry.
//
// Split accumulators: an entry X = floor(v * 2^80) goes into LDS as two words, H = X >> 40
// (signed) and L = X & (2^40 - 1) (fx_hl), each by a NON-returning 64-bit LDS add — no carry to propagate, so a
// wave issues its kFxUnroll entries' adds back to back and never waits on LDS.  The L words of
// at most 2^22 entries (a tile's cap, kFxTileMax) sum below 2^62; X = H * 2^40 + L is rebuilt
// as 128 bits once per accumulator (fx_join).
constexpr int kFxPoint = 80;
constexpr int kFxLowBits = 40;
constexpr unsigned long long kFxLowMask = (1ull << kFxLowBits) - 1ull;
constexpr int kFxThreads = 1024;
constexpr int kFxSlots = 4096;         // LDS accumulators of a tile: rows x copies
// entries per thread per batch: the gathers in flight per wave.  6 with the one-launch head and
// ~1 tile a CU (RMAT-24 same box: 2 0.848, 4 0.786, 5 0.753, 6 0.750, 7 0.765, 8 0.786, 12 1.02,
// 16 1.20 ms/update — more requests in flight thrash the L2; profiles/r06xyz_pr_unroll_ab.log)
constexpr int kFxUnroll = 6;

// An entry's split words straight from the double: X = floor(v * 2^80) as H = floor(v * 2^40)
// and L = floor(frac(v * 2^40) * 2^40), every step exact in fp64 (scalings by powers of two,
// floor, and t - floor(t) are exact), the integers read off the bit patterns of h + 1.5 * 2^52
// and l + 2^52 (ulp 1 there).  Exact while |v| < 2^11 (|h| < 2^51): the FxGuard range keeps
// every entry below that; outside it the words are garbage that the guard's flag discards.
// Ten fp64 / integer operations an entry (the shift-and-select form before it took ~50).
__device__ __forceinline__ void fx_hl(double v, unsigned long long& H, unsigned long long& L) {
    const double t = v * 0x1p40;
    const double h = __builtin_floor(t);
    const double l = __builtin_floor((t - h) * 0x1p40);
    H = static_cast<unsigned long long>(__double_as_longlong(h + 0x1.8p52) - __double_as_longlong(0x1.8p52));
    L = static_cast<unsigned long long>(__double_as_longlong(l + 0x1p52) - __double_as_longlong(0x1p52));
}
// 128-bit X -> (H, L) = (X >> 40, X & (2^40 - 1)); exact for |X| < 2^103
__device__ __forceinline__ void fx_split(unsigned long long lo, unsigned long long hi, unsigned long long& H,
                                         unsigned long long& L) {
    H = (hi << (64 - kFxLowBits)) | (lo >> kFxLowBits);
    L = lo & kFxLowMask;
}
// H * 2^40 + L (H signed, 0 <= L < 2^63) as a 128-bit two's complement integer
__device__ __forceinline__ void fx_join(unsigned long long H, unsigned long long L, unsigned long long& lo,
                                        unsigned long long& hi) {
    const unsigned long long hl = H << kFxLowBits;
    lo = hl + L;
    hi = static_cast<unsigned long long>(static_cast<long long>(H) >> (64 - kFxLowBits)) + (lo < hl ? 1ull : 0ull);
}
// The 128-bit sum * 2^-80 rounded once to the nearest double (ties to even): the magnitude's
// top 64 bits with every lower bit OR-ed into bit 0 (a sticky bit far below the 53-bit rounding
// point: it breaks exact ties the dropped bits would have broken, and changes nothing else),
// converted once (u64 -> f64 is correctly rounded) and scaled by an exact power of two.
__device__ __forceinline__ double fx_to_double(unsigned long long lo, unsigned long long hi) {
    const bool neg = static_cast<long long>(hi) < 0;
    if (neg) {
        lo = ~lo + 1ull;
        hi = ~hi + (lo == 0 ? 1ull : 0ull);
    }
    unsigned long long t = lo;
    int e = -kFxPoint;
    if (hi) {
        const int s = 64 - __clzll(static_cast<long long>(hi));   // 1..64 significant bits in hi
        const unsigned long long below = s == 64 ? lo : lo << (64 - s);
        t = (s == 64 ? hi : (hi << (64 - s)) | (lo >> s)) | (below != 0 ? 1ull : 0ull);
        e += s;
    }
    const double d = __builtin_ldexp(static_cast<double>(t), e);
    return neg ? -d : d;
}
// 128-bit add into global memory (the long rows' chunk totals): few, one thread a tile
__device__ __forceinline__ void fx_add(unsigned long long* plo, unsigned long long* phi, unsigned long long lo,
                                       unsigned long long hi) {
    const unsigned long long old = atomicAdd(plo, lo);
    const unsigned long long c = hi + (old + lo < old ? 1ull : 0ull);
    if (c) atomicAdd(phi, c);
}

// The exact range of the layout (see kFxPoint): a nonzero entry whose biased exponent is outside
// [elo, ehi) — or an infinity / NaN (exponent 0x7FF >= ehi), or a subnormal (0 < elo) — sets *bad.
struct FxGuard {
    unsigned elo = 0, ehi = 0x800;
    unsigned* bad = nullptr;
};
// kFxUnroll * kFxThreads entries from entry b: all index loads, then all gathers, then the
// conversions and the split LDS adds, without a branch between them (a conditional load per
// entry made the compiler wait for every outstanding load before the next gather: one gather
// in flight per wave).  Index positions past ne are clamped to ne - 1 (a valid entry, re-read)
// and their values zeroed.  (Loading the next batch's indices before this batch's adds measured
// 11 % slower: profiles/r06l_pr_branchfree_ab.log.)
template <int diag, bool kGuard>
__device__ __forceinline__ void fx_idx(const uint32_t* __restrict__ p, int64_t b, int64_t ne, uint32_t (&w)[kFxUnroll]) {
#pragma unroll
    for (int j = 0; j < kFxUnroll; ++j)
        w[j] = __builtin_nontemporal_load(p + min(b + j * kFxThreads + static_cast<int64_t>(threadIdx.x), ne - 1));
}
template <int diag, bool kGuard>
__device__ __forceinline__ void fx_batch(const uint32_t* __restrict__ p, int64_t b, int64_t ne,
                                         const double* __restrict__ msg, int rbits, uint32_t rmask, int lc, uint32_t cl,
                                         unsigned long long* s_lo, unsigned long long* s_hi, const FxGuard& guard,
                                         bool& out, unsigned long long& sink) {
    uint32_t w[kFxUnroll];
    fx_idx<diag, kGuard>(p, b, ne, w);
    __builtin_amdgcn_sched_barrier(0);                   // every index load issued before the first wait
    double v[kFxUnroll];
#pragma unroll
    for (int j = 0; j < kFxUnroll; ++j)
        v[j] = diag == 2 ? static_cast<double>(w[j]) * 0x1p-40 : msg[w[j] >> rbits];
#pragma unroll
    for (int j = 0; j < kFxUnroll; ++j) {
        if (b + j * kFxThreads + threadIdx.x >= ne) v[j] = 0.0;
        const unsigned long long bits = static_cast<unsigned long long>(__double_as_longlong(v[j]));
        const unsigned e = static_cast<unsigned>(bits >> 52) & 0x7FFu;
        if (kGuard) out |= (bits << 1) != 0 && e - guard.elo >= guard.ehi - guard.elo;   // unsigned: below elo wraps
        unsigned long long H, L;
        fx_hl(v[j], H, L);
        if (diag == 1) {
            sink += H ^ L ^ (w[j] & rmask);
        } else {
            const uint32_t slot = ((w[j] & rmask) << lc) | cl;
            atomicAdd(&s_lo[slot], L);
            atomicAdd(&s_hi[slot], H);
        }
    }
}
// A tile's entries (packed source << rbits | accumulator) into the split LDS accumulators
// (s_lo: L words, s_hi: H words), kFxUnroll entries per thread in flight.  lc: log2 of the
// copies per accumulator (the lane picks the copy).
// diag (TGO_PR_FX_DIAG, results wrong by design; attribution only): 1 = no LDS atomics (the
// values are folded into one register), 2 = no gathers (the index word stands in for the value),
// 3 = the hot pass's emission without the cold fold and the update
template <int diag = 0, bool kGuard = false>
__device__ __forceinline__ void fx_accumulate(const uint32_t* __restrict__ p, int64_t ne, const double* __restrict__ msg,
                                              int rbits, int lc, unsigned long long* s_lo, unsigned long long* s_hi,
                                              const FxGuard& guard) {
    const uint32_t rmask = (1u << rbits) - 1u;
    const uint32_t cl = threadIdx.x & ((1u << lc) - 1u);
    constexpr int64_t kStep = static_cast<int64_t>(kFxThreads) * kFxUnroll;
    unsigned long long sink = 0;
    bool out = false;
    for (int64_t b = 0; b < ne; b += kStep)
        fx_batch<diag, kGuard>(p, b, ne, msg, rbits, rmask, lc, cl, s_lo, s_hi, guard, out, sink);
    if (diag == 1 && sink == 0x5a5a5a5a5a5a5a5aull) s_lo[0] = sink;      // keep the loads alive
    if (kGuard && out && guard.bad) *guard.bad = 1u;     // rare: the program re-runs in plain fp64
}
__device__ __forceinline__ int fx_copies_log2(int rows, int slots = kFxSlots) {
    int lc = 6;
    while (lc > 0 && (rows << lc) > slots) --lc;
    return lc;
}
// The 128-bit total of accumulator i's copies.
__device__ __forceinline__ void fx_total(const unsigned long long* s_lo, const unsigned long long* s_hi, int i, int lc,
                                         unsigned long long& lo, unsigned long long& hi) {
    unsigned long long H = 0, L = 0;
    for (int c = 0; c < (1 << lc); ++c) {
        H += s_hi[(i << lc) + c];
        L += s_lo[(i << lc) + c];
    }
    fx_join(H, L, lo, hi);
}

// The cold sum of row r at emission (TGO_PR_FX_FOLD): its pieces added in segment order, as
// cold_fold adds them — the same association, so the ranks are bitwise those of the separate
// fold — read here instead of from csum, so the fold kernel and csum's write + read go away.
struct FoldSrc {
    const uint32_t* cptr = nullptr;      // null: csum holds the cold sums (cold_fold ran)
    const int32_t* cpid = nullptr;
    const double* partial = nullptr;
    __device__ __forceinline__ double cold(int64_t r) const {
        double c = 0.0;
        const uint32_t e = cptr[r + 1];
        for (uint32_t k = cptr[r]; k < e; ++k) c += partial[cpid[k]];
        return c;
    }
};
__device__ __forceinline__ void fx_emit(const PrColdFinal& fin, const FoldSrc& fold, int64_t r, double hot) {
    if (fold.cptr) fin.f(r, hot + fold.cold(r));
    else fin(r, hot);
}
// One super-tile per workgroup: desc {first entry, end entry, first row, rows | -(long + 1)}.
// Each row has 2^lc copies of its accumulator (rows * copies <= kSlots), the copy chosen by
// the lane, so a tile of few rows does not serialise its lanes on one LDS address.
// kSlots = 8192 (rbits 13, TGO_PR_FX_HROWS): twice the rows per tile, so a row-limited tile (the
// low-degree tail) holds twice the entries and its gathers share more lines; 128 KB of dynamic
// LDS, one workgroup a CU.
// kPass (source split, TGO_PR_FX_SPLIT = S parts): 0 = the whole tile; otherwise launch p of S
// takes the tile's entries [bnd[t * (S + 1) + p], bnd[t * (S + 1) + p + 1]) (its sources in the
// p-th range) — 1 = the first (row totals to part), 3 = a middle one (from part, back to part),
// 2 = the last (from part, emitted).  The same exact sum in every split, so the ranks are
// bitwise those of kPass 0.
template <int kSlots, int diag, int kPass = 0, bool kGuard = false>
__global__ void __launch_bounds__(kFxThreads) gather_hot_fx(const uint32_t* __restrict__ padj,
        const int64_t* __restrict__ desc, int rbits, const double* __restrict__ msg, PrColdFinal fin,
        unsigned long long* __restrict__ long_acc, FoldSrc fold, FxGuard guard, const int64_t* __restrict__ bnd = nullptr,
        int nsplit = 1, int p = 0, unsigned long long* __restrict__ part = nullptr) {
    // 4096 slots: static LDS as before the 8192 option (the launch then passes no dynamic LDS)
    __shared__ unsigned long long s_static[kSlots == kFxSlots ? 2 * kFxSlots : 1];
    extern __shared__ unsigned long long fx_hot_lds[];
    unsigned long long* s_lo = kSlots == kFxSlots ? s_static : fx_hot_lds;
    unsigned long long* s_hi = s_lo + kSlots;
    const int64_t t = blockIdx.x;
    const int64_t r0 = desc[4 * t + 2], nr = desc[4 * t + 3];
    const int64_t e0 = kPass == 0 ? desc[4 * t] : bnd[t * (nsplit + 1) + p];
    const int64_t e1 = kPass == 0 ? desc[4 * t + 1] : bnd[t * (nsplit + 1) + p + 1];
    const int rows = nr > 0 ? static_cast<int>(nr) : 1;
    const int lc = fx_copies_log2(rows, kSlots);
    const int nslots = rows << lc;
    for (int i = threadIdx.x; i < nslots; i += kFxThreads) {
        const bool carry = (kPass == 2 || kPass == 3) && nr > 0 && (i & ((1 << lc) - 1)) == 0;   // copy 0: the sum so far
        unsigned long long H = 0, L = 0;
        if (carry) fx_split(part[2 * (r0 + (i >> lc))], part[2 * (r0 + (i >> lc)) + 1], H, L);
        s_lo[i] = L;
        s_hi[i] = H;
    }
    __syncthreads();
    fx_accumulate<diag, kGuard>(padj + e0, e1 - e0, msg, rbits, lc, s_lo, s_hi, guard);
    __syncthreads();
    if (nr > 0) {
        for (int i = threadIdx.x; i < rows; i += kFxThreads) {
            unsigned long long lo, hi;
            fx_total(s_lo, s_hi, i, lc, lo, hi);
            if (kPass == 1 || kPass == 3) {
                part[2 * (r0 + i)] = lo;
                part[2 * (r0 + i) + 1] = hi;
            } else if (diag == 3) {                       // attribution: no fold, no update
                fin.f.contrib_next[r0 + i] = fx_to_double(lo, hi);
            } else {
                fx_emit(fin, fold, r0 + i, fx_to_double(lo, hi));   // + the row's cold sum, then the update
            }
        }
    } else if (threadIdx.x == 0) {                        // a long row's chunk: into the row's accumulator
        unsigned long long H = 0, L = 0, lo, hi;
        for (int c = 0; c < nslots; ++c) {
            H += s_hi[c];
            L += s_lo[c];
        }
        fx_join(H, L, lo, hi);
        fx_add(&long_acc[2 * (-nr - 1)], &long_acc[2 * (-nr - 1) + 1], lo, hi);
    }
}
// Cold pass in fixed point: the cold_gather protocol (workgroup b on XCD b % 8 takes that XCD's
// (b / 8)-th block, so each XCD walks its segments in order with the segment's messages in its
// L2), but a block is a run of up to 4096 pieces and TGO_PR_FX_CE entries, packed
// (source - segment base) << 12 | piece - first piece, summed into per-piece accumulators in
// any order — a larger block shares more lines between the lanes of a gather (0.52 L2 requests
// per cold entry against 0.91 for the 4096-entry slot tiles, host count at RMAT-24).  Each
// piece's exact sum goes to partial[] as a double, where cold_fold adds a row's pieces in
// segment order as before.
// kSlots = 8192 (TGO_PR_FX_CP): 13-bit piece ids, 128 KB of dynamic LDS, one workgroup a CU.
template <int kSlots, int diag, bool kGuard = false>
__global__ void __launch_bounds__(kFxThreads) cold_fx(const uint32_t* __restrict__ cadj,
        const int64_t* __restrict__ cfd, XcdBase xb, const double* __restrict__ msg, double* __restrict__ partial,
        int shift, FxGuard guard) {
    extern __shared__ unsigned long long fx_lds[];
    unsigned long long* s_lo = fx_lds;
    unsigned long long* s_hi = fx_lds + kSlots;
    const int x = static_cast<int>(blockIdx.x & 7);
    const int64_t j = xb.b[x] + (blockIdx.x >> 3);
    if (j >= xb.b[x + 1]) return;
    const int64_t e0 = cfd[4 * j], e1 = cfd[4 * j + 1], p0 = cfd[4 * j + 2], w = cfd[4 * j + 3];
    const int np = static_cast<int>(w & 0xFFFF);
    const int lc = fx_copies_log2(np, kSlots);
    for (int i = threadIdx.x; i < (np << lc); i += kFxThreads) { s_lo[i] = 0; s_hi[i] = 0; }
    __syncthreads();
    fx_accumulate<diag, kGuard>(cadj + e0, e1 - e0, msg + (w >> 16), shift, lc, s_lo, s_hi, guard);
    __syncthreads();
    for (int i = threadIdx.x; i < np; i += kFxThreads) {
        unsigned long long lo, hi;
        fx_total(s_lo, s_hi, i, lc, lo, hi);
        partial[p0 + i] = fx_to_double(lo, hi);
    }
}

// The long rows after every chunk has landed: the update, and the accumulator back to zero.
__global__ void finalize_long_fx(const int32_t* __restrict__ long_row, int64_t nlong,
                                 unsigned long long* __restrict__ long_acc, PrColdFinal fin, FoldSrc fold) {
    for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < nlong; i += (int64_t)gridDim.x * blockDim.x) {
        const unsigned long long lo = long_acc[2 * i], hi = long_acc[2 * i + 1];
        long_acc[2 * i] = 0;
        long_acc[2 * i + 1] = 0;
        fx_emit(fin, fold, long_row[i], fx_to_double(lo, hi));
    }
}

// A long row's chunk of packed entries: the chunk sum (source order, fixed).
struct PackedOp {
    using T = double;
    const double* msg;
    int shift = kPackShift;
    __device__ __forceinline__ double load(int32_t v) const { return msg[static_cast<uint32_t>(v) >> shift]; }
    __device__ __forceinline__ static double add(double a, double b) { return a + b; }
    __device__ __forceinline__ static double zero() { return 0.0; }
};

template <class Op>
__global__ void __launch_bounds__(kBlock) gather_chunks(const int32_t* __restrict__ adj,
        const int64_t* __restrict__ cbeg, const int64_t* __restrict__ cend, Op op,
        typename Op::T* __restrict__ partial) {
    using T = typename Op::T;
    __shared__ T s_w[kBlock / 64];
    const int64_t b = cbeg[blockIdx.x], e = cend[blockIdx.x];
    T sum = Op::zero();
    for (int64_t t = b; t < e; t += kTile) {          // chunks are <= kTile: one trip
        T val[kPer];
        gather_tile(adj, t, min(e - t, kTile), op, val);
#pragma unroll
        for (int j = 0; j < kPer; ++j) sum = Op::add(sum, val[j]);
    }
    sum = wave_sum(sum);
    if (lane() == 0) s_w[threadIdx.x >> 6] = sum;
    __syncthreads();
    if (threadIdx.x == 0) {
        T t = Op::zero();
        for (int i = 0; i < kBlock / 64; ++i) t = Op::add(t, s_w[i]);
        partial[blockIdx.x] = t;
    }
}

template <class Op, class Fin>
__global__ void finalize_long(const int64_t* __restrict__ long_row, const int64_t* __restrict__ long_chunk,
                              int64_t nlong, const typename Op::T* __restrict__ partial, Fin fin) {
    using T = typename Op::T;
    for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < nlong; i += (int64_t)gridDim.x * blockDim.x) {
        T s = Op::zero();
        for (int64_t c = long_chunk[i]; c < long_chunk[i + 1]; ++c) s = Op::add(s, partial[c]);
        fin(long_row[i], s);
    }
}

// Cold pass of the cache-blocked PageRank gather.  Workgroup b runs on XCD b % 8 (the
// dispatcher deals workgroups round-robin over the 8 XCDs) and takes that XCD's (b / 8)-th
// cold block, so each XCD walks its own segments in order and its L2 holds the segment slice (384 K sources = 3 MB) of
// messages the block gathers from.  Workgroups past the XCD's block count exit at once.
template <bool kPacked, bool kPf = false>
__global__ void __launch_bounds__(kBlock) cold_gather(const int64_t* __restrict__ poff,
        const int32_t* __restrict__ cadj, const int64_t* __restrict__ bbeg, const int64_t* __restrict__ bend,
        const int32_t* __restrict__ xblk, const int32_t* __restrict__ bsrc, const int64_t* __restrict__ cdesc,
        XcdBase xb, const double* __restrict__ msg, double* __restrict__ partial) {
    __shared__ double s_val[kTile];
    const int x = static_cast<int>(blockIdx.x & 7);
    const int64_t j = xb.b[x] + (blockIdx.x >> 3);
    if (j >= xb.b[x + 1]) return;
    int64_t p0, p1, s0, nnz, src = 0;
    if (kPf) {                                         // one descriptor (ColdBlocks::cdesc)
        p0 = cdesc[4 * j]; p1 = cdesc[4 * j + 1]; s0 = cdesc[4 * j + 2];
        const int64_t w = cdesc[4 * j + 3];
        src = w >> 16;
        nnz = w & 0xFFFF;
    } else {
        const int64_t blk = xblk[j];
        p0 = bbeg[blk]; p1 = bend[blk];
        s0 = poff[p0];
        nnz = poff[p1] - s0;                           // <= kTile by construction
        if (kPacked) src = bsrc[blk];
    }
    // kPf: the first piece bounds of this thread (thread-per-piece) or of its wave's pieces
    // (wave-per-piece, one per lane) load with the indices, as in gather_hot_pf
    const bool tpr = p1 - p0 > 64;
    const int wave = threadIdx.x >> 6;
    int64_t pb = 0, pe = 0;
    if (kPf) {
        const int64_t pp = tpr ? p0 + threadIdx.x : p0 + wave + 4 * lane();
        if (pp < p1) { pb = poff[pp]; pe = poff[pp + 1]; }
    }
    if (kPacked) {                                     // source-sorted tile: values go back to their slot
        const double* seg_msg = msg + src;
        int32_t v[kPer];
#pragma unroll
        for (int q = 0; q < kPer; ++q) {
            const int64_t k = threadIdx.x + static_cast<int64_t>(q) * kBlock;
            v[q] = k < nnz ? stream_idx(cadj + s0 + k) : -1;
        }
        double val[kPer];
#pragma unroll
        for (int q = 0; q < kPer; ++q) val[q] = v[q] >= 0 ? seg_msg[v[q] >> kPackShift] : 0.0;
#pragma unroll
        for (int q = 0; q < kPer; ++q)
            if (v[q] >= 0) s_val[v[q] & ((1 << kPackShift) - 1)] = val[q];
        __syncthreads();
        if (kPf && tpr) {
            bool first = true;
            for (int64_t i = p0 + threadIdx.x; i < p1; i += kBlock) {
                int64_t b = pb, e = pe;
                if (!first) { b = poff[i]; e = poff[i + 1]; }
                first = false;
                double sum = 0.0;
                for (int64_t k = b - s0; k < e - s0; ++k) sum = sum + s_val[k];
                partial[i] = sum;
            }
        } else if (kPf) {
            for (int t = 0; p0 + wave + 4 * t < p1; ++t) {
                const int64_t i = p0 + wave + 4 * t;
                const int64_t b = __shfl(pb, t, 64), e = __shfl(pe, t, 64);
                double sum = 0.0;
                for (int64_t k = b - s0 + lane(); k < e - s0; k += 64) sum = sum + s_val[k];
                sum = wave_sum(sum);
                if (lane() == 0) partial[i] = sum;
            }
        } else {
            reduce_runs<PrOp>(poff, p0, p1, s0, s_val, [&](int64_t p, double sum) { partial[p] = sum; });
        }
    } else {
        stage_tile(cadj, s0, nnz, PrOp{msg}, s_val);
        reduce_runs<PrOp>(poff, p0, p1, s0, s_val, [&](int64_t p, double sum) { partial[p] = sum; });
    }
}

// LDS window pass of the cache-blocked PageRank gather.  The hottest `win` sources of the
// degree-grouped order (about 30 % of RMAT-24's entries for 15.9 K sources) are read from a copy
// of contrib[0, win) in LDS — no L2 request per entry, where the other passes pay one per
// distinct line (the update is bound by the L2 request rate: profiles/r04e_pmc/).  Persistent
// workgroups, one per CU (the window takes 124 KB of the CU's 160 KB LDS), load the window once
// per update and walk the CSR-adaptive tiles of the window CSR (2-byte source ids, row-major):
// a tile's entries are staged in LDS in row order with coalesced index loads, then reduced
// thread-per-row (many short rows) or wave-per-row (<= 64 rows, fixed shuffle tree); a row with
// more window entries than a tile (a hub) is summed by the whole workgroup, strided per thread
// and reduced in wave order.  Every row of [0, n_rows) gets its window sum in csum, which
// cold_fold then accumulates the cold pieces onto: a fixed association, bitwise reproducible.
constexpr int kWinThreads = 1024;                    // 16 independent waves per CU
constexpr int kWinWaveTile = 512;                    // entries per wave item (8 per lane); <= 64 rows

__device__ __forceinline__ void wave_sync() {          // a wave's LDS writes visible to its own later reads
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

// Every wave works alone on items t = global wave, + all waves, ...: an item is <= 64 rows with
// <= 512 window entries (build_row_blocks(tile 512, 64 rows)), or one longer row.  Loads are
// software-pipelined two deep so no wave waits on a chain of dependent loads: while item t is
// reduced from LDS, item t+1's indices and row bounds (its descriptor arrived one trip ago)
// and item t+2's descriptor are in flight.  No workgroup barrier after the window is loaded.
__global__ void __launch_bounds__(kWinThreads) lds_window(const int64_t* __restrict__ woff,
        const uint16_t* __restrict__ widx, const int64_t* __restrict__ bdesc, int64_t nitems, int32_t win,
        const double* __restrict__ msg, double* __restrict__ csum) {
    extern __shared__ double lds[];
    double* s_win = lds;
    const int wave = threadIdx.x >> 6;
    double* s_val = lds + win + wave * kWinWaveTile;
    for (int i = threadIdx.x; i < win; i += kWinThreads) s_win[i] = msg[i];
    __syncthreads();
    constexpr int kPerLane = kWinWaveTile / 64;
    const int64_t nwaves = static_cast<int64_t>(gridDim.x) * (kWinThreads / 64);
    struct Desc { int64_t r0, s0, r1, nnz; };
    struct Data { uint16_t v[kPerLane]; int64_t rb, re; };
    auto desc = [&](int64_t t) {
        Desc d{0, 0, 0, 0};
        if (t < nitems) {
            d.r0 = bdesc[2 * t]; d.s0 = bdesc[2 * t + 1];
            d.r1 = bdesc[2 * t + 2]; d.nnz = bdesc[2 * t + 3] - d.s0;
        }
        return d;
    };
    auto data = [&](const Desc& d) {
        Data x;
        x.rb = x.re = 0;
        const bool small = d.nnz <= kWinWaveTile;     // a long row streams its entries when processed
#pragma unroll
        for (int j = 0; j < kPerLane; ++j) {
            const int k = lane() + 64 * j;
            x.v[j] = small && k < d.nnz ? widx[d.s0 + k] : 0;
        }
        const int64_t i = d.r0 + lane();
        if (small && i < d.r1) { x.rb = woff[i]; x.re = woff[i + 1]; }
        return x;
    };
    int64_t t = blockIdx.x * static_cast<int64_t>(kWinThreads / 64) + wave;
    Desc dc = desc(t), dn = desc(t + nwaves);
    Data xc = data(dc);
    for (; t < nitems; t += nwaves) {
        const Desc dn2 = desc(t + 2 * nwaves);         // two items ahead: the descriptor
        const Data xn = data(dn);                      // one item ahead: indices and row bounds
        if (dc.nnz > kWinWaveTile) {                   // one long row: lanes stride its entries
            double acc = 0.0;
            for (int64_t k = lane(); k < dc.nnz; k += 64) acc = acc + s_win[widx[dc.s0 + k]];
            acc = wave_sum(acc);
            if (lane() == 0) csum[dc.r0] = acc;
        } else {
#pragma unroll
            for (int j = 0; j < kPerLane; ++j) {
                const int k = lane() + 64 * j;
                if (k < dc.nnz) s_val[k] = s_win[xc.v[j]];
            }
            wave_sync();
            const int64_t i = dc.r0 + lane();
            if (i < dc.r1) {
                double sum = 0.0;
                for (int64_t k = xc.rb - dc.s0; k < xc.re - dc.s0; ++k) sum = sum + s_val[k];
                csum[i] = sum;
            }
            wave_sync();                               // s_val is rewritten by the next item
        }
        dc = dn;
        dn = dn2;
        xc = xn;
    }
}

// Per-row cold sums of the rows that own pieces: the pieces added in segment order (onto the
// row's LDS window sum when the window pass ran: acc).
__global__ void cold_fold(const int32_t* __restrict__ crow, int64_t ncrows, const uint32_t* __restrict__ cptr,
                          const int32_t* __restrict__ cpid, const double* __restrict__ partial, double* __restrict__ csum,
                          bool acc) {
    for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < ncrows; i += (int64_t)gridDim.x * blockDim.x) {
        const int64_t r = crow[i];
        double s = acc ? csum[r] : 0.0;
        const uint32_t e = cptr[r + 1];
        for (uint32_t k = cptr[r]; k < e; ++k) s += partial[cpid[k]];
        csum[r] = s;
    }
}

__global__ void pr_init(const int64_t* __restrict__ out_off, double* edge_count, double* contrib,
                        double* pr, double inv_n, int64_t n) {
    for (int64_t v = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; v < n; v += (int64_t)gridDim.x * blockDim.x) {
        // iteration 1 (PageRankVertexProgram.java:78-83): edgeCount = sum of the inE
        // messages (1.0 from every out-neighbour), PR = 1/N, send PR/edgeCount on outE.
        const double ec = static_cast<double>(out_off[v + 1] - out_off[v]);
        edge_count[v] = ec;
        pr[v] = inv_n;
        contrib[v] = inv_n / ec;
    }
}
__global__ void fill_f64(double* p, double v, int64_t n) {
    for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) p[i] = v;
}

inline int grid_for(int64_t work) {
    int64_t g = (work + kBlock - 1) / kBlock;
    if (g < 1) g = 1;
    if (g > 2048) g = 2048;
    return static_cast<int>(g);
}

template <class Op, class Fin>
hipError_t run_gather(const DevCsr& c, const RowBlocks& rb, Op op, Fin fin,
                      typename Op::T* partial, hipStream_t s) {
    if (rb.nblocks > 0) {
        gather_short<Op, Fin><<<static_cast<unsigned>(rb.nblocks), kBlock, 0, s>>>(c.off, c.adj, rb.blk, op, fin);
    }
    if (rb.nchunks > 0) {
        gather_chunks<Op><<<static_cast<unsigned>(rb.nchunks), kBlock, 0, s>>>(c.adj, rb.chunk_beg, rb.chunk_end, op, partial);
        finalize_long<Op, Fin><<<grid_for(rb.nlong), kBlock, 0, s>>>(rb.long_row, rb.long_chunk, rb.nlong, partial, fin);
    }
    return hipGetLastError();
}

}  // namespace

hipError_t k_pr_init(const DevCsr& out, double* edge_count, double* contrib, double* pr,
                     double inv_n, int64_t n, hipStream_t s) {
    pr_init<<<grid_for(n), kBlock, 0, s>>>(out.off, edge_count, contrib, pr, inv_n, n);
    return hipGetLastError();
}
hipError_t k_fill_f64(double* p, double v, int64_t n, hipStream_t s) {
    fill_f64<<<grid_for(n), kBlock, 0, s>>>(p, v, n);
    return hipGetLastError();
}
hipError_t k_pr_iter(const DevCsr& in, const RowBlocks& rb, const double* contrib,
                     const double* edge_count, double* pr, double* contrib_next, double* partial,
                     double alpha, double base, int64_t n, const PrTuning& t, hipStream_t s) {
    (void)n;
    const PrFinal fin{edge_count, pr, contrib_next, alpha, base};
    if (t.diag_hi > t.diag_lo) return run_gather(in, rb, PrDiagOp{contrib, t.diag_lo, t.diag_hi}, fin, partial, s);
    return run_gather(in, rb, PrOp{contrib}, fin, partial, s);
}
static FxGuard fx_guard(const ColdBlocks& cb) {
    FxGuard g;
    g.elo = static_cast<unsigned>(cb.fx_elo);
    g.ehi = static_cast<unsigned>(cb.fx_ehi);
    g.bad = cb.fx_bad;
    return g;
}
// Cold phase: the cold segments' partial sums, folded per row into csum (reads only the cold
// sources [hot, n_src) of `contrib`).
static bool fx_fold_in_hot() {                       // TGO_PR_FX_FOLD (read per launch, A/B)
    const char* e = std::getenv("TGO_PR_FX_FOLD");
    return e ? std::atoi(e) != 0 : true;
}
static int fx_diag() {                                // read per launch: an A/B flips it between runs
    const char* e = std::getenv("TGO_PR_FX_DIAG");
    return e ? std::atoi(e) : 0;
}
static bool row_prefetch() {
    static const bool on = [] { const char* e = std::getenv("TGO_PR_PF"); return !e || std::atoi(e) != 0; }();
    return on;
}
// dynamic LDS past 64 KB, raised once per kernel instantiation
static hipError_t big_lds(const void* fn, size_t lds) {
    static std::mutex mu;                                // the ranks of an in-process partition launch from threads
    static std::vector<const void*> done;
    std::lock_guard<std::mutex> lk(mu);
    if (std::find(done.begin(), done.end(), fn) != done.end()) return hipSuccess;
    const hipError_t e = hipFuncSetAttribute(fn, hipFuncAttributeMaxDynamicSharedMemorySize, static_cast<int>(lds));
    if (e == hipSuccess) done.push_back(fn);
    return e;
}
hipError_t k_pr_cold_phase(const ColdBlocks& cb, const double* contrib, hipStream_t s, bool guard_entries) {
    // fixed-point cold pieces beside a slot hot pass (whose emission does not check the range):
    // every update checks its entries
    guard_entries = guard_entries || (cb.cfx && !cb.fx);
    const bool window = cb.win > 0 && cb.rb_win.nblocks > 0;
    if (window) {
        const size_t lds = static_cast<size_t>(cb.win + (kWinThreads / 64) * kWinWaveTile) * sizeof(double);
        static size_t lds_set = 0;                    // the >64 KB dynamic LDS limit, raised once
        if (lds > lds_set) {
            const hipError_t e = hipFuncSetAttribute(reinterpret_cast<const void*>(&lds_window),
                                                     hipFuncAttributeMaxDynamicSharedMemorySize, static_cast<int>(lds));
            if (e != hipSuccess) return e;
            lds_set = lds;
        }
        const unsigned g = static_cast<unsigned>(std::max<int64_t>(1, std::min<int64_t>(cb.rb_win.nblocks, cb.num_cus)));
        lds_window<<<g, kWinThreads, lds, s>>>(cb.woff, cb.widx, cb.rb_win.bdesc, cb.rb_win.nblocks,
                                                static_cast<int32_t>(cb.win), contrib, cb.csum);
    }
    if (cb.max_xcd_blocks > 0) {
        const unsigned g = static_cast<unsigned>(cb.max_xcd_blocks * 8);
        if (cb.cfx && cb.cfx_shift > kPackShift) {
            constexpr size_t lds = 2 * 8192 * sizeof(unsigned long long);
            auto k = guard_entries ? &cold_fx<8192, 0, true> : &cold_fx<8192, 0, false>;
            if (const hipError_t e = big_lds(reinterpret_cast<const void*>(k), lds)) return e;
            k<<<g, kFxThreads, lds, s>>>(reinterpret_cast<const uint32_t*>(cb.cadj), cb.cfx_desc, cb.xbase, contrib,
                                         cb.partial, cb.cfx_shift, fx_guard(cb));
        } else if (cb.cfx) {
            const size_t lds = 2 * kFxSlots * sizeof(unsigned long long);
            const uint32_t* cadj = reinterpret_cast<const uint32_t*>(cb.cadj);
            const int d = fx_diag();
            if (guard_entries)
                cold_fx<kFxSlots, 0, true><<<g, kFxThreads, lds, s>>>(cadj, cb.cfx_desc, cb.xbase, contrib, cb.partial,
                                                                      cb.cfx_shift, fx_guard(cb));
            else if (d == 1)
                cold_fx<kFxSlots, 1><<<g, kFxThreads, lds, s>>>(cadj, cb.cfx_desc, cb.xbase, contrib, cb.partial, cb.cfx_shift, fx_guard(cb));
            else if (d == 2)
                cold_fx<kFxSlots, 2><<<g, kFxThreads, lds, s>>>(cadj, cb.cfx_desc, cb.xbase, contrib, cb.partial, cb.cfx_shift, fx_guard(cb));
            else
                cold_fx<kFxSlots, 0><<<g, kFxThreads, lds, s>>>(cadj, cb.cfx_desc, cb.xbase, contrib, cb.partial, cb.cfx_shift, fx_guard(cb));
        }
        else if (cb.cpacked && row_prefetch())
            cold_gather<true, true><<<g, kBlock, 0, s>>>(cb.poff, cb.cadj, cb.bbeg, cb.bend, cb.xblk, cb.bsrc, cb.cdesc, cb.xbase,
                                                         contrib, cb.partial);
        else if (cb.cpacked)
            cold_gather<true, false><<<g, kBlock, 0, s>>>(cb.poff, cb.cadj, cb.bbeg, cb.bend, cb.xblk, cb.bsrc, cb.cdesc, cb.xbase,
                                                          contrib, cb.partial);
        else
            cold_gather<false><<<g, kBlock, 0, s>>>(cb.poff, cb.cadj, cb.bbeg, cb.bend, cb.xblk, cb.bsrc, cb.cdesc, cb.xbase,
                                                           contrib, cb.partial);
    }
    int64_t g = (cb.n_crows + kBlock - 1) / kBlock;
    g = std::max<int64_t>(1, std::min<int64_t>(g, 65536));
    if (!(cb.fx && fx_fold_in_hot() && !window))
        cold_fold<<<static_cast<unsigned>(g), kBlock, 0, s>>>(cb.crow, cb.n_crows, cb.cptr, cb.cpid, cb.partial, cb.csum,
                                                              window);
    return hipGetLastError();
}

// bnd[t * (S + 1) + p] = the first entry of tile t with source >= p * hot / S (entries sorted by source)
__global__ void fx_split_points(const uint32_t* __restrict__ padj, const int64_t* __restrict__ desc, int64_t ntiles,
                                int rbits, int64_t hot, int nsplit, int64_t first, int64_t* __restrict__ bnd) {
    for (int64_t t = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; t < ntiles; t += (int64_t)gridDim.x * blockDim.x) {
        const int64_t e0 = desc[4 * t], e1 = desc[4 * t + 1];
        bnd[t * (nsplit + 1)] = e0;
        bnd[t * (nsplit + 1) + nsplit] = e1;
        for (int p = 1; p < nsplit; ++p) {
            // the first boundary at `first` sources when given (the hubs hold most entries), the
            // rest of the range cut evenly
            const int64_t hs = first > 0 ? first + (hot - first) * (p - 1) / (nsplit - 1) : hot * p / nsplit;
            int64_t a = e0, b = e1;
            while (a < b) {
                const int64_t c = (a + b) >> 1;
                if (static_cast<int64_t>(padj[c] >> rbits) < hs) a = c + 1; else b = c;
            }
            bnd[t * (nsplit + 1) + p] = a;
        }
    }
}
hipError_t k_fx_split_points(const uint32_t* padj, const int64_t* desc, int64_t ntiles, int rbits, int64_t hot,
                             int nsplit, int64_t first, int64_t* bnd, hipStream_t s) {
    if (ntiles <= 0) return hipSuccess;
    fx_split_points<<<grid_for(ntiles), kBlock, 0, s>>>(padj, desc, ntiles, rbits, hot, nsplit, first, bnd);
    return hipGetLastError();
}

// Hot phase: every row's hot entries (sources [0, hot)) + its folded cold sum -> the update.
hipError_t k_pr_hot_phase(const ColdBlocks& cb, const double* contrib, const double* edge_count, double* pr,
                          double* contrib_next, double* partial_long, double alpha, double base, hipStream_t s,
                          bool guard_entries) {
    PrColdFinal fin{PrFinal{edge_count, pr, contrib_next, alpha, base}, cb.csum};
    if (cb.fx || cb.cfx) {                           // every emitted contribution against the range
        fin.f.bad = cb.fx_bad;
        fin.f.elo = static_cast<unsigned>(cb.fx_elo);
        fin.f.ehi = static_cast<unsigned>(cb.fx_ehi);
    }
    if (cb.fx) {
        FoldSrc fold;
        if (fx_fold_in_hot() && cb.win == 0) { fold.cptr = cb.cptr; fold.cpid = cb.cpid; fold.partial = cb.partial; }
        if (cb.fx_ntiles > 0) {
            const unsigned g = static_cast<unsigned>(cb.fx_ntiles);
            const uint32_t* padj = reinterpret_cast<const uint32_t*>(cb.hcsr.adj);
            const int d = fx_diag();
            const FxGuard gd = fx_guard(cb);
            if (cb.fx_rbits == 13) {
                const size_t lds = 2 * 8192 * sizeof(unsigned long long);
                auto k = guard_entries ? &gather_hot_fx<8192, 0, 0, true> : &gather_hot_fx<8192, 0, 0, false>;
                if (const hipError_t e = big_lds(reinterpret_cast<const void*>(k), lds)) return e;
                k<<<g, kFxThreads, lds, s>>>(padj, cb.fx_desc, cb.fx_rbits, contrib, fin, cb.fx_long_acc, fold, gd, nullptr, 1,
                                             0, nullptr);
            } else if (cb.fx_split > 1 && d == 0) {  // one launch per source range
                const int S = cb.fx_split;
                for (int p = 0; p < S; ++p) {
                    auto k = p == 0 ? (guard_entries ? &gather_hot_fx<kFxSlots, 0, 1, true> : &gather_hot_fx<kFxSlots, 0, 1, false>)
                           : p + 1 < S ? (guard_entries ? &gather_hot_fx<kFxSlots, 0, 3, true> : &gather_hot_fx<kFxSlots, 0, 3, false>)
                                       : (guard_entries ? &gather_hot_fx<kFxSlots, 0, 2, true> : &gather_hot_fx<kFxSlots, 0, 2, false>);
                    k<<<g, kFxThreads, 0, s>>>(padj, cb.fx_desc, cb.fx_rbits, contrib, fin, cb.fx_long_acc, fold, gd, cb.fx_mid,
                                               S, p, cb.fx_part);
                }
            } else {
                const size_t lds = 0;
                if (guard_entries)
                    gather_hot_fx<kFxSlots, 0, 0, true><<<g, kFxThreads, lds, s>>>(padj, cb.fx_desc, cb.fx_rbits, contrib, fin,
                                                                                   cb.fx_long_acc, fold, gd);
                else if (d == 1)
                    gather_hot_fx<kFxSlots, 1><<<g, kFxThreads, lds, s>>>(padj, cb.fx_desc, cb.fx_rbits, contrib, fin,
                                                                          cb.fx_long_acc, fold, fx_guard(cb));
                else if (d == 2)
                    gather_hot_fx<kFxSlots, 2><<<g, kFxThreads, lds, s>>>(padj, cb.fx_desc, cb.fx_rbits, contrib, fin,
                                                                          cb.fx_long_acc, fold, fx_guard(cb));
                else if (d == 3)
                    gather_hot_fx<kFxSlots, 3><<<g, kFxThreads, lds, s>>>(padj, cb.fx_desc, cb.fx_rbits, contrib, fin,
                                                                          cb.fx_long_acc, fold, fx_guard(cb));
                else
                    gather_hot_fx<kFxSlots, 0><<<g, kFxThreads, lds, s>>>(padj, cb.fx_desc, cb.fx_rbits, contrib, fin,
                                                                          cb.fx_long_acc, fold, fx_guard(cb));
            }
        }
        if (cb.fx_nlong > 0)
            finalize_long_fx<<<grid_for(cb.fx_nlong), kBlock, 0, s>>>(cb.fx_long_row, cb.fx_nlong, cb.fx_long_acc, fin,
                                                                      fold);
        return hipGetLastError();
    }
    if (!cb.packed) return run_gather(cb.hcsr, cb.rb_hot, PrOp{contrib}, fin, partial_long, s);
    const RowBlocks& rb = cb.rb_hot;
    if (rb.nblocks > 0 && cb.hot_pipe) {
        const uint32_t* padj = reinterpret_cast<const uint32_t*>(cb.hcsr.adj);
        const int per_cu = cb.hot_tile == 16384 ? 1 : cb.hot_tile == 8192 ? 2 : 4;
        const unsigned g = static_cast<unsigned>(std::min<int64_t>(rb.nblocks, int64_t(cb.num_cus) * per_cu));
        if (cb.hot_tile == 16384)
            gather_hot_pipe<16384, 1024, 14><<<g, 1024, 0, s>>>(cb.hcsr.off, padj, rb.bdesc, rb.nblocks, contrib, fin);
        else if (cb.hot_tile == 8192)
            gather_hot_pipe<8192, 512, 13><<<g, 512, 0, s>>>(cb.hcsr.off, padj, rb.bdesc, rb.nblocks, contrib, fin);
        else
            gather_hot_pipe<4096, 256, 12><<<g, 256, 0, s>>>(cb.hcsr.off, padj, rb.bdesc, rb.nblocks, contrib, fin);
    } else if (rb.nblocks > 0 && cb.hot_tile != kTile) {
        const unsigned g = static_cast<unsigned>(rb.nblocks);
        const uint32_t* padj = reinterpret_cast<const uint32_t*>(cb.hcsr.adj);
        if (cb.hot_tile == 8192)
            gather_hot_big<8192, 512, 13><<<g, 512, 0, s>>>(cb.hcsr.off, padj, rb.bdesc, contrib, fin);
        else
            gather_hot_big<16384, 1024, 14><<<g, 1024, 0, s>>>(cb.hcsr.off, padj, rb.bdesc, contrib, fin);
    } else if (rb.nblocks > 0) {
        static const int32_t skip_below = static_cast<int32_t>(std::atol(std::getenv("TGO_PR_SKIP_BELOW") ? std::getenv("TGO_PR_SKIP_BELOW") : "0"));
        if (skip_below > 0)
            gather_hot_pf<true><<<static_cast<unsigned>(rb.nblocks), kBlock, 0, s>>>(cb.hcsr.off, cb.hcsr.adj, rb.bdesc,
                                                                                      contrib, fin, skip_below);
        else if (row_prefetch())
            gather_hot_pf<<<static_cast<unsigned>(rb.nblocks), kBlock, 0, s>>>(cb.hcsr.off, cb.hcsr.adj, rb.bdesc,
                                                                                    contrib, fin);
        else
            gather_short_packed<PrColdFinal><<<static_cast<unsigned>(rb.nblocks), kBlock, 0, s>>>(cb.hcsr.off, cb.hcsr.adj,
                                                                                             rb.blk, contrib, fin);
    }
    if (rb.nchunks > 0) {
        gather_chunks<PackedOp><<<static_cast<unsigned>(rb.nchunks), kBlock, 0, s>>>(cb.hcsr.adj, rb.chunk_beg,
                                                                                    rb.chunk_end,
                                                                                    PackedOp{contrib, cb.hot_shift},
                                                                                    partial_long);
        finalize_long<PackedOp, PrColdFinal><<<grid_for(rb.nlong), kBlock, 0, s>>>(rb.long_row, rb.long_chunk,
                                                                                       rb.nlong, partial_long, fin);
    }
    return hipGetLastError();
}

hipError_t k_walk_iter(const DevCsr& out, const RowBlocks& rb, const int32_t* prev, int32_t* next,
                       int32_t* partial, int64_t n, hipStream_t s) {
    (void)n;
    WalkOp op{prev};
    WalkFinal fin{next};
    return run_gather(out, rb, op, fin, reinterpret_cast<uint32_t*>(partial), s);
}

}  // namespace tgo

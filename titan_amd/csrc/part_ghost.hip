// part_ghost.hip — the ghost (halo) exchange of partitioned PageRank.
//
// A rank's rows gather over in-lists whose sources live on every rank
// (PageRankVertexProgram.java:84-89: PR'(v) = a * sum_{u in IN(v)} c(u) + (1 - a) / N).  The
// plain exchange all-gathers every rank's contributions (8 bytes per active vertex per rank,
// per update); but a rank reads only the sources its own lists hold — on RMAT at 8 ranks about
// a third of the remote active vertices.  The ghost exchange sends exactly those:
//   load time  : every rank sorts + uniques the remote sources of its in-lists ("needs", one
//                sorted run per owner), tells each owner how many it needs (all-to-all of
//                counts) and which (all-to-allv of the ids); each owner keeps the ids it must
//                send (local rows), each receiver the gathered-vector position of each need;
//   per update : pack (send[k] = contrib_local[send_row[k]]), all-to-allv of the doubles,
//                unpack (gathered[pos[k]] = recv[k]) and the rank's own slice copied in;
// then the unchanged local step reads the gathered vector.  Only the values the kernels
// read are refreshed, so the results equal the all-gather's bit for bit.
#include <algorithm>
#include <cstdint>
#include <cstring>
#include <string>
#include <vector>

#include <hip/hip_runtime.h>
#include <rocprim/rocprim.hpp>

#include "engine.hpp"

namespace tgo {
namespace {

constexpr int kB = 256;
inline unsigned grid(int64_t work) {
    return static_cast<unsigned>(std::max<int64_t>(1, std::min<int64_t>((work + kB - 1) / kB, 65536)));
}

// remote sources only (owner != rank); own sources are copied, not exchanged
__global__ void remote_flags(const int32_t* __restrict__ adj, int64_t m, int64_t lo, int64_t hi, uint32_t* __restrict__ f) {
    for (int64_t k = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; k < m; k += (int64_t)gridDim.x * blockDim.x)
        f[k] = (adj[k] < lo || adj[k] >= hi) ? 1u : 0u;
}
__global__ void compact_i32(const int32_t* __restrict__ in, const uint32_t* __restrict__ f, const uint64_t* __restrict__ pos,
                            int64_t m, int32_t* __restrict__ out) {
    for (int64_t k = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; k < m; k += (int64_t)gridDim.x * blockDim.x)
        if (f[k]) out[pos[k]] = in[k];
}
// first position of owner q's run in the sorted unique needs: lower bound of q * nl
__global__ void owner_bounds(const int32_t* __restrict__ u, int64_t m, int64_t nl, int world, int64_t* __restrict__ b) {
    const int q = static_cast<int>(blockIdx.x * blockDim.x + threadIdx.x);
    if (q > world) return;
    const int64_t t = static_cast<int64_t>(q) * nl;
    int64_t lo = 0, hi = m;
    while (lo < hi) {
        const int64_t mid = (lo + hi) >> 1;
        if (static_cast<int64_t>(u[mid]) < t) lo = mid + 1; else hi = mid;
    }
    b[q] = lo;
}
// gathered-vector position of global source u: rank-major hot slices, then cold slices
// (tgo_part_pr_blocked); hot = 0 is the plain rank-major layout (position = u)
__global__ void gathered_pos(const int32_t* __restrict__ u, int64_t m, int64_t nl, int64_t A, int64_t H, int64_t W,
                             int32_t* __restrict__ pos) {
    for (int64_t k = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; k < m; k += (int64_t)gridDim.x * blockDim.x) {
        const int64_t x = u[k], r = x / nl, o = x % nl;
        pos[k] = static_cast<int32_t>(H == 0 ? x : (o < H ? r * H + o : W * H + r * (A - H) + (o - H)));
    }
}
__global__ void sub_i32(int32_t* __restrict__ v, int64_t m, int32_t by) {
    for (int64_t k = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; k < m; k += (int64_t)gridDim.x * blockDim.x) v[k] -= by;
}
__global__ void pack_f64(const double* __restrict__ src, const int32_t* __restrict__ row, int64_t m, double* __restrict__ out) {
    for (int64_t k = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; k < m; k += (int64_t)gridDim.x * blockDim.x)
        out[k] = src[row[k]];
}
__global__ void unpack_f64(const double* __restrict__ in, const int32_t* __restrict__ pos, int64_t m, double* __restrict__ g) {
    for (int64_t k = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; k < m; k += (int64_t)gridDim.x * blockDim.x)
        g[pos[k]] = in[k];
}

}  // namespace

// Sorted unique remote neighbours of one or two lists (global internal ids), grouped by owner:
// need (device, owned by the caller via hipFree), need_count[q] per owner q (host).
int ghost_needs(const int32_t* d_adj, int64_t nnz, const int32_t* d_adj2, int64_t nnz2, int64_t nl, int rank, int world,
                int32_t** need, std::vector<int64_t>& need_count, hipStream_t s, std::string& err) {
    *need = nullptr;
    need_count.assign(world, 0);
    const int64_t lo = static_cast<int64_t>(rank) * nl, hi = lo + nl;
    uint32_t* f = nullptr;
    uint64_t* pos = nullptr;
    int32_t *rem = nullptr, *srt = nullptr, *uq = nullptr;
    int64_t *nuniq = nullptr, *bounds = nullptr;
    void* tmp = nullptr;
    size_t tmp_bytes = 0;
    auto cleanup = [&]() {
        for (void* p : {static_cast<void*>(f), static_cast<void*>(pos), static_cast<void*>(rem), static_cast<void*>(srt),
                        static_cast<void*>(nuniq), static_cast<void*>(bounds), tmp})
            if (p) (void)hipFree(p);
    };
    auto fail = [&](hipError_t e) {
        err = std::string("ghost lists: ") + hipGetErrorString(e);
        cleanup();
        if (uq) (void)hipFree(uq);
        return TGO_E_HIP;
    };
    auto need_tmp = [&](size_t b) -> hipError_t {
        if (b <= tmp_bytes) return hipSuccess;
        if (tmp) (void)hipFree(tmp);
        tmp = nullptr;
        tmp_bytes = b;
        return hipMalloc(&tmp, b);
    };
    hipError_t e;
    const size_t m1 = static_cast<size_t>(std::max<int64_t>(std::max(nnz, nnz2), 1));
    if ((e = hipMalloc(&f, m1 * 4)) || (e = hipMalloc(&pos, (m1 + 1) * 8)) || (e = hipMalloc(&nuniq, 8)) ||
        (e = hipMalloc(&bounds, (world + 1) * 8)))
        return fail(e);
    // remote entries of each list, counted then compacted into rem (list 1, then list 2)
    auto count_remote = [&](const int32_t* adj, int64_t m, int64_t& c) -> hipError_t {
        c = 0;
        if (m <= 0) return hipSuccess;
        remote_flags<<<grid(m), kB, 0, s>>>(adj, m, lo, hi, f);
        size_t b = 0;
        hipError_t x;
        if ((x = rocprim::exclusive_scan(nullptr, b, f, pos, uint64_t(0), static_cast<size_t>(m), rocprim::plus<uint64_t>(), s)) ||
            (x = need_tmp(b)) ||
            (x = rocprim::exclusive_scan(tmp, b, f, pos, uint64_t(0), static_cast<size_t>(m), rocprim::plus<uint64_t>(), s)))
            return x;
        uint64_t last = 0;
        uint32_t lastf = 0;
        if ((x = hipMemcpyAsync(&last, pos + m - 1, 8, hipMemcpyDeviceToHost, s)) ||
            (x = hipMemcpyAsync(&lastf, f + m - 1, 4, hipMemcpyDeviceToHost, s)) || (x = hipStreamSynchronize(s)))
            return x;
        c = static_cast<int64_t>(last + lastf);
        return hipSuccess;
    };
    int64_t c1n = 0, c2n = 0;
    if ((e = count_remote(d_adj, nnz, c1n))) return fail(e);
    if ((e = count_remote(d_adj2, nnz2, c2n))) return fail(e);
    const int64_t c = c1n + c2n;
    const size_t c1 = static_cast<size_t>(std::max<int64_t>(c, 1));
    if ((e = hipMalloc(&rem, c1 * 4)) || (e = hipMalloc(&srt, c1 * 4)) || (e = hipMalloc(&uq, c1 * 4))) return fail(e);
    int64_t u = 0;
    if (c > 0) {
        // the flags / positions of list 2 are still in f / pos: compact it first, behind list 1's
        if (c2n > 0) compact_i32<<<grid(nnz2), kB, 0, s>>>(d_adj2, f, pos, nnz2, rem + c1n);
        if (c1n > 0) {
            int64_t again = 0;
            if ((e = count_remote(d_adj, nnz, again))) return fail(e);
            compact_i32<<<grid(nnz), kB, 0, s>>>(d_adj, f, pos, nnz, rem);
        }
        int bits = 1;
        while ((int64_t(1) << bits) < static_cast<int64_t>(world) * nl) ++bits;
        size_t b = 0;
        if ((e = rocprim::radix_sort_keys(nullptr, b, rem, srt, static_cast<size_t>(c), 0, bits, s)) || (e = need_tmp(b)) ||
            (e = rocprim::radix_sort_keys(tmp, b, rem, srt, static_cast<size_t>(c), 0, bits, s)))
            return fail(e);
        b = 0;
        if ((e = rocprim::unique(nullptr, b, srt, uq, nuniq, static_cast<size_t>(c), rocprim::equal_to<int32_t>(), s)) ||
            (e = need_tmp(b)) ||
            (e = rocprim::unique(tmp, b, srt, uq, nuniq, static_cast<size_t>(c), rocprim::equal_to<int32_t>(), s)) ||
            (e = hipMemcpyAsync(&u, nuniq, 8, hipMemcpyDeviceToHost, s)) || (e = hipStreamSynchronize(s)))
            return fail(e);
    }
    owner_bounds<<<1, 128, 0, s>>>(uq, u, nl, world, bounds);
    std::vector<int64_t> hb(world + 1);
    if ((e = hipMemcpyAsync(hb.data(), bounds, (world + 1) * 8, hipMemcpyDeviceToHost, s)) || (e = hipStreamSynchronize(s)))
        return fail(e);
    for (int q = 0; q < world; ++q) need_count[q] = hb[q + 1] - hb[q];
    cleanup();
    *need = uq;
    return TGO_OK;
}

hipError_t k_gathered_pos(const int32_t* u, int64_t m, int64_t nl, int64_t A, int64_t H, int64_t W, int32_t* pos,
                          hipStream_t s) {
    if (m > 0) gathered_pos<<<grid(m), kB, 0, s>>>(u, m, nl, A, H, W, pos);
    return hipGetLastError();
}
hipError_t k_sub_i32(int32_t* v, int64_t m, int32_t by, hipStream_t s) {
    if (m > 0) sub_i32<<<grid(m), kB, 0, s>>>(v, m, by);
    return hipGetLastError();
}
hipError_t k_pack_f64(const double* src, const int32_t* row, int64_t m, double* out, hipStream_t s) {
    if (m > 0) pack_f64<<<grid(m), kB, 0, s>>>(src, row, m, out);
    return hipGetLastError();
}
// 8-byte words moved as integers (multi-source frontier masks; doubles use the same kernels
// through their bits)
hipError_t k_pack_u64(const uint64_t* src, const int32_t* row, int64_t m, uint64_t* out, hipStream_t s) {
    return k_pack_f64(reinterpret_cast<const double*>(src), row, m, reinterpret_cast<double*>(out), s);
}
hipError_t k_unpack_u64(const uint64_t* in, const int32_t* pos, int64_t m, uint64_t* g, hipStream_t s) {
    return k_unpack_f64(reinterpret_cast<const double*>(in), pos, m, reinterpret_cast<double*>(g), s);
}
hipError_t k_unpack_f64(const double* in, const int32_t* pos, int64_t m, double* g, hipStream_t s) {
    if (m > 0) unpack_f64<<<grid(m), kB, 0, s>>>(in, pos, m, g);
    return hipGetLastError();
}

}  // namespace tgo

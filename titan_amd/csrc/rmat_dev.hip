// rmat_dev.hip — the RMAT stream of tgo_rmat_edges (synth.cpp) generated on the device.
//
// The stream is counter-based (edge e's quadrant choices come from splitmix64(seed + e * P +
// level)), so every edge is independent: one thread per edge, the same integer arithmetic as
// the host loop, then the same seeded relabel (the permutation is built on the host — the
// Fisher-Yates shuffle is sequential — and uploaded once).  Used by the full-size tests and
// the bench, where RMAT-27 (2^31 edges) takes ~25 s on 16 host threads.  Output: host arrays,
// written chunk by chunk from device buffers.
#include <algorithm>
#include <cstring>
#include <vector>
#include <hip/hip_runtime.h>
#include <rocprim/rocprim.hpp>
#include "../../include/tgo_synth.h"
#include "../../include/titan_gpu_olap.h"

namespace tgo {
std::vector<int32_t> rmat_relabel(int64_t n, uint64_t seed);
}

namespace {

__device__ __forceinline__ uint64_t splitmix64_d(uint64_t x) {
    x += 0x9E3779B97F4A7C15ULL;
    x = (x ^ (x >> 30)) * 0xBF58476D1CE4E5B9ULL;
    x = (x ^ (x >> 27)) * 0x94D049BB133111EBULL;
    return x ^ (x >> 31);
}

__global__ void rmat_chunk(int32_t scale, uint64_t seed, int64_t e0, int64_t count, const int32_t* __restrict__ perm,
                           int32_t* __restrict__ src, int32_t* __restrict__ dst, int32_t* __restrict__ weight) {
    // quadrant thresholds as in synth.cpp (16-bit fixed point: A=0.57, A+B=0.76, A+B+C=0.95)
    const uint32_t tA = static_cast<uint32_t>(0.57 * 65536.0);
    const uint32_t tB = static_cast<uint32_t>(0.76 * 65536.0);
    const uint32_t tC = static_cast<uint32_t>(0.95 * 65536.0);
    for (int64_t k = blockIdx.x * static_cast<int64_t>(blockDim.x) + threadIdx.x; k < count;
         k += static_cast<int64_t>(gridDim.x) * blockDim.x) {
        const uint64_t e = static_cast<uint64_t>(e0 + k);
        uint64_t u = 0, v = 0, r = 0;
        for (int lvl = 0; lvl < scale; ++lvl) {
            if ((lvl & 3) == 0) r = splitmix64_d(seed + e * 0x100000001B3ULL + static_cast<uint64_t>(lvl));
            const uint32_t x = static_cast<uint32_t>(r & 0xFFFF);
            r >>= 16;
            u = (u << 1) | (x >= tB ? 1u : 0u);
            v = (v << 1) | (((x >= tA && x < tB) || x >= tC) ? 1u : 0u);
        }
        src[k] = perm[u];
        dst[k] = perm[v];
        if (weight) weight[k] = 1 + static_cast<int32_t>(splitmix64_d(seed ^ e) % 255u);
    }
}

__global__ void touch_flags(const int32_t* __restrict__ src, const int32_t* __restrict__ dst, int64_t count, int64_t lo,
                            int64_t hi, uint8_t* __restrict__ flag) {
    for (int64_t k = blockIdx.x * static_cast<int64_t>(blockDim.x) + threadIdx.x; k < count;
         k += static_cast<int64_t>(gridDim.x) * blockDim.x)
        flag[k] = ((src[k] >= lo && src[k] < hi) || (dst[k] >= lo && dst[k] < hi)) ? 1 : 0;
}

}  // namespace

extern "C" int tgo_rmat_edges_device(int32_t scale, int32_t edge_factor, uint64_t seed, int64_t edge_begin,
                                     int64_t count, int32_t* src, int32_t* dst, int32_t* weight, int32_t device) {
    if (scale < 1 || scale > 30 || edge_factor < 1 || count < 0 || edge_begin < 0 || !src || !dst) return TGO_E_INVALID;
    int ndev = 0;
    if (hipGetDeviceCount(&ndev) != hipSuccess || device < 0 || device >= ndev) return TGO_E_HIP;
    if (hipSetDevice(device) != hipSuccess) return TGO_E_HIP;
    const int64_t n = int64_t(1) << scale;
    const std::vector<int32_t> perm = tgo::rmat_relabel(n, seed ^ 0x5EED5EEDULL);
    const int64_t chunk = std::min<int64_t>(std::max<int64_t>(count, 1), int64_t(1) << 26);
    int32_t *d_perm = nullptr, *d_buf = nullptr;
    hipStream_t st = nullptr;
    int rc = TGO_OK;
    if (hipStreamCreateWithFlags(&st, hipStreamNonBlocking) != hipSuccess) return TGO_E_HIP;
    if (hipMalloc(&d_perm, n * 4) != hipSuccess || hipMalloc(&d_buf, chunk * 4 * (weight ? 3 : 2)) != hipSuccess) {
        rc = TGO_E_OOM;
    } else if (hipMemcpyAsync(d_perm, perm.data(), n * 4, hipMemcpyHostToDevice, st) != hipSuccess) {
        rc = TGO_E_HIP;
    }
    for (int64_t c0 = 0; rc == TGO_OK && c0 < count; c0 += chunk) {
        const int64_t c = std::min(chunk, count - c0);
        int32_t* ds = d_buf;
        int32_t* dd = d_buf + chunk;
        int32_t* dw = weight ? d_buf + 2 * chunk : nullptr;
        const unsigned grid = static_cast<unsigned>(std::min<int64_t>((c + 255) / 256, 8192));
        rmat_chunk<<<grid, 256, 0, st>>>(scale, seed, edge_begin + c0, c, d_perm, ds, dd, dw);
        if (hipGetLastError() != hipSuccess ||
            hipMemcpyAsync(src + c0, ds, c * 4, hipMemcpyDeviceToHost, st) != hipSuccess ||
            hipMemcpyAsync(dst + c0, dd, c * 4, hipMemcpyDeviceToHost, st) != hipSuccess ||
            (weight && hipMemcpyAsync(weight + c0, dw, c * 4, hipMemcpyDeviceToHost, st) != hipSuccess) ||
            hipStreamSynchronize(st) != hipSuccess)
            rc = TGO_E_HIP;
    }
    if (rc == TGO_OK && hipStreamSynchronize(st) != hipSuccess) rc = TGO_E_HIP;
    if (d_perm) (void)hipFree(d_perm);
    if (d_buf) (void)hipFree(d_buf);
    (void)hipStreamDestroy(st);
    return rc;
}

// tgo_rmat_partition on the device: the stream's edges with an endpoint in [lo, hi), in stream
// order (a stable selection per chunk), written to the host arrays.
extern "C" int tgo_rmat_partition_device(int32_t scale, int32_t edge_factor, uint64_t seed, int64_t lo, int64_t hi,
                                         int32_t* src, int32_t* dst, int32_t* weight, int64_t capacity, int64_t* count,
                                         int32_t device) {
    if (scale < 1 || scale > 30 || edge_factor < 1 || !count || lo < 0 || hi <= lo) return TGO_E_INVALID;
    int ndev = 0;
    if (hipGetDeviceCount(&ndev) != hipSuccess || device < 0 || device >= ndev) return TGO_E_HIP;
    if (hipSetDevice(device) != hipSuccess) return TGO_E_HIP;
    const int64_t n = int64_t(1) << scale;
    const int64_t m = static_cast<int64_t>(edge_factor) << scale;
    const std::vector<int32_t> perm = tgo::rmat_relabel(n, seed ^ 0x5EED5EEDULL);
    const int64_t chunk = std::min<int64_t>(m, int64_t(1) << 26);
    const int nout = weight ? 3 : 2;
    int32_t *d_perm = nullptr, *d_gen = nullptr, *d_sel = nullptr;
    uint8_t* d_flag = nullptr;
    unsigned int* d_nsel = nullptr;
    void* tmp = nullptr;
    size_t tmp_bytes = 0;
    hipStream_t st = nullptr;
    int rc = TGO_OK;
    if (hipStreamCreateWithFlags(&st, hipStreamNonBlocking) != hipSuccess) return TGO_E_HIP;
    if (hipMalloc(&d_perm, n * 4) != hipSuccess || hipMalloc(&d_gen, chunk * 4 * nout) != hipSuccess ||
        hipMalloc(&d_sel, chunk * 4 * nout) != hipSuccess || hipMalloc(&d_flag, chunk) != hipSuccess ||
        hipMalloc(&d_nsel, sizeof(unsigned int) * 3) != hipSuccess) {
        rc = TGO_E_OOM;
    } else {
        for (int i = 0; i < nout && rc == TGO_OK; ++i) {
            size_t b = 0;
            if (rocprim::select(nullptr, b, d_gen, d_flag, d_sel, d_nsel, static_cast<size_t>(chunk), st) != hipSuccess)
                rc = TGO_E_HIP;
            tmp_bytes = std::max(tmp_bytes, b);
        }
        if (rc == TGO_OK && hipMalloc(&tmp, std::max<size_t>(tmp_bytes, 1)) != hipSuccess) rc = TGO_E_OOM;
        if (rc == TGO_OK && hipMemcpyAsync(d_perm, perm.data(), n * 4, hipMemcpyHostToDevice, st) != hipSuccess) rc = TGO_E_HIP;
    }
    int64_t got = 0;
    bool overflow = false;
    for (int64_t e0 = 0; rc == TGO_OK && e0 < m; e0 += chunk) {
        const int64_t c = std::min(chunk, m - e0);
        const unsigned grid = static_cast<unsigned>(std::min<int64_t>((c + 255) / 256, 8192));
        rmat_chunk<<<grid, 256, 0, st>>>(scale, seed, e0, c, d_perm, d_gen, d_gen + chunk, weight ? d_gen + 2 * chunk : nullptr);
        touch_flags<<<grid, 256, 0, st>>>(d_gen, d_gen + chunk, c, lo, hi, d_flag);
        unsigned int ns[3] = {0, 0, 0};
        for (int i = 0; i < nout && rc == TGO_OK; ++i) {
            size_t b = tmp_bytes;
            if (rocprim::select(tmp, b, d_gen + i * chunk, d_flag, d_sel + i * chunk, d_nsel + i, static_cast<size_t>(c), st) !=
                hipSuccess)
                rc = TGO_E_HIP;
        }
        if (rc == TGO_OK && (hipMemcpyAsync(ns, d_nsel, sizeof(ns), hipMemcpyDeviceToHost, st) != hipSuccess ||
                             hipStreamSynchronize(st) != hipSuccess))
            rc = TGO_E_HIP;
        if (rc != TGO_OK) break;
        const int64_t k = ns[0];
        if (got + k <= capacity && src && dst) {
            if (hipMemcpyAsync(src + got, d_sel, k * 4, hipMemcpyDeviceToHost, st) != hipSuccess ||
                hipMemcpyAsync(dst + got, d_sel + chunk, k * 4, hipMemcpyDeviceToHost, st) != hipSuccess ||
                (weight && hipMemcpyAsync(weight + got, d_sel + 2 * chunk, k * 4, hipMemcpyDeviceToHost, st) != hipSuccess) ||
                hipStreamSynchronize(st) != hipSuccess)
                rc = TGO_E_HIP;
        } else {
            overflow = true;
        }
        got += k;
    }
    for (void* p : {static_cast<void*>(d_perm), static_cast<void*>(d_gen), static_cast<void*>(d_sel),
                    static_cast<void*>(d_flag), static_cast<void*>(d_nsel), tmp})
        if (p) (void)hipFree(p);
    (void)hipStreamDestroy(st);
    *count = got;
    if (rc != TGO_OK) return rc;
    return overflow ? TGO_E_INVALID : TGO_OK;
}

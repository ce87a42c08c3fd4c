// Dev probe (not part of the product): calibration of rocprofv3's FETCH_SIZE / WRITE_SIZE /
// TCC counters for the access shapes of the PageRank and BFS kernels, on known byte counts.
// One dispatch per case (kernel names carry the case), so a --pmc pass reads per-dispatch
// counters that can be divided by the known bytes:
//   stream16   : 1 GiB read with 16-B-per-lane loads           (known bytes = 1 GiB)
//   stream4nt  : 1 GiB read with 4-B non-temporal lane loads    (the index stream's shape)
//   write8     : 1 GiB written with 8-B lane stores             (contrib / level vectors)
//   gather_*   : 2^27 random 8-B gathers (16 in flight/thread) from a table of the given
//                size: 2 GiB (> Infinity Cache, HBM), 128 MiB (Infinity-Cache resident after
//                a warm pass), 1 MiB (L2 resident); index stream read non-temporally.
// build: hipcc --offload-arch=gfx950 -O3 -o gpurun_out/pmc_calib scripts/pmc_calib.hip
#include <hip/hip_runtime.h>
#include <cstdint>
#include <cstdio>

__global__ void stream16(const uint4* __restrict__ p, int64_t n, uint4* out) {
    uint32_t acc = 0;
    for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
        const uint4 v = p[i];
        acc ^= v.x ^ v.y ^ v.z ^ v.w;
    }
    if (acc == 0x9E3779B9u) out[0] = make_uint4(acc, 0, 0, 0);
}
__global__ void stream4nt(const uint32_t* __restrict__ p, int64_t n, uint32_t* out) {
    uint32_t acc = 0;
    for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x)
        acc ^= __builtin_nontemporal_load(p + i);
    if (acc == 0x9E3779B9u) out[0] = acc;
}
__global__ void write8(double* __restrict__ p, int64_t n) {
    for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x)
        p[i] = static_cast<double>(i);
}
template <int CASE>
__global__ void gather(const int32_t* __restrict__ idx, const double* __restrict__ tab, int64_t m, double* out) {
    const int64_t base = static_cast<int64_t>(blockIdx.x) * blockDim.x * 16 + threadIdx.x;
    int32_t ix[16];
#pragma unroll
    for (int j = 0; j < 16; ++j) {
        const int64_t k = base + static_cast<int64_t>(j) * blockDim.x;
        ix[j] = k < m ? __builtin_nontemporal_load(idx + k) : -1;
    }
    double s = 0;
#pragma unroll
    for (int j = 0; j < 16; ++j) s += ix[j] >= 0 ? tab[ix[j]] : 0.0;
    if (s == 12345.678) out[0] = s;
}
__global__ void mkidx(int32_t* idx, int64_t m, int64_t range, uint64_t seed) {
    for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < m; i += (int64_t)gridDim.x * blockDim.x) {
        uint64_t z = seed + 0x9E3779B97F4A7C15ULL * static_cast<uint64_t>(i + 1);
        z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ULL;
        z = (z ^ (z >> 27)) * 0x94D049BB133111EBULL;
        z ^= z >> 31;
        idx[i] = static_cast<int32_t>(z % static_cast<uint64_t>(range));
    }
}

int main() {
    const int64_t gib = int64_t(1) << 30;
    const int64_t m = int64_t(1) << 27;
    void *buf = nullptr, *tab = nullptr, *out = nullptr;
    int32_t* idx = nullptr;
    if (hipMalloc(&buf, gib) != hipSuccess || hipMalloc(&tab, 2 * gib) != hipSuccess ||
        hipMalloc(&idx, m * 4) != hipSuccess || hipMalloc(&out, 64) != hipSuccess) {
        std::printf("alloc failed\n");
        return 1;
    }
    (void)hipMemset(buf, 1, gib);
    (void)hipMemset(tab, 0, 2 * gib);
    hipEvent_t a, b;
    (void)hipEventCreate(&a);
    (void)hipEventCreate(&b);
    auto timed = [&](const char* name, double bytes, auto launch) {
        (void)hipDeviceSynchronize();
        (void)hipEventRecord(a);
        launch();
        (void)hipEventRecord(b);
        (void)hipEventSynchronize(b);
        float ms = 0;
        (void)hipEventElapsedTime(&ms, a, b);
        std::printf("case %-14s known_bytes %.0f ms %.4f GB/s %.1f\n", name, bytes, ms, bytes / ms / 1e6);
    };
    const int grid = 256 * 16;
    timed("stream16", double(gib), [&] { stream16<<<grid, 256>>>((const uint4*)buf, gib / 16, (uint4*)out); });
    timed("stream4nt", double(gib), [&] { stream4nt<<<grid, 256>>>((const uint32_t*)buf, gib / 4, (uint32_t*)out); });
    timed("write8", double(gib), [&] { write8<<<grid, 256>>>((double*)buf, gib / 8); });
    const unsigned gblocks = static_cast<unsigned>((m + 4095) / 4096);
    // HBM: 2 GiB table, uniform random (cold: the table exceeds the Infinity Cache)
    mkidx<<<4096, 256>>>(idx, m, (2 * gib) / 8, 7);
    timed("gather_hbm", double(m) * 8, [&] { gather<0><<<gblocks, 256>>>(idx, (const double*)tab, m, (double*)out); });
    // Infinity Cache: 128 MiB table, warmed by a first pass
    mkidx<<<4096, 256>>>(idx, m, (int64_t(128) << 20) / 8, 9);
    gather<1><<<gblocks, 256>>>(idx, (const double*)tab, m, (double*)out);
    timed("gather_mall", double(m) * 8, [&] { gather<2><<<gblocks, 256>>>(idx, (const double*)tab, m, (double*)out); });
    // L2: 1 MiB table
    mkidx<<<4096, 256>>>(idx, m, (int64_t(1) << 20) / 8, 11);
    gather<3><<<gblocks, 256>>>(idx, (const double*)tab, m, (double*)out);
    timed("gather_l2", double(m) * 8, [&] { gather<4><<<gblocks, 256>>>(idx, (const double*)tab, m, (double*)out); });
    std::printf("index stream per gather case: %.0f bytes (4 B x 2^27, non-temporal)\n", double(m) * 4);
    return 0;
}

// Dev probe (not part of the product): random 8-byte gather rate on MI355X from tables of
// different sizes (XCD-L2-resident, Infinity-Cache-resident, HBM), index stream read like
// the PageRank gather (int32 indices, 8 gathers in flight per thread).
// build: hipcc --offload-arch=gfx950 -O3 -o gpurun_out/gather_probe scripts/gather_probe.hip
#include <hip/hip_runtime.h>
#include <cstdint>
#include <cstdio>

__global__ void gather(const int32_t* __restrict__ idx, const double* __restrict__ tab, double* __restrict__ out,
                       int64_t m) {
    const int64_t base = static_cast<int64_t>(blockIdx.x) * blockDim.x * 8 + threadIdx.x;
    int32_t ix[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) {
        const int64_t k = base + static_cast<int64_t>(j) * blockDim.x;
        ix[j] = k < m ? __builtin_nontemporal_load(idx + k) : -1;
    }
    double s = 0;
#pragma unroll
    for (int j = 0; j < 8; ++j) s += ix[j] >= 0 ? tab[ix[j]] : 0.0;
    if (s == 12345.678) out[0] = s;   // keeps the loads alive
}

// uniform (skew = 0) or power-law-like (skew = 1: v = range^u - 1) indices
__global__ void mkidx(int32_t* idx, int64_t m, int64_t range, uint64_t seed, int skew) {
    for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < m; i += (int64_t)gridDim.x * blockDim.x) {
        uint64_t z = seed + 0x9E3779B97F4A7C15ULL * static_cast<uint64_t>(i + 1);
        z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ULL;
        z = (z ^ (z >> 27)) * 0x94D049BB133111EBULL;
        z ^= z >> 31;
        int64_t v;
        if (skew) {
            const double u = static_cast<double>(z >> 11) * (1.0 / 9007199254740992.0);
            v = static_cast<int64_t>(exp(u * log(static_cast<double>(range)))) - 1;
            if (v >= range) v = range - 1;
        } else {
            v = static_cast<int64_t>(z % static_cast<uint64_t>(range));
        }
        idx[i] = static_cast<int32_t>(v);
    }
}

int main() {
    const int64_t m = 268435456;
    int32_t* idx = nullptr;
    double* tab = nullptr;
    double* out = nullptr;
    if (hipMalloc(&idx, m * 4) != hipSuccess || hipMalloc(&tab, int64_t(1) << 31) != hipSuccess ||
        hipMalloc(&out, 64) != hipSuccess) {
        std::printf("alloc failed\n");
        return 1;
    }
    (void)hipMemset(tab, 0, int64_t(1) << 31);
    hipEvent_t a, b;
    (void)hipEventCreate(&a);
    (void)hipEventCreate(&b);
    const int64_t ranges[] = {int64_t(1) << 15, int64_t(1) << 18, int64_t(1) << 19, int64_t(1) << 21,
                              int64_t(1) << 24, int64_t(1) << 26, int64_t(1) << 28};
    const unsigned blocks = static_cast<unsigned>((m + 2047) / 2048);
    for (int skew = 0; skew < 2; ++skew)
        for (int64_t r : ranges) {
            mkidx<<<4096, 256>>>(idx, m, r, 7, skew);
            gather<<<blocks, 256>>>(idx, tab, out, m);
            (void)hipEventRecord(a);
            for (int it = 0; it < 3; ++it) gather<<<blocks, 256>>>(idx, tab, out, m);
            (void)hipEventRecord(b);
            (void)hipEventSynchronize(b);
            float ms = 0;
            (void)hipEventElapsedTime(&ms, a, b);
            ms /= 3;
            std::printf("%s table %9.1f MB: %7.3f ms per 2^28 gathers (%6.1f G gathers/s)\n",
                        skew ? "skewed " : "uniform", static_cast<double>(r) * 8 / 1048576.0, ms, m / ms / 1e6);
        }
    return 0;
}

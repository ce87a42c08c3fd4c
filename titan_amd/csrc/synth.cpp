// synth.cpp — RMAT generator for the bench / parity tests (see include/tgo_synth.h).
#include <algorithm>
#include <atomic>
#include <thread>
#include <vector>
#include "../../include/tgo_synth.h"
#include "../../include/titan_gpu_olap.h"
#include "../../include/titan_gpu_olap_part.h"

namespace {

inline uint64_t splitmix64(uint64_t x) {
    x += 0x9E3779B97F4A7C15ULL;
    x = (x ^ (x >> 30)) * 0xBF58476D1CE4E5B9ULL;
    x = (x ^ (x >> 27)) * 0x94D049BB133111EBULL;
    return x ^ (x >> 31);
}

}  // namespace

namespace tgo {
// Seeded permutation of [0, n) (Fisher-Yates driven by splitmix64); rmat_dev.hip uses it too.
std::vector<int32_t> rmat_relabel(int64_t n, uint64_t seed) {
    std::vector<int32_t> p(n);
    for (int64_t i = 0; i < n; ++i) p[i] = static_cast<int32_t>(i);
    for (int64_t i = n - 1; i > 0; --i) {
        const uint64_t r = splitmix64(seed ^ (0xA5A5A5A5ULL + static_cast<uint64_t>(i)));
        const int64_t j = static_cast<int64_t>(r % static_cast<uint64_t>(i + 1));
        std::swap(p[i], p[j]);
    }
    return p;
}
}  // namespace tgo
using tgo::rmat_relabel;

static void rmat_range(int32_t scale, uint64_t seed, int64_t edge_begin, int64_t count,
                       const std::vector<int32_t>& perm, int32_t* src, int32_t* dst, int32_t* weight,
                       int threads) {
    // Quadrant thresholds in 16-bit fixed point: A=0.57, A+B=0.76, A+B+C=0.95.
    const uint32_t tA = static_cast<uint32_t>(0.57 * 65536.0);
    const uint32_t tB = static_cast<uint32_t>(0.76 * 65536.0);
    const uint32_t tC = static_cast<uint32_t>(0.95 * 65536.0);
    auto work = [&](int64_t lo, int64_t hi) {
        for (int64_t k = lo; k < hi; ++k) {
            const uint64_t e = static_cast<uint64_t>(edge_begin + k);
            uint64_t u = 0, v = 0;
            uint64_t r = 0;
            for (int lvl = 0; lvl < scale; ++lvl) {
                if ((lvl & 3) == 0) r = splitmix64(seed + e * 0x100000001B3ULL + static_cast<uint64_t>(lvl));
                const uint32_t x = static_cast<uint32_t>(r & 0xFFFF);
                r >>= 16;
                const uint64_t bu = x >= tB ? 1 : 0;               // quadrants C, D: lower half
                const uint64_t bv = (x >= tA && x < tB) || x >= tC ? 1 : 0;   // B, D: right half
                u = (u << 1) | bu;
                v = (v << 1) | bv;
            }
            src[k] = perm[u];
            dst[k] = perm[v];
            if (weight) weight[k] = 1 + static_cast<int32_t>(splitmix64(seed ^ e) % 255u);
        }
    };
    std::vector<std::thread> th;
    for (int t = 0; t < threads; ++t) {
        const int64_t lo = count * t / threads, hi = count * (t + 1) / threads;
        th.emplace_back(work, lo, hi);
    }
    for (auto& x : th) x.join();
}

static int clamp_threads(int threads) {
    if (threads <= 0) threads = static_cast<int>(std::thread::hardware_concurrency());
    return std::max(1, std::min(threads, 64));
}

extern "C" int tgo_rmat_edges(int32_t scale, int32_t edge_factor, uint64_t seed, int64_t edge_begin,
                              int64_t count, int32_t* src, int32_t* dst, int32_t* weight, int32_t threads) {
    if (scale < 1 || scale > 30 || edge_factor < 1 || count < 0 || !src || !dst) return TGO_E_INVALID;
    const std::vector<int32_t> perm = rmat_relabel(int64_t(1) << scale, seed ^ 0x5EED5EEDULL);
    rmat_range(scale, seed, edge_begin, count, perm, src, dst, weight, clamp_threads(threads));
    return TGO_OK;
}

extern "C" int tgo_rmat_partition(int32_t scale, int32_t edge_factor, uint64_t seed, int64_t lo, int64_t hi,
                                  int32_t* src, int32_t* dst, int32_t* weight, int64_t capacity,
                                  int64_t* count, int32_t threads) {
    if (scale < 1 || scale > 30 || edge_factor < 1 || !count || lo < 0 || hi <= lo) return TGO_E_INVALID;
    threads = clamp_threads(threads);
    const std::vector<int32_t> perm = rmat_relabel(int64_t(1) << scale, seed ^ 0x5EED5EEDULL);
    const int64_t m = static_cast<int64_t>(edge_factor) << scale;
    const int64_t chunk = int64_t(1) << 24;
    std::vector<int32_t> s(chunk), d(chunk), w(weight ? chunk : 0);
    int64_t got = 0;
    bool overflow = false;
    // Stream the full edge list in chunks (counter-based, so every rank sees the same
    // stream) and keep the edges with an endpoint in [lo, hi).
    for (int64_t e0 = 0; e0 < m; e0 += chunk) {
        const int64_t c = std::min(chunk, m - e0);
        rmat_range(scale, seed, e0, c, perm, s.data(), d.data(), weight ? w.data() : nullptr, threads);
        for (int64_t k = 0; k < c; ++k) {
            if ((s[k] >= lo && s[k] < hi) || (d[k] >= lo && d[k] < hi)) {
                if (got < capacity && src && dst) {
                    src[got] = s[k];
                    dst[got] = d[k];
                    if (weight) weight[got] = w[k];
                } else {
                    overflow = true;
                }
                ++got;
            }
        }
    }
    *count = got;
    return overflow ? TGO_E_INVALID : TGO_OK;
}

extern "C" int tgo_pick_roots(int64_t n, int64_t m, const int32_t* src, const int32_t* dst, uint64_t seed,
                              int32_t nroots, int64_t* roots_out) {
    if (n <= 0 || nroots < 0 || !roots_out) return TGO_E_INVALID;
    std::vector<uint8_t> has(n, 0);
    for (int64_t k = 0; k < m; ++k) { has[src[k]] = 1; has[dst[k]] = 1; }
    int64_t nz = 0;
    for (int64_t v = 0; v < n; ++v) nz += has[v];
    if (nz < nroots) return TGO_E_INVALID;
    std::vector<uint8_t> used(n, 0);
    int32_t got = 0;
    for (uint64_t i = 0; got < nroots; ++i) {
        const int64_t v = static_cast<int64_t>(splitmix64(seed * 0x9E3779B97F4A7C15ULL + i) % static_cast<uint64_t>(n));
        if (!has[v] || used[v]) continue;
        used[v] = 1;
        roots_out[got++] = v;
    }
    return TGO_OK;
}

// tmp_cache.cpp — reuse of the large temporaries of the load-time device builds.
//
// The assembly, the partition assembly and the PageRank layout build allocate and free tens of
// GB of temporaries (radix-sort keys, scans, compactions) phase after phase.  At RMAT-27 a
// freshly allocated multi-GB buffer sometimes cost seconds on its first use (one phase per
// load, ~4.5 s, in a different phase each time: profiles/r04f_load27.log), while reusing
// memory the process already touched is fast.  So a freed temporary of >= 64 MB is kept and
// handed to the next request it fits (best fit within 2x), and every load entry point trims
// the cache when it ends (tgo::tmp_trim), so nothing stays reserved between loads.
#include <algorithm>
#include <chrono>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <mutex>
#include <vector>

#include <hip/hip_runtime.h>

namespace tgo {
namespace {
constexpr size_t kCacheMin = size_t(64) << 20;
struct Block { void* p; size_t bytes; };
std::mutex g_mu;
std::vector<Block> g_free;

// TGO_TRACE=1: a driver call of >= 50 ms on stderr (the load laps show which phase stalls,
// this shows whether an allocation or a device synchronisation is the stall)
template <class F>
hipError_t timed(const char* what, size_t bytes, F&& f) {
    static const bool trace = std::getenv("TGO_TRACE") && std::atoi(std::getenv("TGO_TRACE")) != 0;
    if (!trace) return f();
    const auto t0 = std::chrono::steady_clock::now();
    const hipError_t e = f();
    const double ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
    if (ms >= 50.0) std::fprintf(stderr, "[tgo]     tmp %s %.2f GB: %.1f ms\n", what, bytes / 1e9, ms);
    return e;
}
}  // namespace

hipError_t tmp_alloc(void** p, size_t bytes) {
    *p = nullptr;
    if (bytes >= kCacheMin) {
        std::lock_guard<std::mutex> lk(g_mu);
        size_t best = g_free.size();
        for (size_t i = 0; i < g_free.size(); ++i)
            if (g_free[i].bytes >= bytes && g_free[i].bytes <= 2 * bytes &&
                (best == g_free.size() || g_free[i].bytes < g_free[best].bytes))
                best = i;
        if (best < g_free.size()) {
            *p = g_free[best].p;
            g_free.erase(g_free.begin() + static_cast<long>(best));
            // its previous user's work may still be queued (on any stream, host copies included):
            // hand it out only once the device is idle
            return timed("reuse sync", bytes, [] { return hipDeviceSynchronize(); });
        }
    }
    hipError_t e = timed("hipMalloc", bytes, [&] { return hipMalloc(p, bytes); });
    if (e == hipErrorOutOfMemory) {             // give the cached blocks back and retry once
        {
            std::lock_guard<std::mutex> lk(g_mu);
            for (const Block& b : g_free) (void)hipFree(b.p);
            g_free.clear();
        }
        (void)hipGetLastError();
        e = hipMalloc(p, bytes);
    }
    return e;
}

// the block's size must be the one it was allocated with (the caller's request, or more when
// it came from the cache: callers pass their request; a cached block's real size is kept here)
void tmp_free(void* p, size_t bytes) {
    if (!p) return;
    if (bytes >= kCacheMin) {
        std::lock_guard<std::mutex> lk(g_mu);
        g_free.push_back({p, bytes});
        return;
    }
    (void)hipFree(p);
}

void tmp_trim() {
    std::lock_guard<std::mutex> lk(g_mu);
    for (const Block& b : g_free) (void)hipFree(b.p);
    g_free.clear();
}

}  // namespace tgo

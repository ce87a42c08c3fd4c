// tmp_cache.cpp — reuse of the large temporaries of the load-time device builds.
//
// The assembly, the partition assembly and the PageRank layout build allocate and free tens of
// GB of temporaries (radix-sort keys, scans, compactions) phase after phase.  At RMAT-27 a
// freshly allocated multi-GB buffer sometimes cost seconds on its first use (one phase per
// load, ~4.5 s, in a different phase each time: profiles/r04f_load27.log), while reusing
// memory the process already touched is fast.  So a freed temporary of >= 64 MB is kept and
// handed to the next request it fits (best fit within 2x), and every load entry point trims
// the cache when it ends (tgo::tmp_trim), so nothing stays reserved between loads.  Cached
// blocks and the copy-out staging are per device: contexts on different GPUs may load at once.
#include <algorithm>
#include <chrono>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <mutex>
#include <thread>
#include <unordered_map>
#include <vector>

#include <sys/mman.h>

#include <hip/hip_runtime.h>

namespace tgo {
namespace {
constexpr size_t kCacheMin = size_t(64) << 20;
struct Block { void* p; size_t bytes; int dev; };
std::mutex g_mu;
std::vector<Block> g_free;
// real sizes of the cached blocks handed out (a reuse may be up to 2x the request; the caller
// frees with its request, and the block goes back to the cache with its real size)
std::unordered_map<void*, size_t> g_real;

int current_device() {
    int d = 0;
    if (hipGetDevice(&d) != hipSuccess) { (void)hipGetLastError(); d = 0; }
    return d;
}

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
        const int dev = current_device();
        std::lock_guard<std::mutex> lk(g_mu);
        size_t best = g_free.size();
        for (size_t i = 0; i < g_free.size(); ++i)
            if (g_free[i].dev == dev && g_free[i].bytes >= bytes && g_free[i].bytes <= 2 * bytes &&
                (best == g_free.size() || g_free[i].bytes < g_free[best].bytes))
                best = i;
        if (best < g_free.size()) {
            *p = g_free[best].p;
            g_real[*p] = g_free[best].bytes;
            g_free.erase(g_free.begin() + static_cast<long>(best));
            // its previous user's work may still be queued (on any stream of this device, host
            // copies included): hand it out only once the device is idle
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
    if (e == hipSuccess && *p) {
        // a fresh address may be one a reused block had before it left the cache for good (a
        // take() into a graph array, freed later with hipFree): its recorded real size is stale
        // and would let the block back into the cache as larger than it is — a later request
        // handed it would write past its end (the world-6 RMAT-24 fault, gpurun_out/r06g)
        std::lock_guard<std::mutex> lk(g_mu);
        g_real.erase(*p);
    }
    return e;
}

// A block handed out by tmp_alloc leaves the cache's management (ScopedBuf / Buf take(): it
// becomes a graph array, freed with hipFree): forget its recorded real size.
void tmp_disown(void* p) {
    if (!p) return;
    std::lock_guard<std::mutex> lk(g_mu);
    g_real.erase(p);
}

// callers pass their request size; a block that came from the cache goes back with its real
// size (g_real), and every block is cached under the device current at its free — the one it
// was allocated on, as every caller allocates and frees under the same context
void tmp_free(void* p, size_t bytes) {
    if (!p) return;
    if (bytes >= kCacheMin) {
        const int dev = current_device();
        std::lock_guard<std::mutex> lk(g_mu);
        const auto it = g_real.find(p);
        if (it != g_real.end()) {
            bytes = std::max(bytes, it->second);
            g_real.erase(it);
        }
        g_free.push_back({p, bytes, dev});
        return;
    }
    (void)hipFree(p);
}

void advise_huge(void* p, size_t bytes) {
    constexpr uintptr_t kHuge = uintptr_t(2) << 20;
    const uintptr_t a = (reinterpret_cast<uintptr_t>(p) + kHuge - 1) & ~(kHuge - 1);
    const uintptr_t b = (reinterpret_cast<uintptr_t>(p) + bytes) & ~(kHuge - 1);
    if (b > a) (void)madvise(reinterpret_cast<void*>(a), b - a, MADV_HUGEPAGE);
}

hipError_t copy_d2h(void* dst, const void* src, size_t bytes) {
    constexpr size_t kPiece = size_t(64) << 20;
    constexpr int kThreads = 8;
    auto plain = [&] {
        for (size_t o = 0; o < bytes; o += 4 * kPiece) {
            const hipError_t e = hipMemcpy(static_cast<char*>(dst) + o, static_cast<const char*>(src) + o,
                                           std::min(4 * kPiece, bytes - o), hipMemcpyDeviceToHost);
            if (e != hipSuccess) return e;
        }
        return hipSuccess;
    };
    if (bytes < 4 * kPiece) return plain();
    // the staging stream, events and pinned buffers of the current device (a stream belongs to
    // the device it was created on: another device's copies must not go through it)
    struct Staging {
        std::mutex mu;
        void* pin[2] = {nullptr, nullptr};
        hipStream_t st = nullptr;
        hipEvent_t ev[2] = {nullptr, nullptr};
        bool ready = false, failed = false;
    };
    constexpr int kMaxDevices = 64;
    static Staging per_dev[kMaxDevices];
    const int dev = current_device();
    if (dev < 0 || dev >= kMaxDevices) return plain();
    Staging& S = per_dev[dev];
    std::lock_guard<std::mutex> lk(S.mu);
    void** const pin = S.pin;
    hipEvent_t* const ev = S.ev;
    hipStream_t& st = S.st;
    bool& ready = S.ready;
    bool& failed = S.failed;
    if (!ready && !failed) {
        failed = hipHostMalloc(&pin[0], kPiece, hipHostMallocDefault) != hipSuccess ||
                 hipHostMalloc(&pin[1], kPiece, hipHostMallocDefault) != hipSuccess ||
                 hipStreamCreateWithFlags(&st, hipStreamNonBlocking) != hipSuccess ||
                 hipEventCreateWithFlags(&ev[0], hipEventDisableTiming) != hipSuccess ||
                 hipEventCreateWithFlags(&ev[1], hipEventDisableTiming) != hipSuccess;
        ready = !failed;
        (void)hipGetLastError();
    }
    if (!ready) return plain();
    const size_t np = (bytes + kPiece - 1) / kPiece;
    auto issue = [&](size_t i) -> hipError_t {
        const size_t o = i * kPiece, len = std::min(kPiece, bytes - o);
        hipError_t e = hipMemcpyAsync(pin[i & 1], static_cast<const char*>(src) + o, len, hipMemcpyDeviceToHost, st);
        if (e == hipSuccess) e = hipEventRecord(ev[i & 1], st);
        return e;
    };
    hipError_t e = issue(0);
    for (size_t i = 0; i < np && e == hipSuccess; ++i) {
        if (i + 1 < np && (e = issue(i + 1)) != hipSuccess) break;
        if ((e = hipEventSynchronize(ev[i & 1])) != hipSuccess) break;
        const size_t o = i * kPiece, len = std::min(kPiece, bytes - o);
        const size_t per = (len + kThreads - 1) / kThreads;
        std::thread th[kThreads];
        for (int t = 0; t < kThreads; ++t) {
            const size_t a = std::min(len, t * per), b = std::min(len, a + per);
            th[t] = std::thread([=] {
                if (b > a) std::memcpy(static_cast<char*>(dst) + o + a, static_cast<const char*>(pin[i & 1]) + a, b - a);
            });
        }
        for (auto& x : th) x.join();
    }
    if (e != hipSuccess) (void)hipStreamSynchronize(st);
    return e;
}

void tmp_trim() {
    std::lock_guard<std::mutex> lk(g_mu);
    for (const Block& b : g_free) (void)hipFree(b.p);
    g_free.clear();
}

}  // namespace tgo

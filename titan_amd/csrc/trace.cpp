// trace.cpp — spans, roctx ranges and the Chrome-trace JSON writer (trace.hpp).
#include "trace.hpp"

#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <mutex>
#include <thread>
#include <vector>

#include <rocprofiler-sdk-roctx/roctx.h>

#include "../../include/titan_gpu_olap.h"

namespace tgo {

std::atomic<int> g_trace_flags{0};

namespace {

struct Event {
    std::string name;
    double ts = 0, dur = 0;            // microseconds since the trace base
    uint64_t tid = 0;
    int dev = 0;                       // 0 host span, 1 device span
    TraceArg a{nullptr, 0}, b{nullptr, 0};
};
struct Pending {
    hipStream_t s;
    std::string name;
    TraceArg a, b;
    hipEvent_t e0, e1;
};

struct State {
    std::mutex mu;
    std::vector<Event> events;
    std::vector<Pending> pending;
    std::vector<hipEvent_t> pool;
    std::string path;
    std::chrono::steady_clock::time_point base = std::chrono::steady_clock::now();
    bool atexit_set = false;
};
State& st() {
    static State* s = new State();     // never destroyed: spans may end during static teardown
    return *s;
}
double now_us() {
    return std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() - st().base).count();
}
uint64_t tid_now() { return static_cast<uint64_t>(std::hash<std::thread::id>()(std::this_thread::get_id()) & 0xFFFFFF); }

hipEvent_t take_event() {
    State& S = st();
    {
        std::lock_guard<std::mutex> lk(S.mu);
        if (!S.pool.empty()) { hipEvent_t e = S.pool.back(); S.pool.pop_back(); return e; }
    }
    hipEvent_t e = nullptr;
    if (hipEventCreate(&e) != hipSuccess) return nullptr;
    return e;
}

void json_escape(std::FILE* f, const std::string& s) {
    for (char c : s) {
        if (c == '"' || c == '\\') std::fputc('\\', f);
        if (static_cast<unsigned char>(c) >= 0x20) std::fputc(c, f);
    }
}

int write_json(const char* path) {
    State& S = st();
    std::lock_guard<std::mutex> lk(S.mu);
    std::FILE* f = std::fopen(path, "w");
    if (!f) return TGO_E_INVALID;
    std::fprintf(f, "{\"displayTimeUnit\": \"ms\", \"otherData\": {\"producer\": \"titan_amd\"}, \"traceEvents\": [\n");
    for (size_t i = 0; i < S.events.size(); ++i) {
        const Event& e = S.events[i];
        std::fprintf(f, "{\"name\": \"");
        json_escape(f, e.name);
        std::fprintf(f, "\", \"cat\": \"%s\", \"ph\": \"X\", \"ts\": %.3f, \"dur\": %.3f, \"pid\": %d, \"tid\": %llu",
                     e.dev ? "device" : "host", e.ts, e.dur, e.dev ? 1 : 0, static_cast<unsigned long long>(e.tid));
        std::fprintf(f, ", \"args\": {");
        bool first = true;
        for (const TraceArg& a : {e.a, e.b}) {
            if (!a.key) continue;
            std::fprintf(f, "%s\"%s\": %lld", first ? "" : ", ", a.key, static_cast<long long>(a.value));
            first = false;
        }
        std::fprintf(f, "}}%s\n", i + 1 < S.events.size() ? "," : "");
    }
    std::fprintf(f, "]}\n");
    return std::fclose(f) == 0 ? TGO_OK : TGO_E_INVALID;
}

void flush_at_exit() {
    State& S = st();
    if (!S.path.empty() && (g_trace_flags.load() & kTraceJson)) (void)write_json(S.path.c_str());
}

// environment switches, read once at load
struct EnvInit {
    EnvInit() {
        int flags = 0;
        if (const char* p = std::getenv("TGO_TRACE_JSON")) {
            if (*p) { st().path = p; flags |= kTraceJson; }
        }
        if (const char* r = std::getenv("TGO_TRACE_ROCTX")) if (std::atoi(r) != 0) flags |= kTraceRoctx;
        if (flags & kTraceJson) { std::atexit(flush_at_exit); st().atexit_set = true; }
        g_trace_flags.store(flags);
    }
} env_init;

}  // namespace

Span::Span(const char* name, TraceArg a, TraceArg b) : name_(name), a_(a), b_(b) {
    const int f = g_trace_flags.load(std::memory_order_relaxed);
    if (!f) return;
    if (f & kTraceRoctx) { roctxRangePushA(name); roctx_ = true; }
    if (f & kTraceJson) t0_ = static_cast<int64_t>(now_us() * 1000.0);
}
Span::~Span() {
    if (roctx_) roctxRangePop();
    if (t0_ < 0) return;
    Event e;
    e.name = name_;
    e.ts = static_cast<double>(t0_) / 1000.0;
    e.dur = now_us() - e.ts;
    e.tid = tid_now();
    e.a = a_;
    e.b = b_;
    State& S = st();
    std::lock_guard<std::mutex> lk(S.mu);
    S.events.push_back(std::move(e));
}

DevSpan::DevSpan(hipStream_t s, const char* name, TraceArg a, TraceArg b) : s_(s), name_(name), a_(a), b_(b) {
    const int f = g_trace_flags.load(std::memory_order_relaxed);
    if (!f) return;
    if (f & kTraceRoctx) { roctxRangePushA(name); roctx_ = true; }
    if (f & kTraceJson) {
        e0_ = take_event();
        e1_ = take_event();
        if (e0_ && e1_ && hipEventRecord(e0_, s_) == hipSuccess) open_ = true;
    }
}
void DevSpan::end() {
    if (roctx_) { roctxRangePop(); roctx_ = false; }
    if (!open_) return;
    open_ = false;
    if (hipEventRecord(e1_, s_) != hipSuccess) return;
    State& S = st();
    std::lock_guard<std::mutex> lk(S.mu);
    S.pending.push_back({s_, name_, a_, b_, e0_, e1_});
}

void trace_complete(const std::string& name, double dur_us) {
    if (!(g_trace_flags.load(std::memory_order_relaxed) & kTraceJson)) return;
    Event e;
    e.name = name;
    e.dur = dur_us;
    e.ts = now_us() - dur_us;
    e.tid = tid_now();
    State& S = st();
    std::lock_guard<std::mutex> lk(S.mu);
    S.events.push_back(std::move(e));
}

void trace_resolve(hipStream_t s) {
    if (!(g_trace_flags.load(std::memory_order_relaxed) & kTraceJson)) return;
    State& S = st();
    std::vector<Pending> mine;
    {
        std::lock_guard<std::mutex> lk(S.mu);
        for (size_t i = 0; i < S.pending.size();) {
            if (S.pending[i].s == s) { mine.push_back(S.pending[i]); S.pending[i] = S.pending.back(); S.pending.pop_back(); }
            else ++i;
        }
    }
    if (mine.empty()) return;
    // reference: an event recorded now, completed before the host clock is read
    hipEvent_t ref = take_event();
    if (!ref || hipEventRecord(ref, s) != hipSuccess || hipEventSynchronize(ref) != hipSuccess) return;
    const double host_ref = now_us();
    const uint64_t tid = 0x1000000ULL + (reinterpret_cast<uintptr_t>(s) & 0xFFFFFF);
    std::vector<Event> out;
    for (const Pending& p : mine) {
        float a = 0.f, d = 0.f;
        if (hipEventElapsedTime(&a, p.e0, ref) != hipSuccess || hipEventElapsedTime(&d, p.e0, p.e1) != hipSuccess) continue;
        Event e;
        e.name = p.name;
        e.ts = host_ref - static_cast<double>(a) * 1000.0;
        e.dur = static_cast<double>(d) * 1000.0;
        e.tid = tid;
        e.dev = 1;
        e.a = p.a;
        e.b = p.b;
        out.push_back(std::move(e));
    }
    std::lock_guard<std::mutex> lk(S.mu);
    for (auto& e : out) S.events.push_back(std::move(e));
    for (const Pending& p : mine) { S.pool.push_back(p.e0); S.pool.push_back(p.e1); }
    S.pool.push_back(ref);
}

}  // namespace tgo

using namespace tgo;

extern "C" {

int tgo_trace_enable(const char* json_path, int32_t flags) {
    if (flags < 0 || flags > (kTraceJson | kTraceRoctx)) return TGO_E_INVALID;
    if ((flags & kTraceJson) && (!json_path || !*json_path)) return TGO_E_INVALID;
    State& S = st();
    {
        std::lock_guard<std::mutex> lk(S.mu);
        if (json_path) S.path = json_path;
        if ((flags & kTraceJson) && !S.atexit_set) { std::atexit(flush_at_exit); S.atexit_set = true; }
    }
    g_trace_flags.store(flags);
    return TGO_OK;
}

int tgo_trace_flush(const char* json_path) {
    State& S = st();
    std::string p = json_path ? std::string(json_path) : S.path;
    if (p.empty()) return TGO_E_INVALID;
    return write_json(p.c_str());
}

int tgo_trace_clear(void) {
    State& S = st();
    std::lock_guard<std::mutex> lk(S.mu);
    S.events.clear();
    return TGO_OK;
}

// caller ranges (the Java computer's supersteps, bench legs): a per-thread stack; pop emits
// the complete span
thread_local std::vector<std::pair<std::string, double>> t_ranges;

int tgo_trace_range_push(const char* name) {
    if (!name) return TGO_E_INVALID;
    const int f = g_trace_flags.load();
    if (f & kTraceRoctx) roctxRangePushA(name);
    t_ranges.emplace_back(name, now_us());
    return TGO_OK;
}

int tgo_trace_range_pop(void) {
    if (t_ranges.empty()) return TGO_E_STATE;
    const int f = g_trace_flags.load();
    if (f & kTraceRoctx) roctxRangePop();
    auto r = std::move(t_ranges.back());
    t_ranges.pop_back();
    if (f & kTraceJson) {
        Event e;
        e.name = std::move(r.first);
        e.ts = r.second;
        e.dur = now_us() - r.second;
        e.tid = tid_now();
        State& S = st();
        std::lock_guard<std::mutex> lk(S.mu);
        S.events.push_back(std::move(e));
    }
    return TGO_OK;
}

}  // extern "C"

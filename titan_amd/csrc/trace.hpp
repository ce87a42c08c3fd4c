// trace.hpp — per-superstep / per-level / per-phase tracing of the engine.
//
// The reference stamps a program's runtime into its memory (FulgoraGraphComputer.java:143,
// 307: memory.setRuntime) and nothing finer.  Here every program marks its supersteps,
// levels and phases as spans:
//   * roctx ranges (roctxRangePushA / Pop) when TGO_TRACE_ROCTX is on, so rocprofv3
//     --marker-trace shows them beside the kernels;
//   * a Chrome-trace JSON ("traceEvents", ph = "X") written by tgo_trace_flush: host spans
//     (load phases, host-driven loops) with host timestamps, and device spans — a pair of HIP
//     events recorded on the engine stream around the span's kernels — resolved to GPU
//     timestamps when the program ends (tgo::trace_resolve after its stream synchronises).
// Off (the default) a span costs one relaxed atomic load.  Enabled with tgo_trace_enable or
// the environment: TGO_TRACE_JSON=<path> (flushed at exit), TGO_TRACE_ROCTX=1.
#pragma once
#include <atomic>
#include <cstdint>
#include <string>

#include <hip/hip_runtime.h>

namespace tgo {

enum : int { kTraceJson = 1, kTraceRoctx = 2 };
extern std::atomic<int> g_trace_flags;
inline bool tracing() { return g_trace_flags.load(std::memory_order_relaxed) != 0; }

// one argument of a span (the level / iteration / frontier size ...)
struct TraceArg {
    const char* key;
    int64_t value;
};

// A host span: [construction, destruction) on this thread.
class Span {
public:
    Span(const char* name, TraceArg a = {nullptr, 0}, TraceArg b = {nullptr, 0});
    ~Span();
    Span(const Span&) = delete;
    Span& operator=(const Span&) = delete;
private:
    const char* name_;
    TraceArg a_, b_;
    int64_t t0_ = -1;
    bool roctx_ = false;
};

// A device span on stream s: events recorded now and at end(); resolved by trace_resolve.
class DevSpan {
public:
    DevSpan(hipStream_t s, const char* name, TraceArg a = {nullptr, 0}, TraceArg b = {nullptr, 0});
    ~DevSpan() { end(); }
    void end();
    DevSpan(const DevSpan&) = delete;
    DevSpan& operator=(const DevSpan&) = delete;
private:
    hipStream_t s_;
    const char* name_;
    TraceArg a_, b_;
    hipEvent_t e0_ = nullptr, e1_ = nullptr;
    bool roctx_ = false, open_ = false;
};

// A finished host phase of `dur_us` ending now (the load paths' phase laps).
void trace_complete(const std::string& name, double dur_us);

// Converts the finished device spans of stream s to timestamped events (call after the
// stream synchronised, e.g. at the end of a program).
void trace_resolve(hipStream_t s);

}  // namespace tgo

// generic.hip — message passing for vertex programs the engine does not implement natively
// (SURVEY.md §8f-4).  The program's execute() runs on the host over whole vectors; the
// device does what Fulgora spends its time on: combining messages.
//
//   Local scope  (MessageScope.Local(incident, edgeFct)): every vertex combines
//                edgeFct(msg[u], e) over the entries of its reversed incident traversal
//                whose sender holds a message (VertexMemoryHandler.receiveMessages,
//                VertexMemoryHandler.java:77-93; reversal FulgoraUtil.java:57), with the
//                program's combiner.  One thread per vertex, entries in list order: MIN/MAX
//                and int64 SUM are exact in any order, fp64 SUM adds in list order (fixed).
//   Global scope (MessageScope.Global): messages to explicit targets are combined per target
//                (VertexState.addMessage with the combiner, VertexState.java:63-78) in MESSAGE
//                order: a stable radix sort by target, then one sequential fold per target —
//                bitwise equal to combining the messages one by one in the order they were sent.
//
// Java semantics: Long + Integer wraps (two's complement), hence unsigned adds for int64.
#include <cstdint>
#include <hip/hip_runtime.h>
#include <hipcub/hipcub.hpp>
#include "engine.hpp"

namespace tgo {
namespace {

constexpr int kBlock = 256;

inline int grid_for(int64_t work) {
    int64_t g = (work + kBlock - 1) / kBlock;
    return static_cast<int>(g < 1 ? 1 : (g > 65536 ? 65536 : g));
}

template <typename T>
__device__ __forceinline__ T combine(int comb, T acc, T m) {
    if (comb == TGO_COMBINE_MIN) return m < acc ? m : acc;
    if (comb == TGO_COMBINE_MAX) return m > acc ? m : acc;
    return acc + m;
}
template <>
__device__ __forceinline__ int64_t combine<int64_t>(int comb, int64_t acc, int64_t m) {
    if (comb == TGO_COMBINE_MIN) return m < acc ? m : acc;
    if (comb == TGO_COMBINE_MAX) return m > acc ? m : acc;
    return static_cast<int64_t>(static_cast<uint64_t>(acc) + static_cast<uint64_t>(m));
}

// edgeFct(m, e): identity, m + 1, m + e.value(weight), m * e.value(weight)
template <typename T>
__device__ __forceinline__ T edge_apply(int fn, T m, int32_t w) {
    if (fn == TGO_EDGE_ADD_ONE) return m + T(1);
    if (fn == TGO_EDGE_ADD_WEIGHT) return m + static_cast<T>(w);
    if (fn == TGO_EDGE_MUL_WEIGHT) return m * static_cast<T>(w);
    return m;
}
template <>
__device__ __forceinline__ int64_t edge_apply<int64_t>(int fn, int64_t m, int32_t w) {
    const uint64_t u = static_cast<uint64_t>(m);
    if (fn == TGO_EDGE_ADD_ONE) return static_cast<int64_t>(u + 1u);
    if (fn == TGO_EDGE_ADD_WEIGHT) return static_cast<int64_t>(u + static_cast<uint64_t>(static_cast<int64_t>(w)));
    if (fn == TGO_EDGE_MUL_WEIGHT) return static_cast<int64_t>(u * static_cast<uint64_t>(static_cast<int64_t>(w)));
    return m;
}

template <typename T>
__global__ void local_gather(View pull, int64_t n, const T* __restrict__ msg, const uint8_t* __restrict__ has,
                             int comb, int fn, T* __restrict__ out, uint8_t* __restrict__ out_has,
                             unsigned long long* err) {
    const bool needs_w = fn == TGO_EDGE_ADD_WEIGHT || fn == TGO_EDGE_MUL_WEIGHT;
    for (int64_t v = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; v < n; v += (int64_t)gridDim.x * blockDim.x) {
        T acc = T(0);
        bool any = false;
        for (int l = 0; l < pull.nlists; ++l) {
            const int64_t* off = l == 0 ? pull.off0 : pull.off1;
            const int32_t* adj = l == 0 ? pull.adj0 : pull.adj1;
            const int32_t* w = l == 0 ? pull.w0 : pull.w1;
            for (int64_t k = off[v]; k < off[v + 1]; ++k) {
                const int32_t u = adj[k];
                if (!has[u]) continue;                            // filter(m != null)
                int32_t wt = 0;
                if (needs_w) {
                    wt = w ? w[k] : kMissingWeight;
                    if (wt == kMissingWeight) { atomicOr(err, 1ull); continue; }   // e.value(key) throws
                }
                const T m = edge_apply<T>(fn, msg[u], wt);
                acc = any ? combine<T>(comb, acc, m) : m;
                any = true;
            }
        }
        out[v] = acc;
        out_has[v] = any ? 1 : 0;
    }
}

// internal[perm[r]] = row[r]
template <typename T>
__global__ void scatter_perm(const T* __restrict__ row, const int32_t* __restrict__ perm, T* __restrict__ internal,
                             int64_t n) {
    for (int64_t r = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; r < n; r += (int64_t)gridDim.x * blockDim.x)
        internal[perm[r]] = row[r];
}
// row[r] = internal[perm[r]]
template <typename T>
__global__ void gather_rows(const T* __restrict__ internal, const int32_t* __restrict__ perm, T* __restrict__ row,
                            int64_t n) {
    for (int64_t r = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; r < n; r += (int64_t)gridDim.x * blockDim.x)
        row[r] = internal[perm[r]];
}

// keys = targets (row ids), values = message index; sorted stably by target.  One thread per
// sorted position that starts a run folds the run in message order into out[target].
template <typename T>
__global__ void fold_runs(const int64_t* __restrict__ tkey, const int64_t* __restrict__ midx, int64_t m,
                          const T* __restrict__ values, int comb, T* __restrict__ out, uint8_t* __restrict__ out_has) {
    for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < m; i += (int64_t)gridDim.x * blockDim.x) {
        const int64_t t = tkey[i];
        if (i > 0 && tkey[i - 1] == t) continue;
        T acc = values[midx[i]];
        for (int64_t j = i + 1; j < m && tkey[j] == t; ++j) acc = combine<T>(comb, acc, values[midx[j]]);
        out[t] = acc;
        out_has[t] = 1;
    }
}
__global__ void iota_i64(int64_t* p, int64_t n) {
    for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) p[i] = i;
}

}  // namespace

hipError_t k_local_gather(const View& pull, int64_t n, int value_type, const void* msg_int, const uint8_t* has_int,
                          int comb, int fn, void* out_int, uint8_t* out_has_int, unsigned long long* err, hipStream_t s) {
    if (value_type == TGO_VAL_INT64)
        local_gather<int64_t><<<grid_for(n), kBlock, 0, s>>>(pull, n, static_cast<const int64_t*>(msg_int), has_int, comb,
                                                            fn, static_cast<int64_t*>(out_int), out_has_int, err);
    else
        local_gather<double><<<grid_for(n), kBlock, 0, s>>>(pull, n, static_cast<const double*>(msg_int), has_int, comb,
                                                           fn, static_cast<double*>(out_int), out_has_int, err);
    return hipGetLastError();
}

hipError_t k_to_internal(const void* row8, const uint8_t* row1, const int32_t* perm, void* int8, uint8_t* int1,
                         int64_t n, hipStream_t s) {
    if (row8) scatter_perm<int64_t><<<grid_for(n), kBlock, 0, s>>>(static_cast<const int64_t*>(row8), perm,
                                                                    static_cast<int64_t*>(int8), n);
    if (row1) scatter_perm<uint8_t><<<grid_for(n), kBlock, 0, s>>>(row1, perm, int1, n);
    return hipGetLastError();
}
hipError_t k_to_rows(const void* int8, const uint8_t* int1, const int32_t* perm, void* row8, uint8_t* row1, int64_t n,
                     hipStream_t s) {
    if (int8) gather_rows<int64_t><<<grid_for(n), kBlock, 0, s>>>(static_cast<const int64_t*>(int8), perm,
                                                                   static_cast<int64_t*>(row8), n);
    if (int1) gather_rows<uint8_t><<<grid_for(n), kBlock, 0, s>>>(int1, perm, row1, n);
    return hipGetLastError();
}

hipError_t k_global_combine(void*& tmp, size_t& tmp_bytes, const int64_t* targets, int64_t m, int64_t n,
                            int value_type, const void* values, int comb, int64_t* scratch4m, void* out,
                            uint8_t* out_has, hipStream_t s) {
    // scratch4m: [keys_out m][idx_in m][idx_out m] (targets are the input keys)
    int64_t* keys_out = scratch4m;
    int64_t* idx_in = scratch4m + m;
    int64_t* idx_out = scratch4m + 2 * m;
    iota_i64<<<grid_for(m), kBlock, 0, s>>>(idx_in, m);
    int end_bit = 1;
    while (end_bit < 63 && (int64_t(1) << end_bit) < n) ++end_bit;
    size_t need = 0;
    hipError_t e = hipcub::DeviceRadixSort::SortPairs(nullptr, need, targets, keys_out, idx_in, idx_out,
                                                      static_cast<int>(m), 0, end_bit, s);
    if (e != hipSuccess) return e;
    if (need > tmp_bytes) {
        if (tmp) (void)hipFree(tmp);
        tmp = nullptr;
        tmp_bytes = 0;
        if ((e = hipMalloc(&tmp, need)) != hipSuccess) return e;
        tmp_bytes = need;
    }
    e = hipcub::DeviceRadixSort::SortPairs(tmp, tmp_bytes, targets, keys_out, idx_in, idx_out, static_cast<int>(m), 0,
                                           end_bit, s);
    if (e != hipSuccess) return e;
    if (value_type == TGO_VAL_INT64)
        fold_runs<int64_t><<<grid_for(m), kBlock, 0, s>>>(keys_out, idx_out, m, static_cast<const int64_t*>(values), comb,
                                                         static_cast<int64_t*>(out), out_has);
    else
        fold_runs<double><<<grid_for(m), kBlock, 0, s>>>(keys_out, idx_out, m, static_cast<const double*>(values), comb,
                                                        static_cast<double*>(out), out_has);
    return hipGetLastError();
}

}  // namespace tgo

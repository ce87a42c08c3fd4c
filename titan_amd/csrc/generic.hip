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

// edgeFct(m, e) = "m op w", w = e.value(weight): the weight column holds 32-bit integers, a
// Float's IEEE bits, or an index into the Long / Double value table (WeightCol).  Error bits:
// 1 = an edge without the weight property (e.value() throws), 2 = int64 division by zero (Java
// ArithmeticException).
constexpr unsigned long long kErrNoWeight = 1, kErrDivZero = 2;
__host__ __device__ __forceinline__ bool weight_fn(int fn, const EdgeProg& pg) {
    return (fn >= TGO_EDGE_ADD_WEIGHT && fn <= TGO_EDGE_DIV_WEIGHT) || (fn == TGO_EDGE_PROGRAM && pg.uses_w);
}

// ---- edge-function programs (TGO_EDGE_PROGRAM): the postfix program interpreted per entry.
// The program is uniform, so every lane takes the same branch at every op; the stack index is
// uniform too.  Java long: + - * and negation wrap, / and % truncate toward zero (C's), / 0 and
// % 0 throw (kErrDivZero), MIN_VALUE / -1 = MIN_VALUE, MIN_VALUE % -1 = 0, Math.abs(MIN_VALUE) =
// MIN_VALUE.  Java double: IEEE; % is fmod; Math.min / max treat NaN and -0.0 as Java does.
__device__ __forceinline__ int64_t prog_op(int op, int64_t a, int64_t b, unsigned long long* err) {
    const uint64_t ua = static_cast<uint64_t>(a), ub = static_cast<uint64_t>(b);
    switch (op) {
        case TGO_OP_ADD: return static_cast<int64_t>(ua + ub);
        case TGO_OP_SUB: return static_cast<int64_t>(ua - ub);
        case TGO_OP_MUL: return static_cast<int64_t>(ua * ub);
        case TGO_OP_DIV:
            if (b == 0) { atomicOr(err, kErrDivZero); return 0; }
            return b == -1 ? static_cast<int64_t>(0ULL - ua) : a / b;
        case TGO_OP_REM:
            if (b == 0) { atomicOr(err, kErrDivZero); return 0; }
            return b == -1 ? 0 : a % b;
        case TGO_OP_MIN: return b < a ? b : a;
        default: return b > a ? b : a;                    // TGO_OP_MAX
    }
}
__device__ __forceinline__ double prog_op(int op, double a, double b, unsigned long long*) {
    switch (op) {
        case TGO_OP_ADD: return a + b;
        case TGO_OP_SUB: return a - b;
        case TGO_OP_MUL: return a * b;
        case TGO_OP_DIV: return a / b;
        case TGO_OP_REM: return fmod(a, b);
        case TGO_OP_MIN:                                   // Math.min(double, double)
            if (a != a) return a;
            if (a == 0.0 && b == 0.0 && signbit(b)) return b;
            return a <= b ? a : b;
        default:                                           // Math.max(double, double)
            if (a != a) return a;
            if (a == 0.0 && b == 0.0 && signbit(a)) return b;
            return a >= b ? a : b;
    }
}
__device__ __forceinline__ int64_t prog_neg(int64_t a) { return static_cast<int64_t>(0ULL - static_cast<uint64_t>(a)); }
__device__ __forceinline__ double prog_neg(double a) { return -a; }
__device__ __forceinline__ int64_t prog_abs(int64_t a) { return a < 0 ? prog_neg(a) : a; }
__device__ __forceinline__ double prog_abs(double a) { return a <= 0.0 ? 0.0 - a : a; }    // Math.abs(double)
__device__ __forceinline__ int64_t prog_const(const EdgeProg& pg, int i, int64_t) { return pg.ic[i]; }
__device__ __forceinline__ double prog_const(const EdgeProg& pg, int i, double) { return pg.fc[i]; }
template <typename T>
__device__ __forceinline__ T run_prog(const EdgeProg& pg, T m, T w, unsigned long long* err) {
    T st[TGO_EDGE_PROGRAM_MAX_STACK];
    int sp = 0;
    for (int i = 0; i < pg.n; ++i) {
        const int op = pg.ops[i] & 0xFF;
        switch (op) {
            case TGO_OP_MSG: st[sp++] = m; break;
            case TGO_OP_WEIGHT: st[sp++] = w; break;
            case TGO_OP_CONST: st[sp++] = prog_const(pg, pg.ops[i] >> 8, T(0)); break;
            case TGO_OP_NEG: st[sp - 1] = prog_neg(st[sp - 1]); break;
            case TGO_OP_ABS: st[sp - 1] = prog_abs(st[sp - 1]); break;
            default: st[sp - 2] = prog_op(op, st[sp - 2], st[sp - 1], err); --sp; break;
        }
    }
    return st[0];
}

// e.value(weight) widened to double (double message): the value by the column's kind
__device__ __forceinline__ double weight_f(int32_t w, const WeightCol& wc) {
    switch (wc.kind) {
        case 1: return static_cast<double>(__int_as_float(w));
        case 2: return static_cast<double>(wc.wide[w]);
        case 3: return __longlong_as_double(static_cast<long long>(wc.wide[w]));
        default: return static_cast<double>(w);
    }
}
__device__ __forceinline__ double edge_apply_f(int fn, double m, int32_t w, const WeightCol& wc, const EdgeProg& pg,
                                               unsigned long long* err) {
    if (fn == TGO_EDGE_IDENTITY) return m;
    if (fn == TGO_EDGE_PROGRAM) return run_prog<double>(pg, m, pg.uses_w ? weight_f(w, wc) : 0.0, err);
    if (fn == TGO_EDGE_ADD_ONE) return m + 1.0;
    const double x = weight_f(w, wc);
    switch (fn) {
        case TGO_EDGE_ADD_WEIGHT: return m + x;
        case TGO_EDGE_MUL_WEIGHT: return m * x;
        case TGO_EDGE_SUB_WEIGHT: return m - x;
        case TGO_EDGE_MIN_WEIGHT: return x < m ? x : m;
        case TGO_EDGE_MAX_WEIGHT: return x > m ? x : m;
        default: return m / x;                               // IEEE: x = 0 gives +-inf / NaN as in Java
    }
}
// Java long arithmetic: + - * wrap, / truncates toward zero, MIN_VALUE / -1 = MIN_VALUE
// (long message: the host admits integral columns only — an int or a Long)
__device__ __forceinline__ int64_t edge_apply_i(int fn, int64_t m, int32_t w, const WeightCol& wc,
                                                const EdgeProg& pg, unsigned long long* err) {
    const uint64_t u = static_cast<uint64_t>(m);
    if (fn == TGO_EDGE_IDENTITY) return m;
    if (fn == TGO_EDGE_PROGRAM)
        return run_prog<int64_t>(pg, m, pg.uses_w ? (wc.kind == 2 ? wc.wide[w] : static_cast<int64_t>(w)) : 0, err);
    if (fn == TGO_EDGE_ADD_ONE) return static_cast<int64_t>(u + 1u);
    const int64_t x = wc.kind == 2 ? wc.wide[w] : static_cast<int64_t>(w);
    switch (fn) {
        case TGO_EDGE_ADD_WEIGHT: return static_cast<int64_t>(u + static_cast<uint64_t>(x));
        case TGO_EDGE_MUL_WEIGHT: return static_cast<int64_t>(u * static_cast<uint64_t>(x));
        case TGO_EDGE_SUB_WEIGHT: return static_cast<int64_t>(u - static_cast<uint64_t>(x));
        case TGO_EDGE_MIN_WEIGHT: return x < m ? x : m;
        case TGO_EDGE_MAX_WEIGHT: return x > m ? x : m;
        default:
            if (x == 0) { atomicOr(err, kErrDivZero); return 0; }
            if (x == -1) return static_cast<int64_t>(0ULL - u);
            return m / x;
    }
}
template <typename T> __device__ __forceinline__ T edge_apply(int fn, T m, int32_t w, const WeightCol& wc,
                                                             const EdgeProg& pg, unsigned long long* err);
template <> __device__ __forceinline__ double edge_apply<double>(int fn, double m, int32_t w, const WeightCol& wc,
                                                               const EdgeProg& pg, unsigned long long* err) {
    return edge_apply_f(fn, m, w, wc, pg, err);
}
template <> __device__ __forceinline__ int64_t edge_apply<int64_t>(int fn, int64_t m, int32_t w, const WeightCol& wc,
                                                                 const EdgeProg& pg, unsigned long long* err) {
    return edge_apply_i(fn, m, w, wc, pg, err);
}

template <typename T>
__global__ void local_gather(View pull, int64_t n, const T* __restrict__ msg, const uint8_t* __restrict__ has,
                             int comb, int fn, WeightCol wc, EdgeProg pg, T* __restrict__ out,
                             uint8_t* __restrict__ out_has, unsigned long long* err) {
    const bool needs_w = weight_fn(fn, pg);
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
                    if (wt == kMissingWeight) { atomicOr(err, kErrNoWeight); continue; }   // e.value(key) throws
                }
                const T m = edge_apply<T>(fn, msg[u], wt, wc, pg, err);
                acc = any ? combine<T>(comb, acc, m) : m;
                any = true;
            }
        }
        out[v] = acc;
        out_has[v] = any ? 1 : 0;
    }
}

// ---- combiner-less receive (tgo_gather_lists): every row's message stream, materialised.
// Pass 1 counts a row's messages (entries whose sender holds one); after the scan, pass 2
// writes (order key, edgeFct(msg[u], e)) at the row's offsets; a segmented radix sort by key
// then puts each row's messages in column order (key = the entry's column position, kept by
// TGO_LOAD_COLUMN_ORDER loads) or (direction, neighbour row) order (key = list << 31 | row).
__global__ void list_count(View pull, const int32_t* __restrict__ perm, int64_t n, const uint8_t* __restrict__ has,
                           bool needs_w, int64_t* __restrict__ cnt, unsigned long long* err) {
    for (int64_t r = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; r < n; r += (int64_t)gridDim.x * blockDim.x) {
        const int64_t v = perm[r];
        int64_t c = 0;
        for (int l = 0; l < pull.nlists; ++l) {
            const int64_t* off = l == 0 ? pull.off0 : pull.off1;
            const int32_t* adj = l == 0 ? pull.adj0 : pull.adj1;
            const int32_t* w = l == 0 ? pull.w0 : pull.w1;
            for (int64_t k = off[v]; k < off[v + 1]; ++k) {
                if (!has[adj[k]]) continue;
                if (needs_w && (!w || w[k] == kMissingWeight)) { atomicOr(err, kErrNoWeight); continue; }
                ++c;
            }
        }
        cnt[r] = c;
    }
    if (blockIdx.x == 0 && threadIdx.x == 0) cnt[n] = 0;
}
template <typename T>
__global__ void list_fill(View pull, const uint32_t* __restrict__ col0, const uint32_t* __restrict__ col1,
                          const int32_t* __restrict__ perm, const int32_t* __restrict__ inv, int64_t n,
                          const T* __restrict__ msg, const uint8_t* __restrict__ has, int fn, WeightCol wc,
                          EdgeProg pg, const int64_t* __restrict__ off_out, uint32_t* __restrict__ key,
                          T* __restrict__ val, unsigned long long* err) {
    const bool needs_w = weight_fn(fn, pg);
    for (int64_t r = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; r < n; r += (int64_t)gridDim.x * blockDim.x) {
        const int64_t v = perm[r];
        int64_t p = off_out[r];
        for (int l = 0; l < pull.nlists; ++l) {
            const int64_t* off = l == 0 ? pull.off0 : pull.off1;
            const int32_t* adj = l == 0 ? pull.adj0 : pull.adj1;
            const int32_t* w = l == 0 ? pull.w0 : pull.w1;
            const uint32_t* col = l == 0 ? col0 : col1;
            for (int64_t k = off[v]; k < off[v + 1]; ++k) {
                const int32_t u = adj[k];
                if (!has[u]) continue;
                int32_t wt = 0;
                if (needs_w) {
                    wt = w ? w[k] : kMissingWeight;
                    if (wt == kMissingWeight) continue;
                }
                key[p] = col ? col[k] : ((static_cast<uint32_t>(l) << 31) | static_cast<uint32_t>(inv[u]));
                val[p] = edge_apply<T>(fn, msg[u], wt, wc, pg, err);
                ++p;
            }
        }
    }
}
__global__ void invert_perm(const int32_t* __restrict__ perm, int32_t* __restrict__ inv, int64_t n) {
    for (int64_t r = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; r < n; r += (int64_t)gridDim.x * blockDim.x)
        inv[perm[r]] = static_cast<int32_t>(r);
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
                          int comb, int fn, WeightCol wc, const EdgeProg& pg, void* out_int, uint8_t* out_has_int,
                          unsigned long long* err, hipStream_t s) {
    if (value_type == TGO_VAL_INT64)
        local_gather<int64_t><<<grid_for(n), kBlock, 0, s>>>(pull, n, static_cast<const int64_t*>(msg_int), has_int, comb,
                                                            fn, wc, pg, static_cast<int64_t*>(out_int), out_has_int, err);
    else
        local_gather<double><<<grid_for(n), kBlock, 0, s>>>(pull, n, static_cast<const double*>(msg_int), has_int, comb,
                                                           fn, wc, pg, static_cast<double*>(out_int), out_has_int, err);
    return hipGetLastError();
}

// Combiner-less receive: counts per row (row order) into cnt[0..n], cnt[n] = 0.
hipError_t k_list_count(const View& pull, const int32_t* perm, int64_t n, const uint8_t* has_int, bool needs_w,
                        int64_t* cnt, unsigned long long* err, hipStream_t s) {
    list_count<<<grid_for(n), kBlock, 0, s>>>(pull, perm, n, has_int, needs_w, cnt, err);
    return hipGetLastError();
}
// ... then the (key, value) pairs of every row at off_out[r], and a segmented sort of each
// row by key into key_out / val_out.  inv: n int32 scratch (internal -> row).
hipError_t k_list_fill_sort(const View& pull, const uint32_t* col0, const uint32_t* col1, const int32_t* perm,
                            int32_t* inv, int64_t n, int value_type, const void* msg_int, const uint8_t* has_int,
                            int fn, WeightCol wc, const EdgeProg& pg, const int64_t* off_out, int64_t total,
                            uint32_t* key_in, uint32_t* key_out, void* val_in, void* val_out, void*& tmp,
                            size_t& tmp_bytes, unsigned long long* err, hipStream_t s) {
    if (!col0) invert_perm<<<grid_for(n), kBlock, 0, s>>>(perm, inv, n);
    if (value_type == TGO_VAL_INT64)
        list_fill<int64_t><<<grid_for(n), kBlock, 0, s>>>(pull, col0, col1, perm, inv, n,
                                                         static_cast<const int64_t*>(msg_int), has_int, fn, wc, pg,
                                                         off_out, key_in, static_cast<int64_t*>(val_in), err);
    else
        list_fill<double><<<grid_for(n), kBlock, 0, s>>>(pull, col0, col1, perm, inv, n,
                                                        static_cast<const double*>(msg_int), has_int, fn, wc, pg,
                                                        off_out, key_in, static_cast<double*>(val_in), err);
    hipError_t e = hipGetLastError();
    if (e != hipSuccess || total == 0) return e;
    const uint64_t* vi = static_cast<const uint64_t*>(val_in);
    uint64_t* vo = static_cast<uint64_t*>(val_out);
    size_t need = 0;
    e = hipcub::DeviceSegmentedRadixSort::SortPairs(nullptr, need, key_in, key_out, vi, vo, static_cast<int>(total),
                                                    static_cast<int>(n), off_out, off_out + 1, 0, 32, s);
    if (e != hipSuccess) return e;
    if (need > tmp_bytes) {
        if (tmp) (void)hipFree(tmp);
        tmp = nullptr;
        tmp_bytes = 0;
        if ((e = hipMalloc(&tmp, need)) != hipSuccess) return e;
        tmp_bytes = need;
    }
    return hipcub::DeviceSegmentedRadixSort::SortPairs(tmp, tmp_bytes, key_in, key_out, vi, vo, static_cast<int>(total),
                                                       static_cast<int>(n), off_out, off_out + 1, 0, 32, s);
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

// results.hip — result write-back: the compute-key properties a finished
// program leaves on its vertices, encoded on the device as the edgestore entries Titan's
// commit path would write for them (FulgoraGraphComputer.java:248-305 writes each vertex's
// mutable properties through VertexPropertyWriter: v.property(Cardinality.single, key, value)).
//
// A SINGLE-cardinality property entry (EdgeSerializer.writeRelation :222-315, property branch
// :261-283; constrained and unique in direction OUT):
//   column = IDHandler.writeRelationType(keyId, PROPERTY_DIR)     (the key alone: a new value
//            for the same key overwrites the column, which is what single cardinality means)
//   valuePos = end of the column
//   value  = StandardSerializer null flag 0x00 + the attribute serializer
//            (LongSerializer: 8 bytes of v - Long.MIN_VALUE; DoubleSerializer: the raw IEEE bits;
//             IntegerSerializer: zig-zag VariableLong)
//            + VariableLong.writePositive(relationId)
// Rows come out in the API's row order (the scan's key order), one row per vertex that holds
// a property, its entries in column byte order; relation ids are base + running entry index
// (the Java side reserves that block from its IDAuthority).
//
// Three passes over the rows (entry counts -> scan -> byte sizes -> scan -> write), all
// HBM-streaming integer work: per row one 8-byte value read through perm and <= 2 entries of
// <= 25 bytes written.
#include <cstring>
#include <hip/hip_runtime.h>
#include "engine.hpp"

namespace tgo {
namespace {

constexpr int kBlock = 256;
inline int64_t grid_for(int64_t n) { return std::max<int64_t>(1, (n + kBlock - 1) / kBlock); }

__device__ inline int bit_len(uint64_t v) { return v == 0 ? 1 : 64 - __clzll(static_cast<long long>(v)); }
__device__ inline int pos_len(uint64_t v) { return (bit_len(v) - 1) / 7 + 1; }
// VariableLong.writePositive (VariableLong.java:84-87): 7-bit groups MSB first, stop bit last.
__device__ inline uint8_t* put_pos(uint8_t* p, uint64_t v) {
    for (int i = pos_len(v) - 1; i >= 0; --i) *p++ = static_cast<uint8_t>(((v >> (7 * i)) & 0x7F) | (i == 0 ? 0x80 : 0));
    return p;
}
__device__ inline uint64_t zigzag(int64_t v) {   // VariableLong.convert2Unsigned (:112-115)
    return v < 0 ? ((static_cast<uint64_t>(-v) << 1) | 1) : (static_cast<uint64_t>(v) << 1);
}

struct ResArgs {
    int kind;
    int vtype;              // TGO_RESULT_VALUES: TGO_VAL_INT64 / TGO_VAL_FP64
    int vdt;                // TGO_RESULT_VALUES: the value's encoding (TGO_DT_LONG / INTEGER / DOUBLE)
    int nkeys;
    uint8_t hdr[2][12];     // column bytes of each key, in column order
    int hlen[2];
    int slot[2];            // value slot of the key in that column position (0 = primary value, 1 = edge count)
    uint8_t lead[2];        // first value byte: 0x00 = the null flag of a typed key; a generic key's
                            // class registration (writePositive(13 / 20 / 12) = 0x8D / 0x94 / 0x8C)
    int64_t rel_base;
};

// Value of slot `k` for internal vertex v; false when the vertex holds no such property.
__device__ inline bool value_of(const ResArgs& a, const void* v0, const void* v1, int64_t v, int k, uint64_t& bits) {
    if (a.kind == TGO_RESULT_DISTANCE) {
        const int64_t d = static_cast<const int64_t*>(v0)[v];
        bits = static_cast<uint64_t>(d);
        return d != TGO_DIST_ABSENT;
    }
    if (a.kind == TGO_RESULT_PAGERANK) {
        const double x = static_cast<const double*>(k == 0 ? v0 : v1)[v];
        bits = static_cast<uint64_t>(__double_as_longlong(x));
        return true;
    }
    if (a.kind == TGO_RESULT_VALUES) {          // v0: 8-byte values, v1: present flags
        bits = static_cast<const uint64_t*>(v0)[v];
        return static_cast<const uint8_t*>(v1)[v] != 0;
    }
    bits = static_cast<uint64_t>(static_cast<int64_t>(static_cast<const int32_t*>(v0)[v]));
    return true;
}

// Integer encodings: DEGREE, or a generic program's Integer key
__device__ inline bool varint_value(const ResArgs& a) {
    return a.kind == TGO_RESULT_DEGREE || (a.kind == TGO_RESULT_VALUES && a.vdt == TGO_DT_INTEGER);
}
__device__ inline int value_len(const ResArgs& a, uint64_t bits) {
    if (varint_value(a)) return 1 + pos_len(zigzag(static_cast<int64_t>(bits)));
    return 9;
}

__global__ void res_count(ResArgs a, const int32_t* perm, const void* v0, const void* v1, int64_t n,
                          int64_t* ecnt, int64_t* rflag) {
    const int64_t r = static_cast<int64_t>(blockIdx.x) * blockDim.x + threadIdx.x;
    if (r > n) return;
    if (r == n) { ecnt[n] = 0; rflag[n] = 0; return; }
    uint64_t bits;
    const bool has = value_of(a, v0, v1, perm[r], 0, bits);
    ecnt[r] = has ? a.nkeys : 0;
    rflag[r] = has ? 1 : 0;
}

__global__ void res_size(ResArgs a, const int32_t* perm, const void* v0, const void* v1, int64_t n,
                         const int64_t* epre, int64_t* bcnt) {
    const int64_t r = static_cast<int64_t>(blockIdx.x) * blockDim.x + threadIdx.x;
    if (r > n) return;
    if (r == n) { bcnt[n] = 0; return; }
    const int64_t e0 = epre[r], ne = epre[r + 1] - e0;
    int64_t bytes = 0;
    for (int64_t j = 0; j < ne; ++j) {
        uint64_t bits;
        value_of(a, v0, v1, perm[r], a.slot[j], bits);
        bytes += a.hlen[j] + value_len(a, bits) + pos_len(static_cast<uint64_t>(a.rel_base + e0 + j));
    }
    bcnt[r] = bytes;
}

__global__ void res_write(ResArgs a, const int32_t* perm, const void* v0, const void* v1, int64_t n,
                          const int64_t* epre, const int64_t* bpre, const int64_t* rpre, int64_t* row_src,
                          int64_t* row_entry_begin, int64_t* row_byte_begin, uint8_t* bytes, int64_t* limval) {
    const int64_t r = static_cast<int64_t>(blockIdx.x) * blockDim.x + threadIdx.x;
    if (r > n) return;
    const int64_t ri = rpre[r];
    if (r == n) { row_entry_begin[ri] = epre[n]; row_byte_begin[ri] = bpre[n]; return; }
    const int64_t e0 = epre[r], ne = epre[r + 1] - e0;
    if (ne == 0) return;
    row_src[ri] = r;
    row_entry_begin[ri] = e0;
    row_byte_begin[ri] = bpre[r];
    uint8_t* const base = bytes + bpre[r];
    uint8_t* p = base;
    for (int64_t j = 0; j < ne; ++j) {
        uint64_t bits;
        value_of(a, v0, v1, perm[r], a.slot[j], bits);
        uint8_t* const ent = p;
        for (int i = 0; i < a.hlen[j]; ++i) *p++ = a.hdr[j][i];
        const int64_t vpos = p - ent;
        *p++ = a.lead[j];                              // null flag (typed key) or value class (generic key)
        if (varint_value(a)) {
            p = put_pos(p, zigzag(static_cast<int64_t>(bits)));
        } else {
            const bool long_bits = a.kind == TGO_RESULT_DISTANCE || (a.kind == TGO_RESULT_VALUES && a.vdt == TGO_DT_LONG);
            const uint64_t be = long_bits ? (bits ^ 0x8000000000000000ULL) : bits;
            for (int i = 7; i >= 0; --i) *p++ = static_cast<uint8_t>(be >> (8 * i));
        }
        p = put_pos(p, static_cast<uint64_t>(a.rel_base + e0 + j));
        limval[e0 + j] = (static_cast<int64_t>(p - base) << 32) | vpos;
    }
}

// IDHandler.writeRelationType (:88-94) for a user property key, direction PROPERTY_DIR: the
// 3-bit prefix 010 then VariableLong.writePositiveWithPrefix(count << 1) (:139-164).
int relation_type_header(int64_t key_id, uint8_t* out) {
    const uint64_t v = static_cast<uint64_t>(key_id >> 6) << 1;
    const int delta = 5;
    auto blen = [](uint64_t x) { return x == 0 ? 1 : 64 - __builtin_clzll(x); };
    uint8_t first = static_cast<uint8_t>(2u << delta);
    int vl = blen(v);
    const int mod = vl % 7;
    uint64_t rest = v;
    if (mod <= delta - 1) {
        const int offset = vl - mod;
        first |= static_cast<uint8_t>(v >> offset);
        rest = offset >= 64 ? v : (v & ((1ULL << offset) - 1));
        vl -= mod;
    } else {
        vl += 7 - mod;
    }
    if (vl > 0) first |= static_cast<uint8_t>(1 << (delta - 1));
    int len = 0;
    out[len++] = first;
    for (int off = vl; off > 0;) {
        off -= 7;
        out[len++] = static_cast<uint8_t>(((rest >> off) & 0x7F) | (off == 0 ? 0x80 : 0));
    }
    return len;
}

}  // namespace

int encode_results(const ResultSource& src, const tgo_result_args* a, const int32_t* perm, int64_t n,
                   int64_t* const scratch[4], void*& cub_tmp, size_t& cub_bytes, ResultRows* out, hipStream_t st,
                   std::string& err) {
    ResArgs ra{};
    ra.kind = a->kind;
    ra.nkeys = a->kind == TGO_RESULT_PAGERANK ? 2 : 1;
    ra.rel_base = a->relation_id_base;
    if (a->kind < TGO_RESULT_DISTANCE || a->kind > TGO_RESULT_VALUES) { err = "unknown result kind"; return TGO_E_INVALID; }
    int want[4][2] = {{TGO_DT_LONG, 0}, {TGO_DT_DOUBLE, TGO_DT_DOUBLE}, {TGO_DT_INTEGER, 0}, {0, 0}};
    // StandardSerializer registration numbers of the value classes (:71-81): Long 13, Double 20, Integer 12
    uint8_t reg[4] = {0x80 | 13, 0x80 | 20, 0x80 | 12, 0};
    if (a->kind == TGO_RESULT_VALUES) {
        // a generic program's key: int64 values as a Long or Integer key (generic: Long),
        // fp64 values as a Double key (generic: Double)
        ra.vtype = a->reserved;
        if (ra.vtype == TGO_VAL_INT64) {
            ra.vdt = a->datatypes[0] == TGO_DT_INTEGER ? TGO_DT_INTEGER : TGO_DT_LONG;
            want[3][0] = a->datatypes[0] == TGO_DT_INTEGER ? TGO_DT_INTEGER : TGO_DT_LONG;
            reg[3] = 0x80 | 13;
        } else if (ra.vtype == TGO_VAL_FP64) {
            ra.vdt = TGO_DT_DOUBLE;
            want[3][0] = TGO_DT_DOUBLE;
            reg[3] = 0x80 | 20;
        } else {
            err = "TGO_RESULT_VALUES needs a value type (args.reserved)";
            return TGO_E_INVALID;
        }
    }
    uint8_t lead[2] = {0, 0};
    for (int k = 0; k < ra.nkeys; ++k) {
        if ((a->key_ids[k] & 63) != 5 || (a->key_ids[k] >> 6) <= 0) { err = "compute key is not a user property key id"; return TGO_E_INVALID; }
        if (a->datatypes[k] == TGO_DT_OBJECT) {
            lead[k] = reg[a->kind];                     // generic key: writeClassAndObject
        } else if (a->datatypes[k] != want[a->kind][k]) {
            err = "compute key datatype must be Long (distance), Double (pageRank, edgeCount), Integer (degree) "
                  "or generic (Object)";
            return TGO_E_UNSUPPORTED;
        }
    }
    if (ra.nkeys == 2 && a->key_ids[0] == a->key_ids[1]) { err = "pageRank and edgeCount keys must differ"; return TGO_E_INVALID; }
    if (a->relation_id_base <= 0) { err = "relation_id_base must be positive"; return TGO_E_INVALID; }
    // column order = byte order of the headers
    uint8_t h[2][12];
    int hl[2];
    for (int k = 0; k < ra.nkeys; ++k) hl[k] = relation_type_header(a->key_ids[k], h[k]);
    int order[2] = {0, 1};
    if (ra.nkeys == 2) {
        const int c = std::memcmp(h[0], h[1], std::min(hl[0], hl[1]));
        if (c > 0 || (c == 0 && hl[0] > hl[1])) std::swap(order[0], order[1]);
    }
    for (int j = 0; j < ra.nkeys; ++j) {
        std::memcpy(ra.hdr[j], h[order[j]], 12);
        ra.hlen[j] = hl[order[j]];
        ra.slot[j] = order[j];
        ra.lead[j] = lead[order[j]];
    }
    // scratch: A = row flags, B = their scan (output row index), C = entries per row then
    // byte sizes, D = entry scan; byte scan into A (free once B holds the row scan)
    int64_t* const rflag = scratch[0];
    int64_t* const rpre = scratch[1];
    int64_t* const cnt = scratch[2];
    int64_t* const epre = scratch[3];
    int64_t* const bpre = scratch[0];
    // pass 1: entries and row flags, scanned
    res_count<<<grid_for(n + 1), kBlock, 0, st>>>(ra, perm, src.v0, src.v1, n, cnt, rflag);
    hipError_t e = hipGetLastError();
    if (e == hipSuccess) e = scan_exclusive_i64(cub_tmp, cub_bytes, rflag, rpre, n + 1, st);
    if (e == hipSuccess) e = scan_exclusive_i64(cub_tmp, cub_bytes, cnt, epre, n + 1, st);
    if (e != hipSuccess) { err = hipGetErrorString(e); return TGO_E_HIP; }
    // pass 2: byte sizes (relation ids depend on the entry index), scanned
    res_size<<<grid_for(n + 1), kBlock, 0, st>>>(ra, perm, src.v0, src.v1, n, epre, cnt);
    e = hipGetLastError();
    if (e == hipSuccess) e = scan_exclusive_i64(cub_tmp, cub_bytes, cnt, bpre, n + 1, st);
    int64_t tot[3] = {0, 0, 0};
    if (e == hipSuccess) e = hipMemcpyAsync(&tot[0], rpre + n, 8, hipMemcpyDeviceToHost, st);
    if (e == hipSuccess) e = hipMemcpyAsync(&tot[1], epre + n, 8, hipMemcpyDeviceToHost, st);
    if (e == hipSuccess) e = hipMemcpyAsync(&tot[2], bpre + n, 8, hipMemcpyDeviceToHost, st);
    if (e == hipSuccess) e = hipStreamSynchronize(st);
    if (e != hipSuccess) { err = hipGetErrorString(e); return TGO_E_HIP; }
    out->nrows = tot[0];
    out->nentries = tot[1];
    out->nbytes = tot[2];
    if (!out->write) return TGO_OK;
    // pass 3: write into device buffers, then copy to the caller
    int64_t *d_src = nullptr, *d_eb = nullptr, *d_bb = nullptr, *d_lv = nullptr;
    uint8_t* d_bytes = nullptr;
    auto cleanup = [&] {
        if (d_src) (void)hipFree(d_src);
        if (d_eb) (void)hipFree(d_eb);
        if (d_bb) (void)hipFree(d_bb);
        if (d_lv) (void)hipFree(d_lv);
        if (d_bytes) (void)hipFree(d_bytes);
    };
    const int64_t nr = tot[0], ne = tot[1], nb = tot[2];
    e = hipMalloc(&d_src, std::max<int64_t>(1, nr) * 8);
    if (e == hipSuccess) e = hipMalloc(&d_eb, (nr + 1) * 8);
    if (e == hipSuccess) e = hipMalloc(&d_bb, (nr + 1) * 8);
    if (e == hipSuccess) e = hipMalloc(&d_lv, std::max<int64_t>(1, ne) * 8);
    if (e == hipSuccess) e = hipMalloc(&d_bytes, std::max<int64_t>(1, nb));
    if (e != hipSuccess) { cleanup(); err = "out of device memory for result rows"; return TGO_E_OOM; }
    res_write<<<grid_for(n + 1), kBlock, 0, st>>>(ra, perm, src.v0, src.v1, n, epre, bpre, rpre, d_src, d_eb, d_bb,
                                                  d_bytes, d_lv);
    e = hipGetLastError();
    if (e == hipSuccess && nr) e = hipMemcpyAsync(out->row_src, d_src, nr * 8, hipMemcpyDeviceToHost, st);
    if (e == hipSuccess) e = hipMemcpyAsync(out->row_entry_begin, d_eb, (nr + 1) * 8, hipMemcpyDeviceToHost, st);
    if (e == hipSuccess) e = hipMemcpyAsync(out->row_byte_begin, d_bb, (nr + 1) * 8, hipMemcpyDeviceToHost, st);
    if (e == hipSuccess && ne) e = hipMemcpyAsync(out->entry_limit_valpos, d_lv, ne * 8, hipMemcpyDeviceToHost, st);
    if (e == hipSuccess && nb) e = hipMemcpyAsync(out->entry_bytes, d_bytes, nb, hipMemcpyDeviceToHost, st);
    if (e == hipSuccess) e = hipStreamSynchronize(st);
    cleanup();
    if (e != hipSuccess) { err = hipGetErrorString(e); return TGO_E_HIP; }
    return TGO_OK;
}

}  // namespace tgo

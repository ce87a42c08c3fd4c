// synth_rows.cpp — synthetic Titan edgestore rows for the bench and the parity tests
// (include/tgo_synth.h).  It stands in for the Java host's edgestore scan: the rows a
// StandardScanner hands to VertexJobConverter.process for a graph written by Titan's commit
// path, byte for byte, so tgo_load_rows decodes what a real scan would deliver.
//
// Per vertex i (id = IDManager.constructId(count = i / 2^pb + 1, partition = i % 2^pb),
// IDManager.java:428-437) one row keyed by IDManager.getKey (:461-473) holding, in column
// byte order (StaticArrayBuffer.compareTo, StaticArrayBuffer.java:381-393):
//   * the VertexExists system property (BaseKey.java:27-28, StandardTitanTx.java:509):
//     column [0x02], value [0x00 0x01] + relation id;
//   * one OUT entry per out-edge and one IN entry per in-edge of the MULTI label
//     (StandardTitanGraph.java:564-591; a self-loop gives both on one row):
//     column [type|dir prefix varint][other id backward][relation id backward], value = the
//     optional Integer signature property (EdgeSerializer.writeRelation :222-315).
// Relation ids: VertexExists of vertex i = 1001 + i, edge k = 1001 + n + k (the numbering of
// tests/edgestore.py, so both writers agree byte for byte).  Rows come in unsigned key order,
// as an ordered scan returns them; the entry list is StaticArrayEntryList's
// (limit << 32 | valuePos) layout (StaticArrayEntryList.java:15-50).
//
// Written independently of oracle/ (the checker): tests compare the two writers' bytes.
#include <algorithm>
#include <cstring>
#include <thread>
#include <vector>
#include "../../include/tgo_synth.h"
#include "../../include/titan_gpu_olap.h"

namespace {

inline int bit_len(uint64_t v) { return v == 0 ? 1 : 64 - __builtin_clzll(v); }

// VariableLong.writePositive (VariableLong.java:84-87): 7-bit groups MSB first, the stop
// bit (0x80) on the LAST byte.
inline int pos_len(uint64_t v) { return (bit_len(v) - 1) / 7 + 1; }
inline uint8_t* put_pos(uint8_t* p, uint64_t v) {
    for (int i = pos_len(v) - 1; i >= 0; --i) *p++ = static_cast<uint8_t>(((v >> (7 * i)) & 0x7F) | (i == 0 ? 0x80 : 0));
    return p;
}
// VariableLong.writePositiveBackward (:234-252): >= 3 bytes, the FIRST byte carries the stop
// marker, the extra-length field (bits 4-6) and the top 4 value bits.
inline int back_len(uint64_t v) {
    const int bl = bit_len(v);
    const int nb = 1 + (bl <= 4 ? 0 : 1 + (bl - 5) / 7);
    return nb < 3 ? 3 : nb;
}
inline uint8_t* put_back(uint8_t* p, uint64_t v) {
    const int nb = back_len(v);
    uint8_t x = static_cast<uint8_t>(((nb - 3) << 4) | 0x80);
    for (int i = nb - 1; i >= 0; --i) {
        x |= static_cast<uint8_t>((v >> (7 * i)) & 0x7F);
        *p++ = x;
        x = 0;
    }
    return p;
}
// VariableLong.writePositiveWithPrefix (:139-164) with a 3-bit prefix (IDHandler.writeRelationType
// :88-94): the first byte holds the prefix, a continue flag and the value's top bits.
inline int prefixed_len(uint64_t v) {
    const int delta = 5, mod = bit_len(v) % 7;
    int vl = bit_len(v);
    if (mod <= delta - 1) vl -= mod; else vl += 7 - mod;
    return 1 + (vl > 0 ? vl / 7 : 0);
}
inline uint8_t* put_prefixed(uint8_t* p, uint64_t v, unsigned prefix) {
    const int delta = 5;
    uint8_t first = static_cast<uint8_t>(prefix << delta);
    int vl = bit_len(v);
    const int mod = vl % 7;
    if (mod <= delta - 1) {
        const int offset = vl - mod;
        first |= static_cast<uint8_t>(v >> offset);
        v = offset >= 64 ? v : (v & ((1ULL << offset) - 1));
        vl -= mod;
    } else {
        vl += 7 - mod;
    }
    if (vl > 0) first |= static_cast<uint8_t>(1 << (delta - 1));
    *p++ = first;
    for (int off = vl; off > 0;) {
        off -= 7;
        *p++ = static_cast<uint8_t>(((v >> off) & 0x7F) | (off == 0 ? 0x80 : 0));
    }
    return p;
}
// IntegerSerializer (IntegerSerializer.java:14-23) behind StandardSerializer's null flag
// (StandardSerializer.java:220-233): 0x00 then the zig-zag VariableLong.
inline uint64_t zigzag(int64_t v) { return v < 0 ? ((static_cast<uint64_t>(-v) << 1) | 1) : (static_cast<uint64_t>(v) << 1); }

struct Plan {
    int64_t n, m;
    int pb;
    uint64_t label_count;          // schema id >> 6
    bool weighted;
};
inline uint64_t vertex_id(int64_t i, int pb) {
    return (((static_cast<uint64_t>(i >> pb) + 1) << pb) + static_cast<uint64_t>(i & ((int64_t(1) << pb) - 1))) << 3;
}
inline int64_t row_key(int64_t i, int pb) {   // IDManager.getKey: partition in the top pb bits
    const uint64_t part = static_cast<uint64_t>(i & ((int64_t(1) << pb) - 1));
    const uint64_t count = static_cast<uint64_t>(i >> pb) + 1;
    return static_cast<int64_t>((pb ? part << (64 - pb) : 0) | (count << 3));
}
inline int edge_entry_len(const Plan& P, int dir, int64_t other, int64_t rel, int32_t w) {
    int len = prefixed_len((P.label_count << 1) | static_cast<uint64_t>(dir)) + back_len(vertex_id(other, P.pb)) +
              back_len(static_cast<uint64_t>(rel));
    if (P.weighted) len += 1 + pos_len(zigzag(w));
    return len;
}
inline int exists_len(int64_t rel) { return 3 + pos_len(static_cast<uint64_t>(rel)); }

// f(lo, hi, t) over [0, n) split into `threads` contiguous ranges.
template <class F>
void parallel(int threads, int64_t n, F f) {
    std::vector<std::thread> th;
    for (int t = 0; t < threads; ++t) th.emplace_back([=] { f(n * t / threads, n * (t + 1) / threads, t); });
    for (auto& x : th) x.join();
}

}  // namespace

extern "C" int tgo_synth_rows(int64_t n, int64_t m, const int32_t* src, const int32_t* dst, const int32_t* weight,
                              int64_t label_id, int32_t partition_bits, int32_t threads, int64_t* sizes_out,
                              int64_t* row_keys, int64_t* row_entry_begin, int64_t* row_byte_begin,
                              uint8_t* entry_bytes, int64_t* entry_limit_valpos) {
    if (n <= 0 || m < 0 || (m > 0 && (!src || !dst)) || !sizes_out || partition_bits < 0 || partition_bits > 16 ||
        (label_id & 63) != 21 || (label_id >> 6) <= 0)
        return TGO_E_INVALID;
    if (threads <= 0) threads = static_cast<int>(std::thread::hardware_concurrency());
    threads = std::max(1, std::min(threads, 64));
    const Plan P{n, m, partition_bits, static_cast<uint64_t>(label_id >> 6), weight != nullptr};
    for (int64_t k = 0; k < m; ++k)
        if (src[k] < 0 || src[k] >= n || dst[k] < 0 || dst[k] >= n) return TGO_E_INVALID;
    // sizes: every edge k writes an OUT entry on row src[k] and an IN entry on row dst[k]
    std::vector<int64_t> part(threads, 0);
    parallel(threads, m, [&](int64_t lo, int64_t hi, int t) {
        int64_t s = 0;
        for (int64_t k = lo; k < hi; ++k) {
            const int64_t rel = 1001 + n + k;
            const int32_t w = weight ? weight[k] : 0;
            s += edge_entry_len(P, 0, dst[k], rel, w) + edge_entry_len(P, 1, src[k], rel, w);
        }
        part[t] = s;
    });
    int64_t nbytes = 0;
    for (int64_t v = 0; v < n; ++v) nbytes += exists_len(1001 + v);
    for (int64_t x : part) nbytes += x;
    sizes_out[0] = n;
    sizes_out[1] = n + 2 * m;
    sizes_out[2] = nbytes;
    if (!row_keys || !row_entry_begin || !row_byte_begin || !entry_bytes || !entry_limit_valpos) return TGO_OK;

    // Per-vertex OUT lists sorted by (other, edge) and IN lists sorted by (other, edge): a
    // stable counting sort by the neighbour, then a stable scatter to the owner.
    std::vector<int64_t> ooff(n + 1, 0), ioff(n + 1, 0);
    for (int64_t k = 0; k < m; ++k) { ++ooff[src[k] + 1]; ++ioff[dst[k] + 1]; }
    for (int64_t v = 0; v < n; ++v) { ooff[v + 1] += ooff[v]; ioff[v + 1] += ioff[v]; }
    std::vector<int64_t> olist(m), ilist(m);   // edge indices
    {
        std::vector<int64_t> by(m), b(n + 1, 0), cur(n);
        for (int pass = 0; pass < 2; ++pass) {
            const int32_t* key = pass == 0 ? dst : src;
            const int32_t* own = pass == 0 ? src : dst;
            std::fill(b.begin(), b.end(), 0);
            for (int64_t k = 0; k < m; ++k) ++b[key[k] + 1];
            for (int64_t v = 0; v < n; ++v) b[v + 1] += b[v];
            for (int64_t k = 0; k < m; ++k) by[b[key[k]]++] = k;
            const std::vector<int64_t>& off = pass == 0 ? ooff : ioff;
            std::vector<int64_t>& list = pass == 0 ? olist : ilist;
            for (int64_t v = 0; v < n; ++v) cur[v] = off[v];
            for (int64_t j = 0; j < m; ++j) { const int64_t k = by[j]; list[cur[own[k]]++] = k; }
        }
    }
    // Row order = unsigned key order = (partition, count).
    const int64_t parts = int64_t(1) << partition_bits;
    std::vector<int64_t> order;
    order.reserve(n);
    for (int64_t p = 0; p < parts && p < n; ++p)
        for (int64_t i = p; i < n; i += parts) order.push_back(i);
    std::vector<int64_t> rbytes(n + 1, 0);
    parallel(threads, n, [&](int64_t lo, int64_t hi, int) {
        for (int64_t r = lo; r < hi; ++r) {
            const int64_t v = order[r];
            int64_t s = exists_len(1001 + v);
            for (int64_t j = ooff[v]; j < ooff[v + 1]; ++j) {
                const int64_t k = olist[j];
                s += edge_entry_len(P, 0, dst[k], 1001 + n + k, weight ? weight[k] : 0);
            }
            for (int64_t j = ioff[v]; j < ioff[v + 1]; ++j) {
                const int64_t k = ilist[j];
                s += edge_entry_len(P, 1, src[k], 1001 + n + k, weight ? weight[k] : 0);
            }
            rbytes[r + 1] = s;
        }
    });
    row_byte_begin[0] = 0;
    row_entry_begin[0] = 0;
    for (int64_t r = 0; r < n; ++r) {
        const int64_t v = order[r];
        row_byte_begin[r + 1] = row_byte_begin[r] + rbytes[r + 1];
        row_entry_begin[r + 1] = row_entry_begin[r] + 1 + (ooff[v + 1] - ooff[v]) + (ioff[v + 1] - ioff[v]);
        row_keys[r] = row_key(v, partition_bits);
    }
    parallel(threads, n, [&](int64_t lo, int64_t hi, int) {
        for (int64_t r = lo; r < hi; ++r) {
            const int64_t v = order[r];
            uint8_t* const base = entry_bytes + row_byte_begin[r];
            uint8_t* p = base;
            int64_t e = row_entry_begin[r];
            auto close = [&](int64_t vpos) { entry_limit_valpos[e++] = (static_cast<int64_t>(p - base) << 32) | vpos; };
            {   // VertexExists: column 0x02, valuePos 1, value = true, then the relation id
                *p++ = 0x02;
                *p++ = 0x00;
                *p++ = 0x01;
                p = put_pos(p, static_cast<uint64_t>(1001 + v));
                close(1);
            }
            for (int dir = 0; dir < 2; ++dir) {
                const std::vector<int64_t>& off = dir == 0 ? ooff : ioff;
                const std::vector<int64_t>& list = dir == 0 ? olist : ilist;
                for (int64_t j = off[v]; j < off[v + 1]; ++j) {
                    const int64_t k = list[j];
                    const int64_t other = dir == 0 ? dst[k] : src[k];
                    uint8_t* s = p;
                    p = put_prefixed(p, (P.label_count << 1) | static_cast<uint64_t>(dir), 3);   // user edge: prefix 011b
                    p = put_back(p, vertex_id(other, partition_bits));
                    p = put_back(p, static_cast<uint64_t>(1001 + n + k));
                    const int64_t vpos = p - s;
                    if (weight) {
                        *p++ = 0x00;
                        p = put_pos(p, zigzag(weight[k]));
                    }
                    close(vpos);
                }
            }
        }
    });
    return TGO_OK;
}

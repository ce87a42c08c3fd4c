// codec.hpp — product-side edgestore decoder, used by the CSR assembler (host) and the
// device row decoder (decode.hip).
//
// Decodes the bytes Titan's edgestore holds for one vertex row into the adjacency the
// OLAP programs read.  Restates (independently of oracle/, which is the checker):
//   VariableLong           graphdb/database/idhandling/VariableLong.java:30-38,171-186,254-272,129-131
//   IDHandler              graphdb/database/idhandling/IDHandler.java:116-127,135-143,158-179
//   IDManager key <-> id   graphdb/idmanagement/IDManager.java:428-437,461-486
//   EdgeSerializer         graphdb/database/EdgeSerializer.java:73-166
//   StandardSerializer     graphdb/database/serialize/StandardSerializer.java:220-233 and the
//                          attribute serializers (serialize/attribute/*Serializer.java)
// All paths relative to titan-core/src/main/java/com/thinkaurelius/titan/.
#pragma once
#include <cstdint>
#include <cstddef>
#include "../../include/titan_gpu_olap.h"

// Functions below run on the host (graph_build.cpp) and inside the device decode kernel
// (decode.hip, which defines TGO_HD as __host__ __device__ before including this file).
#ifndef TGO_HD
#define TGO_HD
#endif

namespace tgo {

// Schema ids: (count << 6) | suffix for relation types (IDManager.VertexIDType :209-300).
constexpr int64_t kSuffixUserPropertyKey = 5, kSuffixSystemPropertyKey = 37;
constexpr int64_t kSuffixUserEdgeLabel = 21, kSuffixSystemEdgeLabel = 53;
constexpr int64_t kVertexExistsId = (1LL << 6) | kSuffixSystemPropertyKey;  // BaseKey.java:27-28

// Bounds-checked forward/backward byte cursor over one entry.  `x` is XORed into every byte
// read: 0xFF reads a DESC sort key, whose bytes the writer inverted (EdgeSerializer.java:137,
// 311-313; WriteByteBuffer.getStaticBufferFlipBytes).
struct Cursor {
    const uint8_t* d;
    size_t n;
    size_t pos;
    bool bad = false;
    uint8_t x = 0;
    TGO_HD inline uint8_t get() {
        if (pos >= n) { bad = true; return 0x80; }
        return static_cast<uint8_t>(d[pos++] ^ x);
    }
    // VariableLong.readUnsigned: 7-bit groups, MSB first, stop bit on the last byte.
    TGO_HD inline uint64_t varint() {
        uint64_t v = 0;
        for (int i = 0; i < 10; ++i) {
            uint8_t b = get();
            v = (v << 7) | (b & 0x7Fu);
            if (b & 0x80u) return v;
        }
        bad = true;
        return 0;
    }
    // VariableLong.read: zig-zag (abs<<1 | sign).
    TGO_HD inline int64_t svarint() {
        uint64_t u = varint();
        return (u & 1) ? -static_cast<int64_t>(u >> 1) : static_cast<int64_t>(u >> 1);
    }
    // VariableLong.readPositiveBackward: from `pos` (one past the last byte) towards the
    // first byte, which carries the stop marker (bit 7) and a 4-bit head.
    TGO_HD inline uint64_t varint_backward() {
        uint64_t v = 0;
        int shift = 0;
        for (int i = 0; i < 10; ++i) {
            if (pos == 0) { bad = true; return 0; }
            uint8_t b = d[--pos];
            if (b & 0x80u) return v | (static_cast<uint64_t>(b & 0x0Fu) << shift);
            v |= static_cast<uint64_t>(b) << shift;
            shift += 7;
        }
        bad = true;
        return 0;
    }
    TGO_HD inline uint64_t be(int nbytes) {
        uint64_t v = 0;
        for (int i = 0; i < nbytes; ++i) v = (v << 8) | get();
        return v;
    }
    TGO_HD inline void skip(uint64_t nbytes) {
        if (nbytes > n - (pos < n ? pos : n)) { bad = true; pos = n; return; }
        pos += static_cast<size_t>(nbytes);
    }
};

struct RelType {
    int64_t type_id;
    bool is_edge;
    int dir;  // 0 = OUT (or property), 1 = IN
};

// IDHandler.readRelationType: 3-bit prefix [system/invisible(2) | is-edge(1)] followed by
// the prefixed varint (typeCount << 1 | dir) (VariableLong.readPositiveWithPrefix).
TGO_HD inline bool read_relation_type(Cursor& c, RelType& rt) {
    const uint8_t first = c.get();
    const int prefix = first >> 5;
    uint64_t v = first & 0x0Fu;
    if (first & 0x10u) {                 // continue mask
        const size_t p0 = c.pos;
        const uint64_t rem = c.varint();
        v = (v << (7 * (c.pos - p0))) + rem;
    }
    const int is_edge = prefix & 1;
    const int dir = static_cast<int>(v & 1);
    if (!is_edge && dir) return false;   // DirectionID.forId(1) is invalid
    const bool system = (prefix >> 1) == 0;
    const int64_t count = static_cast<int64_t>(v >> 1);
    if (count <= 0 || c.bad) return false;
    const int64_t sfx = is_edge ? (system ? kSuffixSystemEdgeLabel : kSuffixUserEdgeLabel)
                                : (system ? kSuffixSystemPropertyKey : kSuffixUserPropertyKey);
    rt.type_id = (count << 6) | sfx;
    rt.is_edge = is_edge != 0;
    rt.dir = dir;
    return true;
}

// IDManager.getKeyID for a row key; partition bits pb.
TGO_HD inline int64_t key_to_vertex_id(int64_t key, int pb) {
    const uint64_t k = static_cast<uint64_t>(key);
    if ((k & 3u) == 1u) return key;      // schema vertex: key is the id
    const int poff = 64 - pb;
    const uint64_t partition = poff < 64 ? (k >> poff) : 0;
    const uint64_t count = (k >> 3) & ((1ULL << (poff - 3)) - 1);
    return static_cast<int64_t>((((count << pb) + partition) << 3) | (k & 7u));
}

// Vertex cuts (VertexIDType.PartitionedVertex, suffix 010b, IDManager.java:78-90).
TGO_HD inline bool is_partitioned_vertex(int64_t vid, int pb) {            // isPartitionedVertex :557-559
    return (vid & 7) == 2 && (static_cast<uint64_t>(vid) >> (pb + 3)) > 0;
}
// getCanonicalVertexId (:530-534): the representative in partition getPartitionHashForId(count)
// (:512-523, XOR of the count's pb-bit chunks).
TGO_HD inline int64_t canonical_vertex_id(int64_t vid, int pb) {
    if (pb <= 0) return vid;
    const uint64_t count = static_cast<uint64_t>(vid) >> (pb + 3);
    uint64_t part = 0;
    for (int off = 0; off < 64; off += pb) part ^= (count >> off) & ((1ULL << pb) - 1);
    return static_cast<int64_t>((((count << pb) + part) << 3) | 2u);
}

TGO_HD inline bool unique_in(int mult, int dir) {  // Multiplicity.isUnique
    return dir == 1 ? (mult == TGO_ONE2MANY || mult == TGO_ONE2ONE)
                    : (mult == TGO_MANY2ONE || mult == TGO_ONE2ONE);
}

// Reads (or skips) one inline value through StandardSerializer (readObjectInternal :220-233):
// a null flag byte unless the serializer handles null itself (StringSerializer), then the
// attribute serializer's read, or readByteOrder for a sort key (byte_order).  Integral values
// (Byte..Long, Boolean, Date, Character) are returned in v, a Float as its IEEE bits (int32);
// String is skipped; Double gives its IEEE bits.
// Returns false on a codec error; present=false for a serialized null.
TGO_HD inline bool read_value(Cursor& c, int dt, bool byte_order, bool& present, int64_t& v) {
    v = 0;
    if (dt == TGO_DT_STRING) {
        if (byte_order) {                          // StringSerializer.readByteOrder :40-51
            const uint8_t p = c.get();
            if (p == 0xFF) { present = false; return !c.bad; }
            if (p != 0) return false;
            present = true;
            for (;;) {                             // 2-byte chars up to (char) 0
                const uint64_t ch = c.be(2);
                if (c.bad) return false;
                if (ch == 0) return true;
            }
        }
        uint64_t len = c.varint();                 // StringSerializer.read :84-135
        if (c.bad) return false;
        if (len == 0) { present = false; return true; }
        present = true;
        const uint64_t cid = len & 7;
        len >>= 3;
        if (cid != 0) { c.skip(len); return !c.bad; }       // compressed: len bytes
        if ((len & 1) == 0) {                      // ASCII: "" or bytes up to the 0x80 marker
            len >>= 1;
            if (len == 1) return true;
            if (len != 2) return false;
            while (!(c.get() & 0x80u)) if (c.bad) return false;
            return !c.bad;
        }
        for (uint64_t i = 0, nch = len >> 1; i < nch; ++i) {   // full UTF, 1-3 bytes per char
            const uint8_t b = c.get();
            if ((b >> 4) == 12 || (b >> 4) == 13) c.get();
            else if ((b >> 4) == 14) { c.get(); c.get(); }
            if (c.bad) return false;
        }
        return true;
    }
    const uint8_t flag = c.get();
    if (flag == 0xFF) { present = false; return !c.bad; }
    if (flag != 0) return false;
    present = true;
    switch (dt) {
        case TGO_DT_BYTE: v = static_cast<int8_t>(c.get() - 128); break;
        case TGO_DT_SHORT: v = static_cast<int16_t>(c.be(2) - 32768); break;
        case TGO_DT_CHARACTER: v = static_cast<int64_t>(c.be(2)); break;
        case TGO_DT_INTEGER:
            if (byte_order) {
                v = static_cast<int32_t>(static_cast<uint32_t>(c.be(4)) + 0x80000000u);
            } else {
                const int64_t l = c.svarint();
                if (l < INT32_MIN || l > INT32_MAX) return false;
                v = l;
            }
            break;
        case TGO_DT_LONG:
        case TGO_DT_DATE: v = static_cast<int64_t>(c.be(8) + 0x8000000000000000ULL); break;
        case TGO_DT_FLOAT: {                       // FloatSerializer :33-46: the IEEE bits, or
            uint32_t u = static_cast<uint32_t>(c.be(4));    // NumericUtils.floatToSortableInt ^ sign
            if (byte_order) {
                u ^= 0x80000000u;
                int32_t si = static_cast<int32_t>(u);
                si ^= (si >> 31) & 0x7fffffff;
                u = static_cast<uint32_t>(si);
            }
            if (u == 0x80000000u) u = 0;           // -0.0f reads as +0.0f (the bits of -0.0f are the
                                                   // missing-weight sentinel INT32_MIN)
            v = static_cast<int32_t>(u);
            break;
        }
        case TGO_DT_DOUBLE: {                      // DoubleSerializer :25-41: the IEEE bits, or
            uint64_t u = c.be(8);                  // NumericUtils.doubleToSortableLong ^ sign
            if (byte_order) {
                int64_t sl = static_cast<int64_t>(u ^ 0x8000000000000000ULL);
                sl ^= (sl >> 63) & 0x7fffffffffffffffLL;
                u = static_cast<uint64_t>(sl);
            }
            v = static_cast<int64_t>(u);
            break;
        }
        case TGO_DT_BOOLEAN: v = c.get(); break;
        default: return false;
    }
    return !c.bad;
}

// Per-edge-label decode plan derived from tgo_schema: a flat, pointer-free record so the same
// decode runs on the host and in a device kernel.  Datatypes of sort-key and signature keys
// live in one shared byte array (dt_off .. + n_sort / n_sig).
enum : int32_t { kWeightNone = 0, kWeightSortKey = 1, kWeightSignature = 2, kWeightRemaining = 3 };
struct LabelPlan {
    int64_t type_id;
    int32_t multiplicity;
    int32_t selected;        // passes the scope's label filter
    int32_t desc;            // sort order DESC: key bytes inverted
    int32_t weight_where;    // kWeight*
    int32_t weight_index;    // index in the sort key / signature
    int32_t n_sort, n_sig;
    int32_t sort_dt_off, sig_dt_off;
};
struct PlanView {
    const LabelPlan* labels;   // sorted by type_id
    int32_t n_labels;
    int32_t n_keys;
    const int64_t* key_ids;    // property keys (for remaining properties), sorted
    const int8_t* key_dts;
    const int8_t* dts;         // sort-key / signature datatypes
    int64_t weight_key;
    TGO_HD const LabelPlan* find(int64_t id) const {
        int32_t lo = 0, hi = n_labels;
        while (lo < hi) {
            const int32_t mid = (lo + hi) / 2;
            if (labels[mid].type_id < id) lo = mid + 1; else hi = mid;
        }
        return lo < n_labels && labels[lo].type_id == id ? &labels[lo] : nullptr;
    }
    TGO_HD int datatype(int64_t key) const {
        int32_t lo = 0, hi = n_keys;
        while (lo < hi) {
            const int32_t mid = (lo + hi) / 2;
            if (key_ids[mid] < key) lo = mid + 1; else hi = mid;
        }
        return lo < n_keys && key_ids[lo] == key ? key_dts[lo] : 0;
    }
};

struct DecodedEdge {
    int64_t type_id;
    int dir;
    int64_t other;
    bool has_weight;
    int32_t weight;          // 32-bit weight keys (Float: the IEEE bits)
    int64_t weight64;        // the same value in 64 bits (Long: the value, Double: the IEEE bits)
};

enum class DecodeResult { kOk, kSkip, kError, kUnsupported };

// EdgeSerializer.parseRelation (:73-166) restricted to what the traversal needs: direction,
// other vertex id and (optionally) the Integer weight property, wherever it is stored: the
// sort key (MULTI labels, read byte-ordered from the key start, inverted when DESC, :130-140),
// the signature (:143-144) or the remaining properties (:147-152).
TGO_HD inline DecodeResult decode_edge(const uint8_t* d, size_t len, size_t value_pos,
                                       const PlanView& plan, DecodedEdge& out) {
    Cursor c{d, len, 0};
    RelType rt;
    if (value_pos > len || !read_relation_type(c, rt) || !rt.is_edge) return DecodeResult::kError;
    const LabelPlan* lp = plan.find(rt.type_id);
    if (!lp) return DecodeResult::kError;            // tx.getExistingRelationType fails
    if (!lp->selected) return DecodeResult::kSkip;
    out.type_id = rt.type_id;
    out.dir = rt.dir;
    const size_t key_start = c.pos;
    size_t props;
    if (lp->multiplicity != TGO_MULTI) {
        if (unique_in(lp->multiplicity, rt.dir)) {
            out.other = static_cast<int64_t>(c.varint());
        } else {
            Cursor b{d, len, value_pos};
            out.other = static_cast<int64_t>(b.varint_backward());
            if (b.bad) return DecodeResult::kError;
            c.pos = value_pos;
        }
        c.varint();                                   // relation id
        props = c.pos;
    } else {
        Cursor b{d, len, value_pos};
        b.varint_backward();                          // relation id
        out.other = static_cast<int64_t>(b.varint_backward());
        if (b.bad) return DecodeResult::kError;
        props = value_pos;
    }
    if (c.bad) return DecodeResult::kError;
    out.has_weight = false;
    out.weight = 0;
    out.weight64 = 0;
    if (plan.weight_key == 0 || lp->weight_where == kWeightNone) return DecodeResult::kOk;
    bool present; int64_t v = 0;
    if (lp->weight_where == kWeightSortKey) {
        Cursor k{d, value_pos, key_start};
        k.x = lp->desc ? 0xFF : 0x00;
        for (int32_t i = 0; i <= lp->weight_index; ++i)
            if (!read_value(k, plan.dts[lp->sort_dt_off + i], true, present, v)) return DecodeResult::kError;
        out.has_weight = present;
        out.weight = static_cast<int32_t>(v);
        out.weight64 = v;
        return DecodeResult::kOk;
    }
    c.pos = props;
    for (int32_t k = 0; k < lp->n_sig; ++k) {
        if (!read_value(c, plan.dts[lp->sig_dt_off + k], false, present, v)) return DecodeResult::kError;
        if (k == lp->weight_index && lp->weight_where == kWeightSignature) {
            out.has_weight = present;
            out.weight = static_cast<int32_t>(v);
            out.weight64 = v;
            return DecodeResult::kOk;
        }
    }
    while (c.pos < len) {                             // remaining properties, sorted by key id
        const int64_t kid = static_cast<int64_t>((c.varint() << 4) | 5u);
        const int dt = plan.datatype(kid);
        if (dt == 0) return DecodeResult::kUnsupported;
        if (!read_value(c, dt, false, present, v)) return DecodeResult::kError;
        if (kid == plan.weight_key) {
            out.has_weight = present;
            out.weight = static_cast<int32_t>(v);
            out.weight64 = v;
            return DecodeResult::kOk;
        }
    }
    return DecodeResult::kOk;
}

}  // namespace tgo

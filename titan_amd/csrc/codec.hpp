// codec.hpp — product-side edgestore decoder (host C++), used by the CSR assembler.
//
// Decodes the bytes Titan's edgestore holds for one vertex row into the adjacency the
// OLAP programs read.  Restates (independently of oracle/, which is the checker):
//   VariableLong           graphdb/database/idhandling/VariableLong.java:30-38,171-186,254-272,129-131
//   IDHandler              graphdb/database/idhandling/IDHandler.java:116-127,135-143,158-179
//   IDManager key <-> id   graphdb/idmanagement/IDManager.java:428-437,461-486
//   EdgeSerializer         graphdb/database/EdgeSerializer.java:73-166
//   StandardSerializer     graphdb/database/serialize/StandardSerializer.java:220-233
// All paths relative to titan-core/src/main/java/com/thinkaurelius/titan/.
#pragma once
#include <cstdint>
#include <cstddef>
#include <vector>
#include "../../include/titan_gpu_olap.h"

namespace tgo {

// Schema ids: (count << 6) | suffix for relation types (IDManager.VertexIDType :209-300).
constexpr int64_t kSuffixUserPropertyKey = 5, kSuffixSystemPropertyKey = 37;
constexpr int64_t kSuffixUserEdgeLabel = 21, kSuffixSystemEdgeLabel = 53;
constexpr int64_t kVertexExistsId = (1LL << 6) | kSuffixSystemPropertyKey;  // BaseKey.java:27-28

// Bounds-checked forward/backward byte cursor over one entry.
struct Cursor {
    const uint8_t* d;
    size_t n;
    size_t pos;
    bool bad = false;
    inline uint8_t get() {
        if (pos >= n) { bad = true; return 0x80; }
        return d[pos++];
    }
    inline uint8_t at(size_t i) {
        if (i >= n) { bad = true; return 0x80; }
        return d[i];
    }
    // VariableLong.readUnsigned: 7-bit groups, MSB first, stop bit on the last byte.
    inline uint64_t varint() {
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
    inline int64_t svarint() {
        uint64_t u = varint();
        return (u & 1) ? -static_cast<int64_t>(u >> 1) : static_cast<int64_t>(u >> 1);
    }
    // VariableLong.readPositiveBackward: from `pos` (one past the last byte) towards the
    // first byte, which carries the stop marker (bit 7) and a 4-bit head.
    inline uint64_t varint_backward() {
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
    inline uint64_t be(int nbytes) {
        uint64_t v = 0;
        for (int i = 0; i < nbytes; ++i) v = (v << 8) | get();
        return v;
    }
};

struct RelType {
    int64_t type_id;
    bool is_edge;
    int dir;  // 0 = OUT (or property), 1 = IN
};

// IDHandler.readRelationType: 3-bit prefix [system/invisible(2) | is-edge(1)] followed by
// the prefixed varint (typeCount << 1 | dir) (VariableLong.readPositiveWithPrefix).
inline bool read_relation_type(Cursor& c, RelType& rt) {
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
inline int64_t key_to_vertex_id(int64_t key, int pb) {
    const uint64_t k = static_cast<uint64_t>(key);
    if ((k & 3u) == 1u) return key;      // schema vertex: key is the id
    const int poff = 64 - pb;
    const uint64_t partition = poff < 64 ? (k >> poff) : 0;
    const uint64_t count = (k >> 3) & ((1ULL << (poff - 3)) - 1);
    return static_cast<int64_t>((((count << pb) + partition) << 3) | (k & 7u));
}

// Vertex cuts (VertexIDType.PartitionedVertex, suffix 010b, IDManager.java:78-90).
inline bool is_partitioned_vertex(int64_t vid, int pb) {            // isPartitionedVertex :557-559
    return (vid & 7) == 2 && (static_cast<uint64_t>(vid) >> (pb + 3)) > 0;
}
// getCanonicalVertexId (:530-534): the representative in partition getPartitionHashForId(count)
// (:512-523, XOR of the count's pb-bit chunks).
inline int64_t canonical_vertex_id(int64_t vid, int pb) {
    if (pb <= 0) return vid;
    const uint64_t count = static_cast<uint64_t>(vid) >> (pb + 3);
    uint64_t part = 0;
    for (int off = 0; off < 64; off += pb) part ^= (count >> off) & ((1ULL << pb) - 1);
    return static_cast<int64_t>((((count << pb) + part) << 3) | 2u);
}

// Per-edge-label decode plan derived from tgo_schema.
struct LabelPlan {
    int64_t type_id = 0;
    int multiplicity = TGO_MULTI;
    bool selected = true;      // passes the scope's label filter
    int weight_sig_index = -1; // weight is signature[k]
    bool weight_in_sortkey = false;
    std::vector<int> sig_types;  // datatype of each signature key (0 = unknown)
};

struct DecodePlan {
    std::vector<LabelPlan> labels;   // small; linear search is fine
    std::vector<std::pair<int64_t, int>> key_types;
    int64_t weight_key = 0;
    const LabelPlan* find(int64_t id) const {
        for (const auto& l : labels) if (l.type_id == id) return &l;
        return nullptr;
    }
    int datatype(int64_t key) const {
        for (const auto& kt : key_types) if (kt.first == key) return kt.second;
        return 0;
    }
};

inline bool unique_in(int mult, int dir) {  // Multiplicity.isUnique
    return dir == 1 ? (mult == TGO_ONE2MANY || mult == TGO_ONE2ONE)
                    : (mult == TGO_MANY2ONE || mult == TGO_ONE2ONE);
}

// Reads one non-byte-ordered inline value (null flag first).  Returns false on a codec
// error; *present=false for a serialized null.
inline bool read_value(Cursor& c, int dt, bool& present, int64_t& v) {
    const uint8_t flag = c.get();
    if (flag == 0xFF) { present = false; return !c.bad; }
    if (flag != 0) return false;
    present = true;
    switch (dt) {
        case TGO_DT_BYTE: v = static_cast<int8_t>(c.get() - 128); break;
        case TGO_DT_SHORT: v = static_cast<int16_t>(c.be(2) - 32768); break;
        case TGO_DT_INTEGER: {
            const int64_t l = c.svarint();
            if (l < INT32_MIN || l > INT32_MAX) return false;
            v = l;
            break;
        }
        case TGO_DT_LONG: v = static_cast<int64_t>(c.be(8) + 0x8000000000000000ULL); break;
        case TGO_DT_FLOAT: c.be(4); v = 0; break;
        case TGO_DT_DOUBLE: c.be(8); v = 0; break;
        case TGO_DT_BOOLEAN: v = c.get(); break;
        default: return false;
    }
    return !c.bad;
}

struct DecodedEdge {
    int64_t type_id;
    int dir;
    int64_t other;
    bool has_weight;
    int32_t weight;
};

enum class DecodeResult { kOk, kSkip, kError, kUnsupported };

// EdgeSerializer.parseRelation restricted to what the traversal needs: direction, other
// vertex id and (optionally) the Integer weight property.
inline DecodeResult decode_edge(const uint8_t* d, size_t len, size_t value_pos,
                                const DecodePlan& plan, DecodedEdge& out) {
    Cursor c{d, len, 0};
    RelType rt;
    if (value_pos > len || !read_relation_type(c, rt) || !rt.is_edge) return DecodeResult::kError;
    const LabelPlan* lp = plan.find(rt.type_id);
    if (!lp) return DecodeResult::kError;            // tx.getExistingRelationType fails
    if (!lp->selected) return DecodeResult::kSkip;
    out.type_id = rt.type_id;
    out.dir = rt.dir;
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
    if (plan.weight_key == 0) return DecodeResult::kOk;
    if (lp->weight_in_sortkey) return DecodeResult::kUnsupported;
    c.pos = props;
    for (size_t k = 0; k < lp->sig_types.size(); ++k) {
        bool present; int64_t v = 0;
        if (!read_value(c, lp->sig_types[k], present, v)) return DecodeResult::kError;
        if (static_cast<int>(k) == lp->weight_sig_index) {
            out.has_weight = present;
            out.weight = static_cast<int32_t>(v);
            return DecodeResult::kOk;
        }
    }
    while (c.pos < len) {                             // remaining properties
        const int64_t kid = static_cast<int64_t>((c.varint() << 4) | 5u);
        bool present; int64_t v = 0;
        const int dt = plan.datatype(kid);
        if (!read_value(c, dt, present, v)) {
            return dt == 0 ? DecodeResult::kUnsupported : DecodeResult::kError;
        }
        if (kid == plan.weight_key) {
            out.has_weight = present;
            out.weight = static_cast<int32_t>(v);
            return DecodeResult::kOk;
        }
    }
    return DecodeResult::kOk;
}

}  // namespace tgo

// graph_build.cpp — one-time CSR assembly on the host (multi-threaded).
//
// Replaces the reference's per-superstep rescan + decode (FulgoraGraphComputer.java:155-164
// runs a full edgestore scan every iteration; VertexJobConverter.process,
// VertexJobConverter.java:109-129, rebuilds a PreloadedVertex per row per superstep).
// Here the rows are decoded once into an out-CSR and an in-CSR of dense vertex ids.
#include <algorithm>
#include <array>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <atomic>
#include <cmath>
#include <cstring>
#include <thread>
#include <unordered_map>
#include "codec.hpp"
#include "engine.hpp"

namespace tgo {

template <class F>
static void parallel_for(int64_t n, int threads, F&& fn) {
    if (threads <= 1 || n < 4096) { fn(int64_t(0), n, 0); return; }
    std::vector<std::thread> th;
    th.reserve(threads);
    for (int t = 0; t < threads; ++t) {
        const int64_t lo = n * t / threads, hi = n * (t + 1) / threads;
        th.emplace_back([&, lo, hi, t] { fn(lo, hi, t); });
    }
    for (auto& x : th) x.join();
}

// Dynamic chunked loop for skewed per-item work (e.g. sorting hub rows).
template <class F>
static void parallel_dynamic(int64_t n, int threads, int64_t chunk, F&& fn) {
    std::atomic<int64_t> next{0};
    auto worker = [&] {
        for (;;) {
            const int64_t lo = next.fetch_add(chunk);
            if (lo >= n) break;
            fn(lo, std::min(n, lo + chunk));
        }
    };
    if (threads <= 1) { worker(); return; }
    std::vector<std::thread> th;
    for (int t = 0; t < threads; ++t) th.emplace_back(worker);
    for (auto& x : th) x.join();
}

// ------------------------------------------------------------------ rows -> staging
// Decode plan: labels sorted by type id, property keys sorted by id (binary-searched by the
// codec on the host and on the device).  The weight is an Integer property
// (ShortestDistanceVertexProgram.java:53 reads edge.<Integer>value(weight): another datatype
// is a ClassCastException in the reference).
int build_plan(const tgo_schema* schema, const tgo_load_opts* opts, HostPlan& hp, std::string& err) {
    hp = HostPlan();
    hp.weight_key = opts->weight_key;
    std::vector<std::pair<int64_t, int8_t>> keys;
    for (int k = 0; k < schema->n_property_keys; ++k)
        keys.emplace_back(schema->property_keys[k].key_id, static_cast<int8_t>(schema->property_keys[k].datatype));
    std::sort(keys.begin(), keys.end());
    for (const auto& kt : keys) { hp.key_ids.push_back(kt.first); hp.key_dts.push_back(kt.second); }
    auto dt_of = [&](int64_t key) -> int8_t {
        auto it = std::lower_bound(hp.key_ids.begin(), hp.key_ids.end(), key);
        return it != hp.key_ids.end() && *it == key ? hp.key_dts[it - hp.key_ids.begin()] : 0;
    };
    // The weight column is 32 bits: the integral datatypes that fit (Byte, Short, Integer,
    // Character, Boolean) as integers, Float as its IEEE bits.  Long and Double keys are wide:
    // the column then holds each entry's staged position and the 64-bit values (the Long, the
    // Double's IEEE bits) ride in a parallel staged array (RowStaging::wv) that becomes the
    // graph's value table (DevGraph::wval).  Date / String weights are not supported.
    // ShortestDistanceVertexProgram itself casts to Integer (edge.<Integer>value, :53): its entry
    // points reject any other weight datatype, as the reference fails with a ClassCastException;
    // generic programs' edge functions take them all.
    if (opts->weight_key != 0) {
        const int dt = dt_of(opts->weight_key);
        if (dt != TGO_DT_INTEGER && dt != TGO_DT_BYTE && dt != TGO_DT_SHORT && dt != TGO_DT_CHARACTER &&
            dt != TGO_DT_BOOLEAN && dt != TGO_DT_FLOAT && !wide_weight_dt(dt)) {
            err = "weight property must be a Byte, Short, Integer, Character, Boolean, Float, Long or Double key";
            return TGO_E_UNSUPPORTED;
        }
        hp.weight_dt = dt;
    }
    std::vector<LabelPlan> labels;
    for (int t = 0; t < schema->n_edge_types; ++t) {
        const tgo_edge_type& et = schema->edge_types[t];
        LabelPlan lp{};
        lp.type_id = et.type_id;
        lp.multiplicity = et.multiplicity;
        lp.desc = et.sort_order == TGO_ORDER_DESC;
        lp.selected = 1;
        if (opts->n_labels > 0) {
            lp.selected = 0;
            for (int j = 0; j < opts->n_labels; ++j) lp.selected |= opts->label_ids[j] == et.type_id;
        }
        const bool multi = et.multiplicity == TGO_MULTI;
        lp.n_sort = multi ? et.n_sort_key : 0;     // constrained labels carry no sort key (:235)
        lp.n_sig = et.n_signature;
        lp.sort_dt_off = static_cast<int32_t>(hp.dts.size());
        for (int k = 0; k < lp.n_sort; ++k) hp.dts.push_back(dt_of(et.sort_key_ids[k]));
        lp.sig_dt_off = static_cast<int32_t>(hp.dts.size());
        for (int k = 0; k < lp.n_sig; ++k) hp.dts.push_back(dt_of(et.signature_ids[k]));
        lp.weight_where = opts->weight_key == 0 ? kWeightNone : kWeightRemaining;
        for (int k = 0; k < lp.n_sort && opts->weight_key != 0; ++k)
            if (et.sort_key_ids[k] == opts->weight_key) { lp.weight_where = kWeightSortKey; lp.weight_index = k; break; }
        for (int k = 0; k < lp.n_sig && lp.weight_where == kWeightRemaining; ++k)
            if (et.signature_ids[k] == opts->weight_key) { lp.weight_where = kWeightSignature; lp.weight_index = k; break; }
        labels.push_back(lp);
    }
    std::sort(labels.begin(), labels.end(), [](const LabelPlan& a, const LabelPlan& b) { return a.type_id < b.type_id; });
    for (size_t i = 1; i < labels.size(); ++i)
        if (labels[i].type_id == labels[i - 1].type_id) { err = "duplicate edge type in schema"; return TGO_E_INVALID; }
    hp.n_labels = static_cast<int32_t>(labels.size());
    hp.label_bytes.resize(labels.size() * sizeof(LabelPlan));
    if (!labels.empty()) std::memcpy(hp.label_bytes.data(), labels.data(), hp.label_bytes.size());
    return TGO_OK;
}

PlanView plan_view(const HostPlan& hp) {
    PlanView v{};
    v.labels = reinterpret_cast<const LabelPlan*>(hp.label_bytes.data());
    v.n_labels = hp.n_labels;
    v.n_keys = static_cast<int32_t>(hp.key_ids.size());
    v.key_ids = hp.key_ids.data();
    v.key_dts = hp.key_dts.data();
    v.dts = hp.dts.data();
    v.weight_key = hp.weight_key;
    return v;
}

int decode_one_entry(const tgo_schema* schema, const tgo_load_opts* opts, const uint8_t* entry,
                     int64_t len, int64_t value_pos, tgo_edge_entry* out, std::string& err) {
    HostPlan hp;
    if (int rc = build_plan(schema, opts, hp, err)) return rc;
    if (opts->weight_key != 0 && wide_weight_dt(hp.weight_dt)) {      // tgo_edge_entry.weight is 32 bits
        err = "tgo_decode_edge_entry: a Long / Double weight key does not fit the 32-bit weight field";
        return TGO_E_UNSUPPORTED;
    }
    if (len < 0 || value_pos < 0 || (len > 0 && !entry)) { err = "invalid entry"; return TGO_E_INVALID; }
    DecodedEdge de{};
    const DecodeResult dr = decode_edge(entry, static_cast<size_t>(len), static_cast<size_t>(value_pos),
                                        plan_view(hp), de);
    *out = tgo_edge_entry{};
    if (dr == DecodeResult::kError) { err = "malformed edge entry"; return TGO_E_CODEC; }
    if (dr == DecodeResult::kUnsupported) { err = "inline property of a key missing from the schema"; return TGO_E_UNSUPPORTED; }
    if (dr == DecodeResult::kSkip) return TGO_OK;
    out->type_id = de.type_id;
    out->other_id = de.other;
    out->dir = de.dir;
    out->selected = 1;
    out->has_weight = de.has_weight ? 1 : 0;
    out->weight = de.weight;
    return TGO_OK;
}


// ------------------------------------------------------------------ rows -> staging
// First batch: remember the load options; later batches must repeat them.
int staging_begin(RowStaging& st, const tgo_load_opts* opts, std::string& err) {
    if (!st.active) {
        st = RowStaging();
        st.active = true;
        st.opts = *opts;
        st.labels.assign(opts->label_ids, opts->label_ids + opts->n_labels);
        st.opts.label_ids = nullptr;
        st.row_begin.push_back(0);
    } else if (st.opts.scope != opts->scope || st.opts.weight_key != opts->weight_key ||
               st.opts.apply_cap != opts->apply_cap) {
        err = "tgo_load_opts differ between row batches";
        return TGO_E_INVALID;
    }
    return TGO_OK;
}

int decode_rows(RowStaging& st, const tgo_rows* rows, const tgo_schema* schema,
                const tgo_load_opts* opts, int pb, int64_t hard_limit, int threads,
                std::string& err) {
    HostPlan hp;
    if (int rc = build_plan(schema, opts, hp, err)) return rc;
    const PlanView plan = plan_view(hp);
    // Untyped single-direction scopes are not "fitted" and get the hard limit; BOTH and
    // typed scopes keep NO_LIMIT (BasicVertexCentricQueryBuilder.java:418-431,469-474;
    // QueryContainer.java:122).
    const bool typed = opts->n_labels > 0;
    const int64_t limit = (opts->apply_cap && !typed && opts->scope != TGO_SCOPE_BOTH_E)
                              ? hard_limit : INT64_MAX;

    struct Local {
        std::vector<int64_t> vid, cnt, other;
        std::vector<uint8_t> dir, rep;
        std::vector<int32_t> w;
        std::vector<int64_t> wv;         // wide weight keys: the 64-bit values
        int64_t ghost = 0, truncated = 0, skipped = 0;
        int rc = TGO_OK;
        std::string msg;
    };
    const bool wide = opts->weight_key != 0 && wide_weight_dt(hp.weight_dt);
    const int64_t nrows = rows->nrows;
    const int nth = std::max(1, std::min<int>(threads, static_cast<int>((nrows + 1023) / 1024)));
    std::vector<Local> loc(nth);
    parallel_for(nrows, nth, [&](int64_t lo, int64_t hi, int t) {
        Local& L = loc[t];
        for (int64_t r = lo; r < hi && L.rc == TGO_OK; ++r) {
            const int64_t vid = key_to_vertex_id(rows->row_keys[r], pb);
            if (vid & 1) { ++L.skipped; continue; }           // key filter: Invisible (:156-162)
            const int64_t sfx = vid & 7;
            if (sfx != 0 && sfx != 2 && sfx != 4) { L.rc = TGO_E_CODEC; L.msg = "row key has an unrecognized vertex id type"; break; }
            // a non-canonical representative row of a vertex cut skips the ghost check
            // (VertexJobConverter.java:132) and is folded into its canonical vertex at assembly
            const bool is_rep = sfx == 2 && vid != canonical_vertex_id(vid, pb);
            const uint8_t* base = rows->entry_bytes + rows->row_byte_begin[r];
            const int64_t e0 = rows->row_entry_begin[r], e1 = rows->row_entry_begin[r + 1];
            auto ent_start = [&](int64_t k) -> int64_t {
                return k == e0 ? 0 : static_cast<int64_t>(static_cast<uint64_t>(rows->entry_limit_valpos[k - 1]) >> 32);
            };
            if (e1 <= e0) { L.rc = TGO_E_CODEC; L.msg = "row without entries"; break; }
            if (!is_rep) {   // ghost check: the first column must be VertexExists (:131-137)
                const int64_t end = static_cast<int64_t>(static_cast<uint64_t>(rows->entry_limit_valpos[e0]) >> 32);
                Cursor c{base, static_cast<size_t>(end), 0};
                RelType rt;
                if (!read_relation_type(c, rt)) { L.rc = TGO_E_CODEC; L.msg = "malformed first column"; break; }
                if (rt.is_edge || rt.type_id != kVertexExistsId) { ++L.ghost; continue; }
            }
            // user-edge slice [0x60,0x80): entries are column-sorted, so it is contiguous.
            int64_t first = -1, cnt = 0;
            for (int64_t k = e0; k < e1; ++k) {
                const uint8_t c0 = base[ent_start(k)];
                if (c0 >= 0x60 && c0 < 0x80) { if (first < 0) first = k; ++cnt; }
                else if (first >= 0) break;
            }
            if (limit != INT64_MAX && cnt >= limit) ++L.truncated;     // TRUNCATED_ENTRY_LISTS
            const int64_t keep = std::min(cnt, limit);
            int64_t kept = 0;
            for (int64_t k = first; k >= 0 && k < first + keep; ++k) {
                const int64_t s = ent_start(k);
                const int64_t e = static_cast<int64_t>(static_cast<uint64_t>(rows->entry_limit_valpos[k]) >> 32);
                const int64_t vp = rows->entry_limit_valpos[k] & 0x7FFFFFFF;
                DecodedEdge de;
                const DecodeResult dr = decode_edge(base + s, static_cast<size_t>(e - s), static_cast<size_t>(vp), plan, de);
                if (dr == DecodeResult::kSkip) continue;
                if (dr != DecodeResult::kOk) {
                    L.rc = dr == DecodeResult::kUnsupported ? TGO_E_UNSUPPORTED : TGO_E_CODEC;
                    L.msg = dr == DecodeResult::kUnsupported ? "inline property of a key missing from the schema"
                                                             : "malformed edge entry";
                    break;
                }
                // messages are looked up by canonical id (VertexMemoryHandler.java:89)
                L.other.push_back(is_partitioned_vertex(de.other, pb) ? canonical_vertex_id(de.other, pb) : de.other);
                L.dir.push_back(static_cast<uint8_t>(de.dir));
                L.w.push_back(opts->weight_key == 0 ? 1 : (de.has_weight ? de.weight : kMissingWeight));
                if (wide) L.wv.push_back(de.has_weight ? de.weight64 : 0);
                ++kept;
            }
            if (L.rc != TGO_OK) break;
            L.vid.push_back(is_rep ? canonical_vertex_id(vid, pb) : vid);
            L.rep.push_back(is_rep ? 1 : 0);
            L.cnt.push_back(kept);
        }
    });
    for (auto& L : loc) if (L.rc != TGO_OK) { err = L.msg; return L.rc; }
    if (int rc = staging_begin(st, opts, err)) return rc;
    st.plan.weight_dt = hp.weight_dt;     // the assembly types the weight column from it (Float / Long / Double)
    for (auto& L : loc) {
        st.ghost += L.ghost; st.truncated += L.truncated; st.skipped += L.skipped;
        for (size_t i = 0; i < L.vid.size(); ++i) {
            st.vid.push_back(L.vid[i]);
            st.rep.push_back(L.rep[i]);
            st.n_rep += L.rep[i];
            st.row_begin.push_back(st.row_begin.back() + L.cnt[i]);
        }
        st.other.insert(st.other.end(), L.other.begin(), L.other.end());
        st.dir.insert(st.dir.end(), L.dir.begin(), L.dir.end());
        const size_t base = st.w.size();
        st.w.insert(st.w.end(), L.w.begin(), L.w.end());
        if (wide) {                      // the column of a wide key: each entry's staged position
            if (st.w.size() >= static_cast<size_t>(INT32_MAX)) { err = "wide weights: more than 2^31 - 1 staged entries"; return TGO_E_UNSUPPORTED; }
            for (size_t i = base; i < st.w.size(); ++i)
                if (st.w[i] != kMissingWeight) st.w[i] = static_cast<int32_t>(i);
            st.wv.insert(st.wv.end(), L.wv.begin(), L.wv.end());
        }
    }
    return TGO_OK;
}

// ------------------------------------------------------------------ helpers
// Open-addressing Titan id -> dense index map (the role of FulgoraVertexMemory's
// NonBlockingHashMapLong keyed by Titan id, FulgoraVertexMemory.java:30,49-58).
struct IdMap {
    std::vector<int64_t> keys;
    std::vector<int32_t> vals;
    uint64_t mask = 0;
    static uint64_t h(uint64_t x) { x ^= x >> 31; x *= 0x7fb5d329728ea185ULL; x ^= x >> 27; x *= 0x81dadef4bc2dd44dULL; return x ^ (x >> 33); }
    void build(const std::vector<int64_t>& ids) {
        uint64_t cap = 16;
        while (cap < ids.size() * 2) cap <<= 1;
        mask = cap - 1;
        keys.assign(cap, INT64_MIN);
        vals.assign(cap, -1);
        for (size_t i = 0; i < ids.size(); ++i) {
            uint64_t p = h(static_cast<uint64_t>(ids[i])) & mask;
            while (keys[p] != INT64_MIN && keys[p] != ids[i]) p = (p + 1) & mask;
            keys[p] = ids[i];
            vals[p] = static_cast<int32_t>(i);
        }
    }
    int32_t find(int64_t id) const {
        uint64_t p = h(static_cast<uint64_t>(id)) & mask;
        for (;;) {
            if (keys[p] == id) return vals[p];
            if (keys[p] == INT64_MIN) return -1;
            p = (p + 1) & mask;
        }
    }
};

// Transpose of the union of `lists` (each an n-row CSR): t[w] gets v for every w in L(v), each
// transposed row sorted by source id.  Threads own contiguous source ranges of equal entry
// counts; per-thread histograms give every thread its slots in every row, so the scatter is
// stable (source order) without atomics.
static void transpose_lists(int64_t n, const std::vector<const HostCsr*>& lists, bool weighted,
                            HostCsr& t, int threads) {
    int64_t E = 0;
    for (const HostCsr* L : lists) E += static_cast<int64_t>(L->adj.size());
    const int T = std::max(1, std::min<int>(threads, static_cast<int>(std::max<int64_t>(1, E / 65536))));
    // source ranges [vb[i], vb[i+1]) with ~E/T entries each
    std::vector<int64_t> vb(T + 1, n);
    vb[0] = 0;
    {
        int64_t acc = 0, next = 1;
        for (int64_t v = 0; v < n && next < T; ++v) {
            for (const HostCsr* L : lists) acc += L->off[v + 1] - L->off[v];
            while (next < T && acc >= E * next / T) vb[next++] = v + 1;
        }
    }
    std::vector<std::vector<int64_t>> pos(T, std::vector<int64_t>(static_cast<size_t>(n), 0));
    auto run = [&](auto&& body) {
        std::vector<std::thread> th;
        for (int i = 0; i < T; ++i) th.emplace_back([&, i] { body(i); });
        for (auto& x : th) x.join();
    };
    run([&](int i) {
        int64_t* c = pos[i].data();
        for (int64_t v = vb[i]; v < vb[i + 1]; ++v)
            for (const HostCsr* L : lists)
                for (int64_t k = L->off[v]; k < L->off[v + 1]; ++k) ++c[L->adj[k]];
    });
    t.off.assign(n + 1, 0);
    parallel_for(n, threads, [&](int64_t a, int64_t b, int) {
        for (int64_t w = a; w < b; ++w) {
            int64_t s = 0;
            for (int i = 0; i < T; ++i) s += pos[i][w];
            t.off[w + 1] = s;
        }
    });
    for (int64_t w = 0; w < n; ++w) t.off[w + 1] += t.off[w];
    parallel_for(n, threads, [&](int64_t a, int64_t b, int) {
        for (int64_t w = a; w < b; ++w) {
            int64_t p = t.off[w];
            for (int i = 0; i < T; ++i) { const int64_t c = pos[i][w]; pos[i][w] = p; p += c; }
        }
    });
    t.adj.assign(static_cast<size_t>(E), 0);
    if (weighted) t.w.assign(static_cast<size_t>(E), 0);
    run([&](int i) {
        int64_t* p = pos[i].data();
        for (int64_t v = vb[i]; v < vb[i + 1]; ++v)
            for (const HostCsr* L : lists)
                for (int64_t k = L->off[v]; k < L->off[v + 1]; ++k) {
                    const int64_t q = p[L->adj[k]]++;
                    t.adj[q] = static_cast<int32_t>(v);
                    if (weighted) t.w[q] = L->w[k];
                }
    });
}

// Degree-grouped relabel (DBG, Faldu et al., IISWC'19): vertices are grouped by
// half-octave of their total degree, hottest group first, keeping row order inside a
// group.  High-degree vertices then share cache lines in every per-vertex array, so the
// random message gathers of the pull kernels and the frontier-bitmap probes of bottom-up
// BFS hit the XCD L2 / Infinity Cache instead of HBM.  Purely a device layout: the API
// keeps row-order dense ids (perm maps them) and every result is mapped back.
// order[v] = position of vertex v (0..n-1) when grouped by half-octave of its degree deg(v),
// hottest group first, index order kept inside a group.
template <class Deg>
static void degree_group_order(int64_t n, Deg deg, std::vector<int32_t>& order) {
    std::vector<int> bucket(n);
    int maxb = 0;
    for (int64_t v = 0; v < n; ++v) {
        const int64_t d = deg(v);
        const int b = d == 0 ? 0 : 1 + static_cast<int>(2.0 * std::log2(static_cast<double>(d)));
        bucket[v] = b;
        maxb = std::max(maxb, b);
    }
    std::vector<int64_t> start(maxb + 2, 0);
    for (int64_t v = 0; v < n; ++v) ++start[maxb - bucket[v] + 1];          // descending buckets
    for (int b = 0; b <= maxb; ++b) start[b + 1] += start[b];
    order.assign(n, 0);
    for (int64_t v = 0; v < n; ++v) order[v] = static_cast<int32_t>(start[maxb - bucket[v]]++);
}

// Rows move to g.perm[v]; every neighbour id u becomes nbr(u); rows are re-sorted by the
// new neighbour ids (stable).
template <class Nbr>
static void permute_graph(HostGraph& g, Nbr nbr, int threads) {
    const int64_t n = g.n;
    std::vector<int32_t> inv(n);
    for (int64_t v = 0; v < n; ++v) inv[g.perm[v]] = static_cast<int32_t>(v);
    auto remap = [&](HostCsr& c) {
        HostCsr r;
        r.off.assign(n + 1, 0);
        for (int64_t u = 0; u < n; ++u) r.off[u + 1] = r.off[u] + (c.off[inv[u] + 1] - c.off[inv[u]]);
        r.adj.resize(c.adj.size());
        const bool hw = !c.w.empty(), hc = !c.col.empty();
        const bool w = hw || hc;                    // payloads follow their entries (stable)
        if (hw) r.w.resize(c.w.size());
        if (hc) r.col.resize(c.col.size());
        // neighbour ids first, in one streaming parallel pass
        parallel_for(static_cast<int64_t>(c.adj.size()), threads, [&](int64_t lo, int64_t hi, int) {
            for (int64_t k = lo; k < hi; ++k) c.adj[k] = static_cast<int32_t>(nbr(c.adj[k]));
        });
        // small chunks: rows are hottest-first, so the first rows are the hubs
        parallel_dynamic(n, threads, 64, [&](int64_t lo, int64_t hi) {
            std::vector<uint64_t> key;
            for (int64_t u = lo; u < hi; ++u) {
                const int64_t b = c.off[inv[u]], len = c.off[inv[u] + 1] - b;
                int32_t* dst = r.adj.data() + r.off[u];
                if (!w) {                           // equal neighbours are indistinguishable: sort ids
                    std::memcpy(dst, c.adj.data() + b, static_cast<size_t>(len) * sizeof(int32_t));
                    if (len <= 32) {
                        for (int64_t i = 1; i < len; ++i) {
                            const int32_t x = dst[i];
                            int64_t j = i - 1;
                            while (j >= 0 && dst[j] > x) { dst[j + 1] = dst[j]; --j; }
                            dst[j + 1] = x;
                        }
                    } else {
                        std::sort(dst, dst + len);
                    }
                    continue;
                }
                key.resize(len);
                for (int64_t j = 0; j < len; ++j)   // (new neighbour, original position): stable
                    key[j] = (static_cast<uint64_t>(static_cast<uint32_t>(c.adj[b + j])) << 32) | static_cast<uint64_t>(j);
                std::sort(key.begin(), key.end());
                for (int64_t j = 0; j < len; ++j) {
                    dst[j] = static_cast<int32_t>(key[j] >> 32);
                    const int64_t src = b + static_cast<int64_t>(key[j] & 0xFFFFFFFFULL);
                    if (hw) r.w[r.off[u] + j] = c.w[src];
                    if (hc) r.col[r.off[u] + j] = c.col[src];
                }
            }
        });
        c = std::move(r);
    };
    remap(g.out);
    remap(g.in);
}

// Degree-grouped relabel (DBG, Faldu et al., IISWC'19): vertices are grouped by
// half-octave of their total degree, hottest group first, keeping row order inside a
// group.  High-degree vertices then share cache lines in every per-vertex array, so the
// random message gathers of the pull kernels and the frontier-bitmap probes of bottom-up
// BFS hit the XCD L2 / Infinity Cache instead of HBM.  Purely a device layout: the API
// keeps row-order dense ids (perm maps them) and every result is mapped back.
static void relabel_by_degree(HostGraph& g, int threads) {
    auto t0 = std::chrono::steady_clock::now();
    degree_group_order(g.n, [&](int64_t v) {
        return (g.out.off[v + 1] - g.out.off[v]) + (g.in.off[v + 1] - g.in.off[v]);
    }, g.perm);
    auto t1 = std::chrono::steady_clock::now();
    const int32_t* p = g.perm.data();
    permute_graph(g, [p](int32_t u) { return p[u]; }, threads);
    if (std::getenv("TGO_TRACE") && std::atoi(std::getenv("TGO_TRACE")))
        std::fprintf(stderr, "[tgo] relabel: order %.1f ms, permute %.1f ms\n",
                     std::chrono::duration<double, std::milli>(t1 - t0).count(),
                     std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t1).count());
}

// Multi-GPU layout (tgo_part_layout): the degree-grouped order of the owned range, as
// global internal ids lo + order[v].  Degrees = entries of the owned rows.
int partition_layout(const tgo_edges* e, int64_t n_global, int64_t lo, int64_t hi, int threads,
                     int32_t* layout_local, std::string& err) {
    const int64_t n = hi - lo;
    if (lo < 0 || hi > n_global || n <= 0 || n_global >= INT32_MAX) { err = "invalid partition range"; return TGO_E_INVALID; }
    std::vector<std::atomic<int64_t>> deg(n);
    for (auto& d : deg) d.store(0, std::memory_order_relaxed);
    parallel_for(e->m, threads, [&](int64_t a, int64_t b, int) {
        for (int64_t k = a; k < b; ++k) {
            if (e->src[k] >= lo && e->src[k] < hi) deg[e->src[k] - lo].fetch_add(1, std::memory_order_relaxed);
            if (e->dst[k] >= lo && e->dst[k] < hi) deg[e->dst[k] - lo].fetch_add(1, std::memory_order_relaxed);
        }
    });
    std::vector<int32_t> order;
    degree_group_order(n, [&](int64_t v) { return deg[v].load(std::memory_order_relaxed); }, order);
    for (int64_t v = 0; v < n; ++v) layout_local[v] = static_cast<int32_t>(lo + order[v]);
    return TGO_OK;
}

// Decide whether the push view equals the stored opposite list; if not, build it.
static void finish_views(HostGraph& g, int threads) {
    const int64_t n = g.n;
    bool consistent = g.truncated == 0;
    if (consistent) {   // every OUT entry u->v must have a matching IN entry at v (count check)
        std::vector<std::atomic<int64_t>> indeg(n);
        for (auto& c : indeg) c.store(0, std::memory_order_relaxed);
        parallel_for(static_cast<int64_t>(g.out.adj.size()), threads, [&](int64_t lo, int64_t hi, int) {
            for (int64_t k = lo; k < hi; ++k) indeg[g.out.adj[k]].fetch_add(1, std::memory_order_relaxed);
        });
        for (int64_t v = 0; v < n && consistent; ++v)
            consistent = indeg[v].load(std::memory_order_relaxed) == g.in.off[v + 1] - g.in.off[v];
    }
    g.has_transpose = !consistent;
    g.push_t = HostCsr();
    if (!consistent) {
        std::vector<const HostCsr*> pull;
        if (g.scope == TGO_SCOPE_IN_E) pull = {&g.out};
        else if (g.scope == TGO_SCOPE_OUT_E) pull = {&g.in};
        else pull = {&g.out, &g.in};
        transpose_lists(n, pull, g.has_weight, g.push_t, threads);
    }
}

// ------------------------------------------------------------------ vertex cuts
// Fold every non-canonical representative row into its canonical vertex: Fulgora combines
// each representative row's messages with the program's combiner, aggregates them per
// canonical id and executes the program once on the aggregate (VertexProgramScanJob.java
// :76-92, FulgoraVertexMemory.java:121-147, PartitionedVertexProgramExecutor.java:47-103).
// With an associative combiner (ShortestDistance min, DegreeCounter sum) that equals one
// vertex holding the union of the rows, which is what the device sees.  Representative rows
// whose canonical row was not processed never execute (GHOTST_PARTITION_VERTEX, :53-56).
// Entry order per vertex: its own row, then the other representatives in scan order.
static void fold_representatives(RowStaging& st, HostGraph& g) {
    const int64_t rows = static_cast<int64_t>(st.vid.size());
    std::vector<int64_t> live;
    for (int64_t r = 0; r < rows; ++r)
        if (!st.rep[r]) live.push_back(st.vid[r]);
    IdMap map;
    map.build(live);
    const int64_t n = static_cast<int64_t>(live.size());
    std::vector<int32_t> owner(rows);
    std::vector<int64_t> cnt(n + 1, 0);
    std::vector<uint8_t> pv(n, 0);
    for (int64_t r = 0, v = 0; r < rows; ++r) {
        owner[r] = st.rep[r] ? map.find(st.vid[r]) : static_cast<int32_t>(v++);
        if (owner[r] < 0) { ++g.ghost_partition_rows; continue; }
        if (st.rep[r]) { ++g.partition_rows; pv[owner[r]] = 1; }
        cnt[owner[r] + 1] += st.row_begin[r + 1] - st.row_begin[r];
    }
    for (int64_t r = 0; r < rows; ++r)    // every canonical row of a cut (PartitionedVertex suffix)
        if (!st.rep[r] && (st.vid[r] & 7) == 2) pv[owner[r]] = 1;
    for (int64_t v = 0; v < n; ++v) cnt[v + 1] += cnt[v];
    std::vector<int64_t> pos(cnt.begin(), cnt.end() - 1);
    std::vector<int64_t> other(cnt[n]);
    std::vector<uint8_t> dir(cnt[n]);
    std::vector<int32_t> w(st.w.empty() ? 0 : cnt[n]);
    for (int pass = 0; pass < 2; ++pass)
        for (int64_t r = 0; r < rows; ++r) {
            if (owner[r] < 0 || st.rep[r] != pass) continue;
            for (int64_t k = st.row_begin[r]; k < st.row_begin[r + 1]; ++k) {
                const int64_t p = pos[owner[r]]++;
                other[p] = st.other[k];
                dir[p] = st.dir[k];
                if (!w.empty()) w[p] = st.w[k];
            }
        }
    for (int64_t v = 0; v < n; ++v) g.partitioned += pv[v];
    st.vid = std::move(live);
    st.row_begin = std::move(cnt);
    st.other = std::move(other);
    st.dir = std::move(dir);
    st.w = std::move(w);
    st.rep.assign(n, 0);
    st.n_rep = 0;
    g.pv_flags = std::move(pv);
}

// ------------------------------------------------------------------ staging -> CSR
// TGO_TRACE=1: per-phase host assembly times on stderr.
struct PhaseClock {
    bool on;
    std::chrono::steady_clock::time_point t = std::chrono::steady_clock::now();
    PhaseClock() : on(std::getenv("TGO_TRACE") && std::atoi(std::getenv("TGO_TRACE")) != 0) {}
    void lap(const char* what) {
        if (!on) return;
        const auto now = std::chrono::steady_clock::now();
        std::fprintf(stderr, "[tgo] assemble %-12s %8.1f ms\n", what, std::chrono::duration<double, std::milli>(now - t).count());
        t = now;
    }
};

int assemble_from_rows(RowStaging& st, HostGraph& g, int threads, std::string& err) {
    PhaseClock clk;
    g = HostGraph();
    if (st.n_rep > 0 || std::any_of(st.vid.begin(), st.vid.end(), [](int64_t v) { return (v & 7) == 2; }))
        fold_representatives(st, g);
    g.n = static_cast<int64_t>(st.vid.size());
    if (g.n >= INT32_MAX) { err = "more than 2^31-1 vertices per device"; return TGO_E_UNSUPPORTED; }
    g.titan_id = st.vid;
    g.scope = st.opts.scope;
    g.has_weight = st.opts.weight_key != 0;
    g.weight_dt = st.plan.weight_dt ? st.plan.weight_dt : TGO_DT_INTEGER;
    const bool keep_col = (st.opts.flags & TGO_LOAD_COLUMN_ORDER) != 0;
    g.ghost = st.ghost; g.truncated = st.truncated; g.skipped = st.skipped;
    clk.lap("folds");
    IdMap map;
    map.build(st.vid);
    clk.lap("id map");
    const int64_t n = g.n;
    // Map Titan ids to dense ids; entries to non-executed vertices can never carry a
    // message (EMPTY_STATE => null, VertexState.java:103-137) and are dropped.
    std::vector<int32_t> dense(st.other.size());
    parallel_for(static_cast<int64_t>(st.other.size()), threads, [&](int64_t lo, int64_t hi, int) {
        for (int64_t k = lo; k < hi; ++k) dense[k] = map.find(st.other[k]);
    });
    clk.lap("lookups");
    std::vector<int64_t> co(n + 1, 0), ci(n + 1, 0);
    parallel_for(n, threads, [&](int64_t lo, int64_t hi, int) {
        for (int64_t v = lo; v < hi; ++v) {
            int64_t a = 0, b = 0;
            for (int64_t k = st.row_begin[v]; k < st.row_begin[v + 1]; ++k) {
                if (dense[k] < 0) continue;
                if (st.dir[k] == 0) ++a; else ++b;
            }
            co[v + 1] = a; ci[v + 1] = b;
        }
    });
    for (int64_t v = 0; v < static_cast<int64_t>(g.pv_flags.size()); ++v)
        if (g.pv_flags[v]) { g.pv_max_out = std::max(g.pv_max_out, co[v + 1]); g.pv_max_in = std::max(g.pv_max_in, ci[v + 1]); }
    for (int64_t v = 0; v < n; ++v) { co[v + 1] += co[v]; ci[v + 1] += ci[v]; }
    g.out.off = co; g.in.off = ci;
    g.out.adj.resize(co[n]); g.in.adj.resize(ci[n]);
    if (g.has_weight) { g.out.w.resize(co[n]); g.in.w.resize(ci[n]); }
    if (keep_col) { g.out.col.resize(co[n]); g.in.col.resize(ci[n]); }
    parallel_for(n, threads, [&](int64_t lo, int64_t hi, int) {
        for (int64_t v = lo; v < hi; ++v) {
            int64_t a = co[v], b = ci[v];
            for (int64_t k = st.row_begin[v]; k < st.row_begin[v + 1]; ++k) {
                if (dense[k] < 0) continue;
                // staged entries of a row are in the scan's column order
                const uint32_t col = static_cast<uint32_t>(k - st.row_begin[v]);
                if (st.dir[k] == 0) {
                    g.out.adj[a] = dense[k];
                    if (g.has_weight) g.out.w[a] = st.w[k];
                    if (keep_col) g.out.col[a] = col;
                    ++a;
                } else {
                    g.in.adj[b] = dense[k];
                    if (g.has_weight) g.in.w[b] = st.w[k];
                    if (keep_col) g.in.col[b] = col;
                    ++b;
                }
            }
        }
    });
    clk.lap("csr");
    relabel_by_degree(g, threads);
    clk.lap("relabel");
    finish_views(g, threads);
    clk.lap("views");
    st = RowStaging();
    return TGO_OK;
}

// Rows of the owners in [lo, hi) from an edge list: for every edge k with own[k] in range an
// entry (nbr[k] << 32 | k) in row own[k] - lo, each row sorted by (neighbour, edge index).
// Counting sort with per-thread histograms over contiguous edge chunks (no atomics: hub rows
// made a shared-counter scatter contention-bound), then the short per-row sorts.
static void rows_by_owner(int64_t m, const int32_t* own, const int32_t* nbr, int64_t lo, int64_t hi, int threads,
                          std::vector<int64_t>& off, std::vector<uint64_t>& keys) {
    const int64_t n = hi - lo;
    const int T = std::max(1, std::min<int>(threads, static_cast<int>(std::max<int64_t>(1, m / 65536))));
    std::vector<std::vector<int64_t>> pos(T, std::vector<int64_t>(static_cast<size_t>(n), 0));
    auto chunk = [&](int t) { return std::make_pair(m * t / T, m * (t + 1) / T); };
    {
        std::vector<std::thread> th;
        for (int t = 0; t < T; ++t)
            th.emplace_back([&, t] {
                const auto [a, b] = chunk(t);
                int64_t* c = pos[t].data();
                for (int64_t k = a; k < b; ++k)
                    if (own[k] >= lo && own[k] < hi) ++c[own[k] - lo];
            });
        for (auto& x : th) x.join();
    }
    off.assign(n + 1, 0);
    parallel_for(n, threads, [&](int64_t a, int64_t b, int) {
        for (int64_t v = a; v < b; ++v) {
            int64_t s = 0;
            for (int t = 0; t < T; ++t) s += pos[t][v];
            off[v + 1] = s;
        }
    });
    for (int64_t v = 0; v < n; ++v) off[v + 1] += off[v];
    parallel_for(n, threads, [&](int64_t a, int64_t b, int) {      // counts -> each thread's first slot
        for (int64_t v = a; v < b; ++v) {
            int64_t p = off[v];
            for (int t = 0; t < T; ++t) { const int64_t c = pos[t][v]; pos[t][v] = p; p += c; }
        }
    });
    keys.resize(static_cast<size_t>(off[n]));
    {
        std::vector<std::thread> th;
        for (int t = 0; t < T; ++t)
            th.emplace_back([&, t] {
                const auto [a, b] = chunk(t);
                int64_t* p = pos[t].data();
                for (int64_t k = a; k < b; ++k)
                    if (own[k] >= lo && own[k] < hi)
                        keys[p[own[k] - lo]++] = (static_cast<uint64_t>(static_cast<uint32_t>(nbr[k])) << 32) |
                                                  static_cast<uint64_t>(k);
            });
        for (auto& x : th) x.join();
    }
    std::vector<std::vector<int64_t>>().swap(pos);
    parallel_dynamic(n, threads, 256, [&](int64_t a, int64_t b) {   // edge order inside a row: sort by neighbour
        for (int64_t v = a; v < b; ++v) {
            uint64_t* r = keys.data() + off[v];
            const int64_t len = off[v + 1] - off[v];
            if (len <= 32) {
                for (int64_t i = 1; i < len; ++i) {
                    const uint64_t x = r[i];
                    int64_t j = i - 1;
                    while (j >= 0 && r[j] > x) { r[j + 1] = r[j]; --j; }
                    r[j + 1] = x;
                }
            } else {
                std::sort(r, r + len);
            }
        }
    });
}

// ------------------------------------------------------------------ edges -> CSR
// Each directed edge u->v contributes an OUT entry to row u and an IN entry to row v
// (StandardTitanGraph.java:564-591; loops therefore give two entries on one row).
// Within a row the column order is (direction, other Titan id, relation id)
// (IDHandler.writeRelationType puts the direction bit in the type varint;
// EdgeSerializer.java:255-259 writes the other id then the relation id backward-encoded,
// which is byte-order preserving, VariableLong.java:223-233).  Relation ids follow the
// edge index.  Titan ids, when not given, are assigned monotonically in dense order.
int assemble_from_edges(const tgo_edges* e, const tgo_load_opts* opts, int64_t hard_limit,
                        HostGraph& g, int threads, std::string& err) {
    PhaseClock clk;
    g = HostGraph();
    const int64_t n = e->n, m = e->m;
    if (n <= 0 || n >= INT32_MAX) { err = "vertex count out of range"; return TGO_E_INVALID; }
    g.n = n;
    g.scope = opts->scope;
    g.has_weight = opts->weight_key != 0 && e->weight != nullptr;
    g.weight_dt = TGO_DT_INTEGER;
    const bool keep_col = (opts->flags & TGO_LOAD_COLUMN_ORDER) != 0;
    g.titan_id.resize(n);
    for (int64_t v = 0; v < n; ++v)
        g.titan_id[v] = e->titan_ids ? e->titan_ids[v] : ((v + 1) << 3);  // NormalVertex, 0 partition bits
    for (int64_t v = 1; e->titan_ids && v < n; ++v)
        if (e->titan_ids[v] <= e->titan_ids[v - 1]) { err = "titan_ids must be strictly increasing"; return TGO_E_INVALID; }
    // Range check (a bad id would scatter out of bounds).
    std::atomic<bool> bad{false};
    parallel_for(m, threads, [&](int64_t lo, int64_t hi, int) {
        for (int64_t k = lo; k < hi; ++k)
            if (e->src[k] < 0 || e->src[k] >= n || e->dst[k] < 0 || e->dst[k] >= n) { bad = true; return; }
    });
    if (bad) { err = "edge endpoint out of range"; return TGO_E_INVALID; }

    const bool cap = opts->apply_cap && opts->n_labels == 0 && opts->scope != TGO_SCOPE_BOTH_E;
    const int64_t limit = cap ? hard_limit : INT64_MAX;

    // Full (uncapped) sorted rows for one direction: keys = neighbor << 32 | edge index.
    auto build_dir = [&](bool out_dir, std::vector<int64_t>& off, std::vector<uint64_t>& keys) {
        rows_by_owner(m, out_dir ? e->src : e->dst, out_dir ? e->dst : e->src, 0, n, threads, off, keys);
    };
    if (m >= (int64_t(1) << 32)) { err = "more than 2^32 edges per load"; return TGO_E_UNSUPPORTED; }
    std::vector<int64_t> off_o, off_i;
    std::vector<uint64_t> keys_o, keys_i;
    clk.lap("checks");
    build_dir(true, off_o, keys_o);
    clk.lap("out rows");
    build_dir(false, off_i, keys_i);
    clk.lap("in rows");
    // Cap: keep the first `limit` entries of [OUT... | IN...] per row.
    std::vector<int64_t> ko(n + 1, 0), ki(n + 1, 0);
    int64_t truncated = 0;
    for (int64_t v = 0; v < n; ++v) {
        const int64_t a = off_o[v + 1] - off_o[v], b = off_i[v + 1] - off_i[v];
        if (limit != INT64_MAX && a + b >= limit) ++truncated;
        const int64_t ka = std::min(a, limit);
        const int64_t kb = std::min(b, limit - ka);
        ko[v + 1] = ko[v] + ka;
        ki[v + 1] = ki[v] + kb;
    }
    g.truncated = truncated;
    // col_base: column position of the list's first entry in the row (OUT entries, direction
    // id 2, precede IN entries, id 3: IDHandler.DirectionID)
    auto fill = [&](const std::vector<int64_t>& off, const std::vector<uint64_t>& keys,
                    const std::vector<int64_t>& koff, HostCsr& c, const std::vector<int64_t>* col_base) {
        c.off = koff;
        c.adj.resize(koff[n]);
        if (g.has_weight) c.w.resize(koff[n]);
        if (keep_col) c.col.resize(koff[n]);
        parallel_for(n, threads, [&](int64_t lo, int64_t hi, int) {
            for (int64_t v = lo; v < hi; ++v) {
                const int64_t len = koff[v + 1] - koff[v];
                const int64_t cb = col_base ? (*col_base)[v + 1] - (*col_base)[v] : 0;
                for (int64_t j = 0; j < len; ++j) {
                    const uint64_t key = keys[off[v] + j];
                    c.adj[koff[v] + j] = static_cast<int32_t>(key >> 32);
                    if (g.has_weight) c.w[koff[v] + j] = e->weight[key & 0xFFFFFFFFULL];
                    if (keep_col) c.col[koff[v] + j] = static_cast<uint32_t>(cb + j);
                }
            }
        });
    };
    fill(off_o, keys_o, ko, g.out, nullptr);
    std::vector<uint64_t>().swap(keys_o);
    fill(off_i, keys_i, ki, g.in, &ko);
    clk.lap("fill");
    relabel_by_degree(g, threads);
    clk.lap("relabel");
    finish_views(g, threads);
    clk.lap("views");
    return TGO_OK;
}

// ------------------------------------------------------------------ 1-D vertex partition
// Multi-GPU: this device owns global vertices [lo, hi).  Its rows are the Titan rows of
// those vertices (OUT entries of edges leaving them, IN entries of edges entering them),
// with GLOBAL neighbour ids, so a gather reads remote messages from an all-gathered
// global vector and bottom-up BFS probes an all-gathered global frontier bitmap.
// No relabel (ids are global) and no push transposes (the partitioned path serves bothE
// BFS, which is symmetric, and pull-only gathers).
int assemble_partition(const tgo_edges* e, int64_t n_global, int64_t lo, int64_t hi,
                       const tgo_load_opts* opts, int64_t hard_limit, const int32_t* layout, HostGraph& g,
                       int threads, std::string& err) {
    g = HostGraph();
    const int64_t n = hi - lo, m = e->m;
    if (lo < 0 || hi > n_global || n <= 0 || n_global >= INT32_MAX) { err = "invalid partition range"; return TGO_E_INVALID; }
    g.n = n;
    g.scope = opts->scope;
    g.has_weight = opts->weight_key != 0 && e->weight != nullptr;
    g.titan_id.resize(n);
    for (int64_t v = 0; v < n; ++v) g.titan_id[v] = (lo + v + 1) << 3;
    std::atomic<bool> bad{false};
    parallel_for(m, threads, [&](int64_t a, int64_t b, int) {
        for (int64_t k = a; k < b; ++k)
            if (e->src[k] < 0 || e->src[k] >= n_global || e->dst[k] < 0 || e->dst[k] >= n_global) { bad = true; return; }
    });
    if (bad) { err = "edge endpoint out of range"; return TGO_E_INVALID; }
    const bool cap = opts->apply_cap && opts->n_labels == 0 && opts->scope != TGO_SCOPE_BOTH_E;
    const int64_t limit = cap ? hard_limit : INT64_MAX;
    auto build_dir = [&](bool out_dir, std::vector<int64_t>& off, std::vector<uint64_t>& keys) {
        rows_by_owner(m, out_dir ? e->src : e->dst, out_dir ? e->dst : e->src, lo, hi, threads, off, keys);
    };
    if (m >= (int64_t(1) << 32)) { err = "more than 2^32 edges per load"; return TGO_E_UNSUPPORTED; }
    std::vector<int64_t> off_o, off_i;
    std::vector<uint64_t> keys_o, keys_i;
    build_dir(true, off_o, keys_o);
    build_dir(false, off_i, keys_i);
    std::vector<int64_t> ko(n + 1, 0), ki(n + 1, 0);
    int64_t truncated = 0;
    for (int64_t v = 0; v < n; ++v) {
        const int64_t a = off_o[v + 1] - off_o[v], b = off_i[v + 1] - off_i[v];
        if (limit != INT64_MAX && a + b >= limit) ++truncated;
        const int64_t ka = std::min(a, limit);
        ko[v + 1] = ko[v] + ka;
        ki[v + 1] = ki[v] + std::min(b, limit - ka);
    }
    g.truncated = truncated;
    auto fill = [&](const std::vector<int64_t>& off, const std::vector<uint64_t>& keys,
                    const std::vector<int64_t>& koff, HostCsr& c) {
        c.off = koff;
        c.adj.resize(koff[n]);
        if (g.has_weight) c.w.resize(koff[n]);
        parallel_for(n, threads, [&](int64_t a, int64_t b, int) {
            for (int64_t v = a; v < b; ++v)
                for (int64_t j = 0; j < koff[v + 1] - koff[v]; ++j) {
                    const uint64_t key = keys[off[v] + j];
                    c.adj[koff[v] + j] = static_cast<int32_t>(key >> 32);
                    if (g.has_weight) c.w[koff[v] + j] = e->weight[key & 0xFFFFFFFFULL];
                }
        });
    };
    fill(off_o, keys_o, ko, g.out);
    std::vector<uint64_t>().swap(keys_o);
    fill(off_i, keys_i, ki, g.in);
    g.has_transpose = false;
    if (layout) {   // owned rows move inside [lo, hi); neighbours take their owners' layout
        g.perm.resize(n);
        std::vector<uint8_t> seen(n, 0);
        for (int64_t v = 0; v < n; ++v) {
            const int64_t p = static_cast<int64_t>(layout[lo + v]) - lo;
            if (p < 0 || p >= n || seen[p]) { err = "layout is not a permutation of the owned range"; return TGO_E_INVALID; }
            seen[p] = 1;
            g.perm[v] = static_cast<int32_t>(p);
        }
        permute_graph(g, [layout](int32_t u) { return layout[u]; }, threads);
    }
    // push view of a cut single-direction scope (assemble_partition_device): u pushes to v iff
    // u survived in v's cut pull list, whichever rank owns v
    if (cap && m) {
        const bool pull_out = opts->scope == TGO_SCOPE_IN_E;
        const int32_t* prow = pull_out ? e->src : e->dst;
        const int32_t* pnbr = pull_out ? e->dst : e->src;
        std::vector<int64_t> dout(n_global, 0), din(n_global, 0);
        for (int64_t k = 0; k < m; ++k) { ++dout[e->src[k]]; ++din[e->dst[k]]; }
        std::vector<int64_t> kept(n_global);
        bool any = false;
        for (int64_t v = 0; v < n_global; ++v) {
            const int64_t a = dout[v], b = din[v];
            any = any || a + b > limit;
            const int64_t ka = std::min(a, limit);
            kept[v] = pull_out ? ka : std::min(b, limit - ka);
        }
        if (any) {
            const std::vector<int64_t>& len = pull_out ? dout : din;
            std::vector<uint8_t> dropped(m, 0);
            std::vector<std::array<int64_t, 3>> cut;       // (pull row, neighbour, edge) of the cut rows
            for (int64_t k = 0; k < m; ++k)
                if (kept[prow[k]] < len[prow[k]]) cut.push_back({prow[k], pnbr[k], k});
            std::sort(cut.begin(), cut.end());
            for (size_t i = 0, j = 0; i < cut.size(); ++i) {
                j = (i > 0 && cut[i][0] == cut[i - 1][0]) ? j + 1 : 0;
                if (static_cast<int64_t>(j) >= kept[cut[i][0]]) dropped[cut[i][2]] = 1;
            }
            std::vector<std::array<int64_t, 3>> push;      // (push row, target, edge), layout ids
            for (int64_t k = 0; k < m; ++k)
                if (pnbr[k] >= lo && pnbr[k] < hi && !dropped[k])
                    push.push_back({layout ? layout[pnbr[k]] - lo : pnbr[k] - lo, layout ? layout[prow[k]] : prow[k], k});
            std::sort(push.begin(), push.end());
            HostCsr& pt = g.push_t;
            pt.off.assign(n + 1, 0);
            pt.adj.resize(push.size());
            if (g.has_weight) pt.w.resize(push.size());
            for (size_t i = 0; i < push.size(); ++i) {
                ++pt.off[push[i][0] + 1];
                pt.adj[i] = static_cast<int32_t>(push[i][1]);
                if (g.has_weight) pt.w[i] = e->weight[push[i][2]];
            }
            for (int64_t v = 0; v < n; ++v) pt.off[v + 1] += pt.off[v];
            g.has_transpose = true;
        }
    }
    return TGO_OK;
}

// ------------------------------------------------------------------ 1-D partition from rows
// The multi-GPU load from the edgestore (tgo_load_partition_rows): rank `rank` holds the rows
// of its live vertices, decoded with the cut already applied in column order (decode_rows:
// QueryContainer.java:28,122 over ColumnValueStore.java:47-69 — the one-GPU rule, per row).
// Global ids are slots: the i-th live row of rank r is r * S + i; slots past a rank's live
// count are entry-less padding.  slot_vid holds every rank's live Titan ids at their slots
// (padding: negative).  Entries whose other endpoint is no live vertex anywhere are dropped,
// as on one GPU (a vertex that never executes sends nothing, VertexState.java:103-137).
int assemble_partition_rows(RowStaging& st, const std::vector<int64_t>& slot_vid, int64_t S, int rank,
                            HostGraph& g, int threads, std::string& err) {
    g = HostGraph();
    const int64_t count = static_cast<int64_t>(st.vid.size()), lo = static_cast<int64_t>(rank) * S;
    if (count > S || static_cast<int64_t>(slot_vid.size()) < lo + S || slot_vid.size() >= size_t(INT32_MAX)) {
        err = "partition slots out of range";
        return TGO_E_INVALID;
    }
    g.n = S;
    g.scope = st.opts.scope;
    g.has_weight = st.opts.weight_key != 0;
    g.weight_dt = TGO_DT_INTEGER;
    g.ghost = st.ghost; g.truncated = st.truncated; g.skipped = st.skipped;
    g.titan_id.assign(static_cast<size_t>(S), 0);
    std::copy(st.vid.begin(), st.vid.end(), g.titan_id.begin());
    IdMap map;
    map.build(slot_vid);
    std::vector<int32_t> dense(st.other.size());
    parallel_for(static_cast<int64_t>(st.other.size()), threads, [&](int64_t a, int64_t b, int) {
        for (int64_t k = a; k < b; ++k) dense[k] = st.other[k] < 0 ? -1 : map.find(st.other[k]);
    });
    std::vector<int64_t> co(S + 1, 0), ci(S + 1, 0);
    for (int64_t v = 0; v < count; ++v) {
        int64_t a = 0, b = 0;
        for (int64_t k = st.row_begin[v]; k < st.row_begin[v + 1]; ++k) {
            if (dense[k] < 0) continue;
            if (st.dir[k] == 0) ++a; else ++b;
        }
        co[v + 1] = a; ci[v + 1] = b;
    }
    for (int64_t v = 0; v < S; ++v) { co[v + 1] += co[v]; ci[v + 1] += ci[v]; }
    g.out.off = co; g.in.off = ci;
    g.out.adj.resize(co[S]); g.in.adj.resize(ci[S]);
    if (g.has_weight) { g.out.w.resize(co[S]); g.in.w.resize(ci[S]); }
    parallel_for(count, threads, [&](int64_t a0, int64_t b0, int) {
        for (int64_t v = a0; v < b0; ++v) {
            int64_t a = co[v], b = ci[v];
            for (int64_t k = st.row_begin[v]; k < st.row_begin[v + 1]; ++k) {   // column order kept
                if (dense[k] < 0) continue;
                if (st.dir[k] == 0) {
                    g.out.adj[a] = dense[k];
                    if (g.has_weight) g.out.w[a] = st.w[k];
                    ++a;
                } else {
                    g.in.adj[b] = dense[k];
                    if (g.has_weight) g.in.w[b] = st.w[k];
                    ++b;
                }
            }
        }
    });
    (void)lo;
    st = RowStaging();
    return TGO_OK;
}

// tgo_part_layout for a rows partition: the owned slots grouped by half-octave of their kept
// entries (padding last), as global ids in [lo, lo + n).
void partition_rows_layout(const HostGraph& g, int64_t lo, int32_t* layout_local) {
    std::vector<int32_t> order;
    degree_group_order(g.n, [&](int64_t v) {
        return (g.out.off[v + 1] - g.out.off[v]) + (g.in.off[v + 1] - g.in.off[v]);
    }, order);
    for (int64_t v = 0; v < g.n; ++v) layout_local[v] = static_cast<int32_t>(lo + order[v]);
}

// Owned rows move inside [lo, lo + n) and neighbours take their owners' layout (the
// all-gathered layout of every rank), as assemble_partition does for an edge list.
int apply_partition_layout(HostGraph& g, int64_t lo, const int32_t* layout, int threads, std::string& err) {
    const int64_t n = g.n;
    g.perm.resize(n);
    std::vector<uint8_t> seen(n, 0);
    for (int64_t v = 0; v < n; ++v) {
        const int64_t p = static_cast<int64_t>(layout[lo + v]) - lo;
        if (p < 0 || p >= n || seen[p]) { err = "layout is not a permutation of the owned range"; return TGO_E_INVALID; }
        seen[p] = 1;
        g.perm[v] = static_cast<int32_t>(p);
    }
    permute_graph(g, [layout](int32_t u) { return layout[u]; }, threads);
    return TGO_OK;
}

// The push view of a cut single-direction scope needs the pull lists of EVERY rank: pull entry
// (v <- u) of owned row v becomes push entry (u -> v) at u's owner.  pairs: owner-major, two
// int64 per entry {(u - owner * S) << 32 | (lo + v), weight}; counts[p] = entries for rank p.
void partition_pull_pairs(const HostGraph& g, int64_t lo, int64_t S, int world, std::vector<int64_t>& counts,
                          std::vector<int64_t>& pairs) {
    const HostCsr& pull = g.scope == TGO_SCOPE_IN_E ? g.out : g.in;
    const int64_t n = g.n;
    counts.assign(world, 0);
    for (int64_t k = 0; k < static_cast<int64_t>(pull.adj.size()); ++k) ++counts[pull.adj[k] / S];
    std::vector<int64_t> pos(world + 1, 0);
    for (int p = 0; p < world; ++p) pos[p + 1] = pos[p] + counts[p];
    pairs.assign(static_cast<size_t>(2 * pos[world]), 0);
    for (int64_t v = 0; v < n; ++v)
        for (int64_t k = pull.off[v]; k < pull.off[v + 1]; ++k) {
            const int64_t u = pull.adj[k], owner = u / S, at = pos[owner]++;
            pairs[2 * at] = ((u - owner * S) << 32) | (lo + v);
            pairs[2 * at + 1] = pull.w.empty() ? 0 : pull.w[k];
        }
}

// The push rows of the owned slots from the pairs every rank sent here (partition_pull_pairs),
// each row ordered by (target, weight).
void partition_push_from_pairs(HostGraph& g, const int64_t* pairs, int64_t npairs) {
    std::vector<std::pair<int64_t, int64_t>> e(static_cast<size_t>(npairs));
    for (int64_t i = 0; i < npairs; ++i) e[i] = {pairs[2 * i], pairs[2 * i + 1]};
    std::sort(e.begin(), e.end());
    HostCsr& pt = g.push_t;
    pt = HostCsr();
    pt.off.assign(g.n + 1, 0);
    pt.adj.resize(static_cast<size_t>(npairs));
    if (g.has_weight) pt.w.resize(static_cast<size_t>(npairs));
    for (int64_t i = 0; i < npairs; ++i) {
        ++pt.off[(e[i].first >> 32) + 1];
        pt.adj[i] = static_cast<int32_t>(e[i].first & 0xFFFFFFFFLL);
        if (g.has_weight) pt.w[i] = static_cast<int32_t>(e[i].second);
    }
    for (int64_t v = 0; v < g.n; ++v) pt.off[v + 1] += pt.off[v];
    g.has_transpose = true;
}

// ------------------------------------------------------------------ CSR-adaptive blocks
// Greedy partition of rows into blocks of <= tile entries and <= max_rows rows
// (CSR-Adaptive, Greathouse & Daga SC'14); rows longer than `tile` become "long rows"
// split into tile-sized chunks whose partial sums are added in chunk order.
void build_row_blocks(const std::vector<int64_t>& off, int64_t tile, int64_t max_rows,
                      std::vector<int64_t>& blk, std::vector<int64_t>& chunk_row,
                      std::vector<int64_t>& chunk_beg, std::vector<int64_t>& chunk_end,
                      std::vector<int64_t>& long_row, std::vector<int64_t>& long_chunk) {
    const int64_t n = static_cast<int64_t>(off.size()) - 1;
    blk.clear(); chunk_row.clear(); chunk_beg.clear(); chunk_end.clear();
    long_row.clear(); long_chunk.clear();
    blk.push_back(0);
    long_chunk.push_back(0);
    int64_t r = 0;
    while (r < n) {
        const int64_t d = off[r + 1] - off[r];
        if (d > tile) {
            // long row: an empty short block marks its position, chunks carry the work
            long_row.push_back(r);
            for (int64_t s = off[r]; s < off[r + 1]; s += tile) {
                chunk_row.push_back(r);
                chunk_beg.push_back(s);
                chunk_end.push_back(std::min(off[r + 1], s + tile));
            }
            long_chunk.push_back(static_cast<int64_t>(chunk_row.size()));
            ++r;
            blk.push_back(r);   // block [r-1, r) is a long row: skipped by the short kernel
            continue;
        }
        int64_t e = r, nnz = 0;
        while (e < n && e - r < max_rows) {
            const int64_t de = off[e + 1] - off[e];
            if (de > tile || nnz + de > tile) break;
            nnz += de;
            ++e;
        }
        r = e;
        blk.push_back(r);
    }
}

// Source-sorted tiles (engine.hpp kPackShift): every CSR-adaptive tile's (and long-row
// chunk's) entries are re-ordered by source and packed as (source << 12 | slot), slot = the
// entry's position in the tile.  Lanes of one wave instruction then read neighbouring
// sources — shared 128-byte lines are fetched once — and the gathered values are written
// back to their slot, so the row sums keep the tile's row order.
bool pack_tiles(const std::vector<int64_t>& off, std::vector<int32_t>& adj, const std::vector<int64_t>& blk,
                const std::vector<int64_t>& cbeg, const std::vector<int64_t>& cend, int64_t tile, int threads,
                int shift) {
    if (shift < 1 || shift > 20 || tile > (int64_t(1) << shift)) return false;
    // shift 12: the word stays a non-negative int32 (kernels read it signed); wider slot spaces
    // use all 32 bits (their kernels read it as uint32)
    const int64_t src_limit = shift == kPackShift ? (int64_t(1) << (31 - shift)) : (int64_t(1) << (32 - shift));
    for (int32_t u : adj)
        if (u < 0 || u >= src_limit) return false;
    const int64_t nblk = static_cast<int64_t>(blk.size()) - 1, nch = static_cast<int64_t>(cbeg.size());
    auto pack_range = [&](int64_t b, int64_t e, std::vector<uint32_t>& tmp) {
        tmp.resize(static_cast<size_t>(e - b));
        for (int64_t k = b; k < e; ++k)
            tmp[k - b] = (static_cast<uint32_t>(adj[k]) << shift) | static_cast<uint32_t>(k - b);
        std::sort(tmp.begin(), tmp.end());
        for (int64_t k = b; k < e; ++k) adj[k] = static_cast<int32_t>(tmp[k - b]);
    };
    threads = std::max(1, threads);
    std::vector<std::thread> th;
    for (int t = 0; t < threads; ++t)
        th.emplace_back([&, t] {
            std::vector<uint32_t> tmp;
            for (int64_t b = t; b < nblk; b += threads) {
                const int64_t s0 = off[blk[b]], s1 = off[blk[b + 1]];
                if (s1 - s0 <= tile) pack_range(s0, s1, tmp);       // longer: a long row, packed per chunk
            }
            for (int64_t c = t; c < nch; c += threads) pack_range(cbeg[c], cend[c], tmp);
        });
    for (auto& x : th) x.join();
    return true;
}

// ------------------------------------------------------------------ weight-sorted push lists
// Light/heavy delta-stepping (delta.hip): every vertex's push entries (the push view of the
// loaded scope: the explicit transpose when the cap made lists asymmetric, both lists for
// bothE) in one list sorted by (weight, target) — the light entries of any bucket width are a
// prefix.  An entry without the weight property (kMissingWeight = INT32_MIN) sorts first,
// so the first light relaxation reports it.  A min over the list does not depend on order.
void weight_sorted_push(const HostGraph& g, HostCsr& ws, int threads) {
    const int64_t n = g.n;
    std::vector<const HostCsr*> lists;
    if (g.has_transpose) lists = {&g.push_t};
    else if (g.scope == TGO_SCOPE_IN_E) lists = {&g.in};
    else if (g.scope == TGO_SCOPE_OUT_E) lists = {&g.out};
    else lists = {&g.out, &g.in};
    ws.off.assign(n + 1, 0);
    for (int64_t v = 0; v < n; ++v) {
        int64_t d = 0;
        for (const HostCsr* c : lists) d += c->off[v + 1] - c->off[v];
        ws.off[v + 1] = ws.off[v] + d;
    }
    ws.adj.assign(static_cast<size_t>(ws.off[n]), 0);
    ws.w.assign(static_cast<size_t>(ws.off[n]), 0);
    // rows in small dynamic chunks: the degree-grouped order puts the hubs first, and a static
    // split left one thread sorting all of them (8.2 s for the capped RMAT-24 graph)
    parallel_dynamic(n, std::max(1, threads), 256, [&](int64_t lo, int64_t hi) {
        std::vector<std::pair<int32_t, int32_t>> buf;
        for (int64_t v = lo; v < hi; ++v) {
            buf.clear();
            for (const HostCsr* c : lists)
                for (int64_t k = c->off[v]; k < c->off[v + 1]; ++k) buf.emplace_back(c->w[k], c->adj[k]);
            std::sort(buf.begin(), buf.end());
            int64_t o = ws.off[v];
            for (const auto& e : buf) { ws.w[o] = e.first; ws.adj[o] = e.second; ++o; }
        }
    });
}

// ------------------------------------------------------------------ cache-blocked gather
// ColdBlocks layout (engine.hpp).  Rows are split over `threads` contiguous ranges; pass 1
// counts every row's hot entries and cold pieces per segment (per-thread segment totals),
// pass 2 writes the hot CSR and scatters the cold runs into their segment, rows in order
// (a thread's rows follow the previous thread's rows in every segment).
bool build_cold_blocks(const std::vector<int64_t>& off, const std::vector<int32_t>& adj, int64_t n_src,
                       int64_t hot, int64_t seg, int64_t tile, int64_t max_pieces, int threads, bool pack,
                       HostColdBlocks& hc, int64_t win) {
    const int64_t n = static_cast<int64_t>(off.size()) - 1;
    if (hot <= 0 || seg <= 0 || n_src <= hot || n <= 0) return false;
    if (win < 0 || win > 65536 || win > hot) win = 0;       // the device build's rule (pr_layout.hip)
    const int64_t nseg = (n_src - hot + seg - 1) / seg;
    threads = std::max(1, std::min<int>(threads, static_cast<int>(std::max<int64_t>(1, n / 4096))));
    hc.hot = hot;
    hc.seg = seg;
    std::vector<int64_t> hcount(n), npc(n), wcount(n, 0);
    std::vector<std::vector<int64_t>> tpieces(threads, std::vector<int64_t>(nseg, 0)),
        tentries(threads, std::vector<int64_t>(nseg, 0));
    // A row's cold entries grouped by segment (stable: list order inside a segment).  Lists
    // are sorted by internal id after the relabel, so the runs are normally contiguous.
    auto cold_runs = [&](int64_t r, std::vector<std::pair<int64_t, int32_t>>& buf) {
        buf.clear();
        bool sorted = true;
        int64_t last = -1;
        for (int64_t k = off[r]; k < off[r + 1]; ++k) {
            const int32_t u = adj[k];
            if (u < hot) continue;
            const int64_t sg = (u - hot) / seg;
            if (sg < last) sorted = false;
            last = sg;
            buf.emplace_back(sg, u);
        }
        if (!sorted)
            std::stable_sort(buf.begin(), buf.end(), [](const auto& a, const auto& b) { return a.first < b.first; });
    };
    auto range = [&](int t) { return std::make_pair(n * t / threads, n * (t + 1) / threads); };
    {
        std::vector<std::thread> th;
        for (int t = 0; t < threads; ++t)
            th.emplace_back([&, t] {
                std::vector<std::pair<int64_t, int32_t>> buf;
                const auto [lo, hi] = range(t);
                for (int64_t r = lo; r < hi; ++r) {
                    int64_t h = 0, wc = 0;
                    for (int64_t k = off[r]; k < off[r + 1]; ++k) {
                        h += adj[k] < hot && adj[k] >= win;
                        wc += adj[k] < win;
                    }
                    hcount[r] = h;
                    wcount[r] = wc;
                    cold_runs(r, buf);
                    int64_t pcs = 0;
                    for (size_t i = 0; i < buf.size();) {
                        size_t j = i;
                        while (j < buf.size() && buf[j].first == buf[i].first) ++j;
                        const int64_t c = static_cast<int64_t>(j - i);
                        const int64_t p = (c + tile - 1) / tile;
                        tpieces[t][buf[i].first] += p;
                        tentries[t][buf[i].first] += c;
                        pcs += p;
                        i = j;
                    }
                    npc[r] = pcs;
                }
            });
        for (auto& x : th) x.join();
    }
    hc.hoff.assign(n + 1, 0);
    hc.cptr.assign(n + 1, 0);
    int64_t acc = 0;
    for (int64_t r = 0; r < n; ++r) { hc.hoff[r + 1] = hc.hoff[r] + hcount[r]; acc += npc[r]; }
    hc.win = win;
    if (win > 0) {
        hc.woff.assign(n + 1, 0);
        for (int64_t r = 0; r < n; ++r) hc.woff[r + 1] = hc.woff[r] + wcount[r];
        hc.widx.assign(static_cast<size_t>(hc.woff[n]), 0);
    }
    if (acc >= (int64_t(1) << 31)) return false;
    hc.crow.clear();
    for (int64_t r = 0; r < n; ++r) {
        hc.cptr[r + 1] = hc.cptr[r] + static_cast<uint32_t>(npc[r]);
        if (npc[r]) hc.crow.push_back(static_cast<int32_t>(r));
    }
    const int64_t npieces = acc;
    // bases: segment-major, then thread order inside a segment
    std::vector<int64_t> seg_pbase(nseg + 1, 0), seg_ebase(nseg + 1, 0);
    std::vector<std::vector<int64_t>> pbase(threads, std::vector<int64_t>(nseg)), ebase(threads, std::vector<int64_t>(nseg));
    {
        int64_t pp = 0, ee = 0;
        for (int64_t sg = 0; sg < nseg; ++sg) {
            seg_pbase[sg] = pp;
            seg_ebase[sg] = ee;
            for (int t = 0; t < threads; ++t) {
                pbase[t][sg] = pp; ebase[t][sg] = ee;
                pp += tpieces[t][sg]; ee += tentries[t][sg];
            }
        }
        seg_pbase[nseg] = pp;
        seg_ebase[nseg] = ee;
    }
    hc.hadj.assign(static_cast<size_t>(hc.hoff[n]), 0);
    hc.cadj.assign(static_cast<size_t>(seg_ebase[nseg]), 0);
    hc.poff.assign(npieces + 1, 0);
    hc.cpid.assign(npieces, 0);
    {
        std::vector<std::thread> th;
        for (int t = 0; t < threads; ++t)
            th.emplace_back([&, t] {
                std::vector<std::pair<int64_t, int32_t>> buf;
                std::vector<int64_t> pc = pbase[t], ec = ebase[t];
                const auto [lo, hi] = range(t);
                for (int64_t r = lo; r < hi; ++r) {
                    int64_t h = hc.hoff[r], wq = win > 0 ? hc.woff[r] : 0;
                    for (int64_t k = off[r]; k < off[r + 1]; ++k) {
                        if (adj[k] < win) hc.widx[wq++] = static_cast<uint16_t>(adj[k]);
                        else if (adj[k] < hot) hc.hadj[h++] = adj[k];
                    }
                    cold_runs(r, buf);
                    int64_t slot = hc.cptr[r];
                    for (size_t i = 0; i < buf.size();) {
                        const int64_t sg = buf[i].first;
                        size_t j = i;
                        while (j < buf.size() && buf[j].first == sg) ++j;
                        for (size_t q = i; q < j; q += static_cast<size_t>(tile)) {
                            const size_t qe = std::min(j, q + static_cast<size_t>(tile));
                            hc.poff[pc[sg]] = ec[sg];
                            hc.cpid[slot++] = static_cast<int32_t>(pc[sg]++);
                            for (size_t z = q; z < qe; ++z) hc.cadj[ec[sg]++] = buf[z].second;
                        }
                        i = j;
                    }
                }
            });
        for (auto& x : th) x.join();
    }
    hc.poff[npieces] = seg_ebase[nseg];
    // cold blocks: greedy per segment (<= tile entries, <= max_pieces pieces), segment-major.
    // The block list is cut into 8 contiguous ranges of equal entry counts, range x for XCD
    // x: every XCD walks consecutive segments in order (a dense segment may be shared by two
    // neighbouring XCDs, each caching its slice) and the XCDs finish together.
    hc.bbeg.clear();
    hc.bend.clear();
    hc.bsrc.clear();
    for (int64_t sg = 0; sg < nseg; ++sg) {
        int64_t p = seg_pbase[sg];
        while (p < seg_pbase[sg + 1]) {
            int64_t e = p;
            while (e < seg_pbase[sg + 1] && e - p < max_pieces && hc.poff[e + 1] - hc.poff[p] <= tile) ++e;
            hc.bbeg.push_back(p);
            hc.bend.push_back(e);
            hc.bsrc.push_back(static_cast<int32_t>(hot + sg * seg));
            p = e;
        }
    }
    const int64_t nb = static_cast<int64_t>(hc.bbeg.size());
    // Source-sorted, packed cold tiles: (source - segment base) << kPackShift | slot.
    if (pack && seg <= (int64_t(1) << (31 - kPackShift)) && tile <= (int64_t(1) << kPackShift)) {
        std::vector<std::thread> th;
        for (int t = 0; t < threads; ++t)
            th.emplace_back([&, t] {
                std::vector<uint32_t> tmp;
                for (int64_t b = t; b < nb; b += threads) {
                    const int64_t s0 = hc.poff[hc.bbeg[b]], s1 = hc.poff[hc.bend[b]];
                    tmp.resize(static_cast<size_t>(s1 - s0));
                    for (int64_t k = s0; k < s1; ++k)
                        tmp[k - s0] = (static_cast<uint32_t>(hc.cadj[k] - hc.bsrc[b]) << kPackShift) |
                                      static_cast<uint32_t>(k - s0);
                    std::sort(tmp.begin(), tmp.end());
                    for (int64_t k = s0; k < s1; ++k) hc.cadj[k] = static_cast<int32_t>(tmp[k - s0]);
                }
            });
        for (auto& x : th) x.join();
        hc.cpacked = true;
    }
    hc.xblk.resize(nb);
    for (int64_t b = 0; b < nb; ++b) hc.xblk[b] = static_cast<int32_t>(b);
    const int64_t total = hc.poff[npieces];
    hc.max_xcd_blocks = 0;
    int64_t b = 0;
    for (int x = 0; x < 8; ++x) {
        hc.xbase.b[x] = b;
        const int64_t target = total * (x + 1) / 8;
        while (b < nb && (x == 7 || hc.poff[hc.bend[b]] <= target)) ++b;
        hc.max_xcd_blocks = std::max<int64_t>(hc.max_xcd_blocks, b - hc.xbase.b[x]);
    }
    hc.xbase.b[8] = static_cast<int64_t>(hc.xblk.size());
    return true;
}

}  // namespace tgo

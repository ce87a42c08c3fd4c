// decode.hip — device decode of scanned edgestore rows: the per-row rules of
// VertexJobConverter.process (key filter, ghost check, user-edge slice, QueryContainer limit;
// VertexJobConverter.java:109-171) and EdgeSerializer.parseRelation for every kept entry
// (EdgeSerializer.java:73-166), on the GPU, with the same codec as the host path (codec.hpp,
// compiled here as __host__ __device__).
//
// Per batch: the StaticArrayEntryList arrays are uploaded; `dec_rows` (one thread per row)
// classifies the row and finds its user-edge slice [0x60, 0x80) by binary search over the
// column-sorted entries' first bytes; an exclusive scan of the kept counts gives every kept
// entry an output slot; `dec_entries` (one thread per kept entry, its row found by binary
// search over the scan) decodes it.  The staging arrays come back to the host, which keeps
// the same RowStaging as the host decoder: parity is checked by running both paths.
// Byte work over HBM: the batch's row bytes are read once, 13 bytes per kept entry written.
#define TGO_HD __host__ __device__
#include <cstring>
#include <hip/hip_runtime.h>
#include "codec.hpp"
#include "engine.hpp"

namespace tgo {
namespace {

constexpr int kBlock = 256;
inline unsigned grid_for(int64_t n) {
    int64_t g = (n + kBlock - 1) / kBlock;
    return static_cast<unsigned>(std::max<int64_t>(1, std::min<int64_t>(g, 65536)));
}

enum : int32_t { kRowLive = 0, kRowSkipped = 1, kRowGhost = 2, kRowBadId = -1, kRowEmpty = -2, kRowBadFirst = -3 };

__device__ __forceinline__ int64_t ent_start(const int64_t* lv, int64_t e0, int64_t k) {
    return k == e0 ? 0 : static_cast<int64_t>(static_cast<uint64_t>(lv[k - 1]) >> 32);
}

__global__ void __launch_bounds__(kBlock) dec_rows(const int64_t* __restrict__ keys, const int64_t* __restrict__ eb,
        const int64_t* __restrict__ bb, const uint8_t* __restrict__ bytes, const int64_t* __restrict__ lv,
        int64_t nrows, int pb, int64_t limit, int64_t* __restrict__ vid_out, int64_t* __restrict__ first_out,
        int64_t* __restrict__ keep_out, int32_t* __restrict__ status, uint8_t* __restrict__ rep_out,
        unsigned long long* __restrict__ truncated) {
    for (int64_t r = blockIdx.x * static_cast<int64_t>(blockDim.x) + threadIdx.x; r <= nrows;
         r += static_cast<int64_t>(gridDim.x) * blockDim.x) {
        if (r == nrows) { keep_out[nrows] = 0; continue; }
        keep_out[r] = 0;
        first_out[r] = 0;
        rep_out[r] = 0;
        const int64_t vid = key_to_vertex_id(keys[r], pb);
        vid_out[r] = vid;
        if (vid & 1) { status[r] = kRowSkipped; continue; }          // key filter: Invisible (:156-162)
        const int64_t sfx = vid & 7;
        if (sfx != 0 && sfx != 2 && sfx != 4) { status[r] = kRowBadId; continue; }
        const bool is_rep = sfx == 2 && vid != canonical_vertex_id(vid, pb);
        const int64_t e0 = eb[r], e1 = eb[r + 1];
        if (e1 <= e0) { status[r] = kRowEmpty; continue; }
        const uint8_t* base = bytes + bb[r];
        if (!is_rep) {                                               // ghost check (:131-137)
            Cursor c{base, static_cast<size_t>(static_cast<uint64_t>(lv[e0]) >> 32), 0};
            RelType rt;
            if (!read_relation_type(c, rt)) { status[r] = kRowBadFirst; continue; }
            if (rt.is_edge || rt.type_id != kVertexExistsId) { status[r] = kRowGhost; continue; }
        }
        // user-edge slice [0x60, 0x80): entries are column-sorted, so two lower bounds
        int64_t lo = e0, hi = e1;
        while (lo < hi) { const int64_t m = (lo + hi) >> 1; if (base[ent_start(lv, e0, m)] < 0x60) lo = m + 1; else hi = m; }
        const int64_t first = lo;
        hi = e1;
        while (lo < hi) { const int64_t m = (lo + hi) >> 1; if (base[ent_start(lv, e0, m)] < 0x80) lo = m + 1; else hi = m; }
        const int64_t cnt = lo - first;
        if (cnt >= limit) atomicAdd(truncated, 1ULL);                // TRUNCATED_ENTRY_LISTS (:125)
        status[r] = kRowLive;
        rep_out[r] = is_rep ? 1 : 0;
        vid_out[r] = is_rep ? canonical_vertex_id(vid, pb) : vid;
        first_out[r] = first;
        keep_out[r] = cnt < limit ? cnt : limit;
    }
}

__global__ void __launch_bounds__(kBlock) dec_entries(const int64_t* __restrict__ bb, const uint8_t* __restrict__ bytes,
        const int64_t* __restrict__ eb, const int64_t* __restrict__ lv, const int64_t* __restrict__ first,
        const int64_t* __restrict__ koff, int64_t nrows, int64_t total, PlanView plan, int pb, int weighted,
        int64_t* __restrict__ other, uint8_t* __restrict__ dir, int32_t* __restrict__ w, uint8_t* __restrict__ sel,
        int32_t* __restrict__ err, int64_t* __restrict__ wv) {
    for (int64_t p = blockIdx.x * static_cast<int64_t>(blockDim.x) + threadIdx.x; p < total;
         p += static_cast<int64_t>(gridDim.x) * blockDim.x) {
        int64_t lo = 0, hi = nrows;                                  // row r: koff[r] <= p < koff[r+1]
        while (lo < hi) { const int64_t m = (lo + hi + 1) >> 1; if (koff[m] <= p) lo = m; else hi = m - 1; }
        const int64_t r = lo;
        const int64_t e0 = eb[r];
        const int64_t k = first[r] + (p - koff[r]);
        const int64_t s = ent_start(lv, e0, k);
        const int64_t e = static_cast<int64_t>(static_cast<uint64_t>(lv[k]) >> 32);
        const int64_t vp = lv[k] & 0x7FFFFFFF;
        DecodedEdge de{};
        const DecodeResult dr = e >= s ? decode_edge(bytes + bb[r] + s, static_cast<size_t>(e - s),
                                                     static_cast<size_t>(vp), plan, de)
                                       : DecodeResult::kError;
        if (dr == DecodeResult::kSkip) { sel[p] = 0; continue; }
        if (dr != DecodeResult::kOk) {
            atomicOr(err, dr == DecodeResult::kUnsupported ? 2 : 1);
            sel[p] = 0;
            continue;
        }
        sel[p] = 1;
        other[p] = is_partitioned_vertex(de.other, pb) ? canonical_vertex_id(de.other, pb) : de.other;  // :89
        dir[p] = static_cast<uint8_t>(de.dir);
        w[p] = weighted ? (de.has_weight ? de.weight : kMissingWeight) : 1;
        if (wv) wv[p] = de.has_weight ? de.weight64 : 0;          // wide keys (Long / Double)
    }
}

// Compaction of the kept entries (sel) into staging order: the exclusive scan ks of sel
// places entry p at ks[p]; a row's kept entries start at ks[koff[r]].
__global__ void sel_to_i64(const uint8_t* __restrict__ sel, int64_t total, int64_t* __restrict__ out) {
    for (int64_t p = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; p <= total; p += (int64_t)gridDim.x * blockDim.x)
        out[p] = p < total ? sel[p] : 0;
}
// wv (wide weight keys): the values follow their entries, and the weight column becomes the
// entry's staged position (base + q) — the index into the graph's value table.
__global__ void compact_entries(const uint8_t* __restrict__ sel, const int64_t* __restrict__ ks, int64_t total,
                                const int64_t* __restrict__ other, const uint8_t* __restrict__ dir,
                                const int32_t* __restrict__ w, int64_t* __restrict__ c_other,
                                uint8_t* __restrict__ c_dir, int32_t* __restrict__ c_w,
                                const int64_t* __restrict__ wv, int64_t* __restrict__ c_wv, int64_t base) {
    for (int64_t p = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; p < total; p += (int64_t)gridDim.x * blockDim.x) {
        if (!sel[p]) continue;
        const int64_t q = ks[p];
        c_other[q] = other[p];
        c_dir[q] = dir[p];
        c_w[q] = (wv && w[p] != kMissingWeight) ? static_cast<int32_t>(base + q) : w[p];
        if (wv) c_wv[q] = wv[p];
    }
}
__global__ void row_kept_begin(const int64_t* __restrict__ koff, const int64_t* __restrict__ ks, int64_t nrows,
                               int64_t* __restrict__ out) {
    for (int64_t r = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; r <= nrows; r += (int64_t)gridDim.x * blockDim.x)
        out[r] = ks[koff[r]];
}

}  // namespace

void DecodeScratch::release() {
    keys.release(); eb.release(); bb.release(); bytes.release(); lv.release(); vid.release(); first.release();
    keep.release(); koff.release(); status.release(); rep.release(); other.release(); dir.release(); w.release();
    sel.release(); err.release(); trunc.release(); plan_labels.release(); plan_keys.release(); plan_kdts.release();
    plan_dts.release(); ks.release(); c_other.release(); c_dir.release(); c_w.release(); wv.release(); c_wv.release();
    bytes_used = lv_used = 0;
    if (cub_tmp) (void)hipFree(cub_tmp);
    cub_tmp = nullptr;
    cub_bytes = 0;
}

// One work block of scanned rows: validated, its entry bytes and limit/valuePos words
// appended to device buffers (no host copy), its keys and rebased row offsets to the host
// staging; the device decodes every block in one pass at tgo_finish_load.
int stage_rows_raw(RowStaging& st, const tgo_rows* rows, const tgo_schema* schema, const tgo_load_opts* opts,
                   DecodeScratch& ds, hipStream_t stream, std::string& err) {
    HostPlan hp;
    if (int rc = build_plan(schema, opts, hp, err)) return rc;
    std::vector<uint8_t> pb;                              // the plan's bytes: batches must agree
    auto put = [&](const void* p, size_t n) { pb.insert(pb.end(), static_cast<const uint8_t*>(p), static_cast<const uint8_t*>(p) + n); };
    put(hp.label_bytes.data(), hp.label_bytes.size());
    put(hp.key_ids.data(), hp.key_ids.size() * 8);
    put(hp.key_dts.data(), hp.key_dts.size());
    put(hp.dts.data(), hp.dts.size());
    const bool first = !st.active;
    if (int rc = staging_begin(st, opts, err)) return rc;
    if (first) { st.plan = hp; st.plan_bytes = pb; }
    else if (pb != st.plan_bytes) { err = "tgo_schema differs between row batches"; return TGO_E_INVALID; }
    // a new load starts from empty device buffers even when its first block has no rows (an
    // earlier load aborted mid-batch may have left the counters behind)
    if (first) ds.bytes_used = ds.lv_used = 0;
    const int64_t nrows = rows->nrows;
    if (nrows == 0) return TGO_OK;
    const int64_t nent = rows->row_entry_begin[nrows] - rows->row_entry_begin[0];
    const int64_t nbytes = rows->row_byte_begin[nrows] - rows->row_byte_begin[0];
    if (nent < 0 || nbytes < 0) { err = "row offsets decrease"; return TGO_E_INVALID; }
    st.raw_keys.insert(st.raw_keys.end(), rows->row_keys, rows->row_keys + nrows);
    for (int64_t r = 1; r <= nrows; ++r) {
        const int64_t de = rows->row_entry_begin[r] - rows->row_entry_begin[r - 1];
        const int64_t db = rows->row_byte_begin[r] - rows->row_byte_begin[r - 1];
        if (de < 0 || db < 0) { err = "row offsets decrease"; return TGO_E_INVALID; }
        st.raw_eb.push_back(st.raw_eb.back() + de);
        st.raw_bb.push_back(st.raw_bb.back() + db);
    }
    hipError_t e = ds.lv.append(rows->entry_limit_valpos + rows->row_entry_begin[0], nent, ds.lv_used, stream);
    if (e == hipSuccess) e = ds.bytes.append(rows->entry_bytes + rows->row_byte_begin[0], nbytes, ds.bytes_used, stream);
    if (e == hipSuccess) e = hipStreamSynchronize(stream);    // the caller may reuse its buffers on return
    if (e != hipSuccess) { err = hipGetErrorString(e); return e == hipErrorOutOfMemory ? TGO_E_OOM : TGO_E_HIP; }
    ds.lv_used += nent;
    ds.bytes_used += nbytes;
    return TGO_OK;
}

int decode_staged_raw(RowStaging& st, int pb, int64_t hard_limit, DecodeScratch& ds, hipStream_t stream,
                      std::string& err, bool device_entries) {
    const HostPlan& hp = st.plan;
    const tgo_load_opts* opts = &st.opts;
    const bool typed = !st.labels.empty();
    const int64_t limit = (opts->apply_cap && !typed && opts->scope != TGO_SCOPE_BOTH_E) ? hard_limit : INT64_MAX;
    const int64_t nrows = static_cast<int64_t>(st.raw_keys.size());
    if (nrows == 0) return TGO_OK;
    const tgo_rows staged{nrows, st.raw_keys.data(), st.raw_eb.data(), st.raw_bb.data(), nullptr, nullptr};
    const tgo_rows* rows = &staged;
    const int64_t nent = rows->row_entry_begin[nrows], nbytes = rows->row_byte_begin[nrows];
    if (nent != ds.lv_used || nbytes != ds.bytes_used) { err = "raw staging out of step"; return TGO_E_STATE; }
    hipError_t e = hipSuccess;
#define DEC_TRY(x) do { e = (x); if (e != hipSuccess) { err = hipGetErrorString(e); return e == hipErrorOutOfMemory ? TGO_E_OOM : TGO_E_HIP; } } while (0)
    for (DBuf<int64_t>* b : {&ds.keys, &ds.eb, &ds.bb, &ds.vid, &ds.first, &ds.keep, &ds.koff}) DEC_TRY(b->grow(nrows + 1));
    DEC_TRY(ds.status.grow(nrows + 1));
    DEC_TRY(ds.rep.grow(nrows + 1));
    DEC_TRY(ds.err.grow(1));
    DEC_TRY(ds.trunc.grow(1));
    DEC_TRY(ds.plan_labels.grow(static_cast<int64_t>(hp.label_bytes.size()) + 1));
    DEC_TRY(ds.plan_keys.grow(static_cast<int64_t>(hp.key_ids.size()) + 1));
    DEC_TRY(ds.plan_kdts.grow(static_cast<int64_t>(hp.key_dts.size()) + 1));
    DEC_TRY(ds.plan_dts.grow(static_cast<int64_t>(hp.dts.size()) + 1));
    auto h2d = [&](void* d, const void* h, size_t n) { return n ? hipMemcpyAsync(d, h, n, hipMemcpyHostToDevice, stream) : hipSuccess; };
    DEC_TRY(h2d(ds.keys.p, rows->row_keys, nrows * 8));
    DEC_TRY(h2d(ds.eb.p, rows->row_entry_begin, (nrows + 1) * 8));
    DEC_TRY(h2d(ds.bb.p, rows->row_byte_begin, (nrows + 1) * 8));
    DEC_TRY(h2d(ds.plan_labels.p, hp.label_bytes.data(), hp.label_bytes.size()));
    DEC_TRY(h2d(ds.plan_keys.p, hp.key_ids.data(), hp.key_ids.size() * 8));
    DEC_TRY(h2d(ds.plan_kdts.p, hp.key_dts.data(), hp.key_dts.size()));
    DEC_TRY(h2d(ds.plan_dts.p, hp.dts.data(), hp.dts.size()));
    DEC_TRY(hipMemsetAsync(ds.err.p, 0, sizeof(int32_t), stream));
    DEC_TRY(hipMemsetAsync(ds.trunc.p, 0, sizeof(unsigned long long), stream));
    dec_rows<<<grid_for(nrows + 1), kBlock, 0, stream>>>(ds.keys.p, ds.eb.p, ds.bb.p, ds.bytes.p, ds.lv.p, nrows, pb, limit, ds.vid.p,
                                                         ds.first.p, ds.keep.p, ds.status.p, ds.rep.p, ds.trunc.p);
    DEC_TRY(hipGetLastError());
    DEC_TRY(scan_exclusive_i64(ds.cub_tmp, ds.cub_bytes, ds.keep.p, ds.koff.p, nrows + 1, stream));
    std::vector<int64_t> vid(nrows), koff(nrows + 1);
    std::vector<int32_t> status(nrows);
    std::vector<uint8_t> rep(nrows);
    unsigned long long trunc = 0;
    DEC_TRY(hipMemcpyAsync(koff.data(), ds.koff.p, (nrows + 1) * 8, hipMemcpyDeviceToHost, stream));
    DEC_TRY(hipMemcpyAsync(vid.data(), ds.vid.p, nrows * 8, hipMemcpyDeviceToHost, stream));
    DEC_TRY(hipMemcpyAsync(status.data(), ds.status.p, nrows * 4, hipMemcpyDeviceToHost, stream));
    DEC_TRY(hipMemcpyAsync(rep.data(), ds.rep.p, nrows, hipMemcpyDeviceToHost, stream));
    DEC_TRY(hipMemcpyAsync(&trunc, ds.trunc.p, sizeof(trunc), hipMemcpyDeviceToHost, stream));
    DEC_TRY(hipStreamSynchronize(stream));
    for (int64_t r = 0; r < nrows; ++r) {
        if (status[r] >= 0) continue;
        err = status[r] == kRowBadId ? "row key has an unrecognized vertex id type"
            : status[r] == kRowEmpty ? "row without entries" : "malformed first column";
        return TGO_E_CODEC;
    }
    const int64_t total = koff[nrows];
    DEC_TRY(ds.other.grow(total + 1));
    DEC_TRY(ds.w.grow(total + 1));
    DEC_TRY(ds.dir.grow(total + 1));
    DEC_TRY(ds.sel.grow(total + 1));
    const PlanView plan{reinterpret_cast<const LabelPlan*>(ds.plan_labels.p), hp.n_labels,
                        static_cast<int32_t>(hp.key_ids.size()), ds.plan_keys.p, ds.plan_kdts.p, ds.plan_dts.p, hp.weight_key};
    const bool wide = opts->weight_key != 0 && wide_weight_dt(hp.weight_dt);
    if (wide) DEC_TRY(ds.wv.grow(total + 1));
    if (total > 0) {
        dec_entries<<<grid_for(total), kBlock, 0, stream>>>(ds.bb.p, ds.bytes.p, ds.eb.p, ds.lv.p, ds.first.p, ds.koff.p, nrows, total,
                                                             plan, pb, opts->weight_key != 0 ? 1 : 0, ds.other.p, ds.dir.p,
                                                             ds.w.p, ds.sel.p, ds.err.p, wide ? ds.wv.p : nullptr);
        DEC_TRY(hipGetLastError());
    }
    // kept entries compacted on the device, in staging order
    DEC_TRY(ds.ks.grow(total + 1));
    DEC_TRY(ds.c_other.grow(total + 1));
    DEC_TRY(ds.c_dir.grow(total + 1));
    DEC_TRY(ds.c_w.grow(total + 1));
    if (wide) DEC_TRY(ds.c_wv.grow(total + 1));
    DEC_TRY(ds.keep.grow(std::max(nrows, total) + 1));
    const int64_t e_base = static_cast<int64_t>(st.other.size());     // staged position of the first kept entry
    if (wide && e_base + total >= INT32_MAX) { err = "wide weights: more than 2^31 - 1 staged entries"; return TGO_E_UNSUPPORTED; }
    sel_to_i64<<<grid_for(total + 1), kBlock, 0, stream>>>(ds.sel.p, total, ds.keep.p);
    DEC_TRY(hipGetLastError());
    DEC_TRY(scan_exclusive_i64(ds.cub_tmp, ds.cub_bytes, ds.keep.p, ds.ks.p, total + 1, stream));
    if (total > 0) {
        compact_entries<<<grid_for(total), kBlock, 0, stream>>>(ds.sel.p, ds.ks.p, total, ds.other.p, ds.dir.p, ds.w.p,
                                                                ds.c_other.p, ds.c_dir.p, ds.c_w.p, wide ? ds.wv.p : nullptr,
                                                                wide ? ds.c_wv.p : nullptr, e_base);
        DEC_TRY(hipGetLastError());
    }
    row_kept_begin<<<grid_for(nrows + 1), kBlock, 0, stream>>>(ds.koff.p, ds.ks.p, nrows, ds.keep.p);
    DEC_TRY(hipGetLastError());
    std::vector<int64_t> rk(nrows + 1);
    int32_t eflag = 0;
    DEC_TRY(hipMemcpyAsync(&eflag, ds.err.p, 4, hipMemcpyDeviceToHost, stream));
    DEC_TRY(hipMemcpyAsync(rk.data(), ds.keep.p, (nrows + 1) * 8, hipMemcpyDeviceToHost, stream));
    DEC_TRY(hipStreamSynchronize(stream));
    if (eflag) {
        err = (eflag & 1) ? "malformed edge entry" : "inline property of a key missing from the schema";
        return (eflag & 1) ? TGO_E_CODEC : TGO_E_UNSUPPORTED;
    }
    const int64_t kept = rk[nrows];
    const size_t e0 = st.other.size();
    if (device_entries && e0 == 0 && !st.d_other.present()) {
        // the compacted entries stay where they are: the device assembly reads them in place
        st.d_other.own(ds.c_other.p, kept); ds.c_other.p = nullptr; ds.c_other.cap = 0;
        st.d_dir.own(ds.c_dir.p, kept); ds.c_dir.p = nullptr; ds.c_dir.cap = 0;
        st.d_w.own(ds.c_w.p, kept); ds.c_w.p = nullptr; ds.c_w.cap = 0;
        if (wide) { st.d_wv.own(ds.c_wv.p, kept); ds.c_wv.p = nullptr; ds.c_wv.cap = 0; }
    } else if (kept > 0) {
        st.other.resize(e0 + static_cast<size_t>(kept));
        st.dir.resize(e0 + static_cast<size_t>(kept));
        st.w.resize(e0 + static_cast<size_t>(kept));
        DEC_TRY(hipMemcpyAsync(st.other.data() + e0, ds.c_other.p, kept * 8, hipMemcpyDeviceToHost, stream));
        DEC_TRY(hipMemcpyAsync(st.dir.data() + e0, ds.c_dir.p, kept, hipMemcpyDeviceToHost, stream));
        DEC_TRY(hipMemcpyAsync(st.w.data() + e0, ds.c_w.p, kept * 4, hipMemcpyDeviceToHost, stream));
        if (wide) {
            st.wv.resize(e0 + static_cast<size_t>(kept));
            DEC_TRY(hipMemcpyAsync(st.wv.data() + e0, ds.c_wv.p, kept * 8, hipMemcpyDeviceToHost, stream));
        }
        DEC_TRY(hipStreamSynchronize(stream));
    }
#undef DEC_TRY
    if (st.d_other.present() && st.d_other.n != kept) { err = "staged entries out of step"; return TGO_E_STATE; }
    std::vector<int64_t>().swap(st.raw_keys);
    st.raw_eb.assign(1, 0);
    st.raw_bb.assign(1, 0);
    st.truncated += static_cast<int64_t>(trunc);
    // rows in order, exactly as the host decoder stages them
    for (int64_t r = 0; r < nrows; ++r) {
        if (status[r] == kRowSkipped) { ++st.skipped; continue; }
        if (status[r] == kRowGhost) { ++st.ghost; continue; }
        st.vid.push_back(vid[r]);
        st.rep.push_back(rep[r]);
        st.n_rep += rep[r];
        st.row_begin.push_back(static_cast<int64_t>(e0) + rk[r + 1]);
    }
    return TGO_OK;
}

int staging_entries_to_host(RowStaging& st, hipStream_t stream, std::string& err) {
    if (!st.d_other.present()) return TGO_OK;
    const int64_t E = st.d_other.n;
    hipError_t e = hipStreamSynchronize(stream);
    st.other.resize(static_cast<size_t>(E));
    st.dir.resize(static_cast<size_t>(E));
    st.w.resize(static_cast<size_t>(E));
    if (E > 0 && e == hipSuccess) e = copy_chunked(st.other.data(), st.d_other.p, E * 8, hipMemcpyDeviceToHost);
    if (E > 0 && e == hipSuccess) e = copy_chunked(st.dir.data(), st.d_dir.p, E, hipMemcpyDeviceToHost);
    if (E > 0 && e == hipSuccess) e = copy_chunked(st.w.data(), st.d_w.p, E * 4, hipMemcpyDeviceToHost);
    if (st.d_wv.present()) {
        st.wv.resize(static_cast<size_t>(E));
        if (E > 0 && e == hipSuccess) e = copy_chunked(st.wv.data(), st.d_wv.p, E * 8, hipMemcpyDeviceToHost);
    }
    if (e != hipSuccess) { err = hipGetErrorString(e); return TGO_E_HIP; }
    st.d_other.reset();
    st.d_dir.reset();
    st.d_w.reset();
    st.d_wv.reset();
    return TGO_OK;
}

}  // namespace tgo

// part_driver.cpp — the partitioned multi-source BFS sweep driven from C++.
//
// titan_amd/distributed.py drives the partitioned (multi-GPU) programs from Python: every
// level is a local step through the C-ABI plus an RCCL collective through torch.distributed,
// and each level pays Python dispatch and several host round trips.  tgo_part_msbfs_run runs
// the same protocol (dense level: in-place all-gather of the owned frontier masks + pull;
// sparse level: push into candidate masks, packed (owner-local id, mask) pairs in a fixed-
// capacity or sized all-to-all, settle; level counts all-reduced on the device) as one C++
// loop over an exchange object:
//   * tgo_exchange_rccl_*  : RCCL over xGMI on the ctx stream (production, one process per GPU);
//   * tgo_exchange_local_group : ranks as threads of one process on one device (tests: the
//     same loop at world 2 / 4 on a one-GPU box), collectives as device-to-device copies
//     between the ranks' buffers at a barrier.
// The reference has no multi-process OLAP executor (FulgoraGraphComputer.java:117-311 is one
// JVM); this is the multi-GPU form of ShortestDistanceVertexProgram with unit weights
// (ShortestDistanceVertexProgram.java:96-130) over bothE.
#include <algorithm>
#include <chrono>
#include <condition_variable>
#include <cstdlib>
#include <cstring>
#include <memory>
#include <mutex>
#include <string>
#include <vector>

#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include "engine.hpp"
#include "trace.hpp"
#include "../../include/titan_gpu_olap_part.h"

// Exchange: the four collectives the sweep needs, all on device buffers, ordered on `s`.
struct tgo_exchange {
    int world = 1, rank = 0;
    virtual ~tgo_exchange() = default;
    // buf holds `world` slices of `bytes` (this rank's at rank * bytes); every rank's slice
    // ends up in every buffer
    virtual int all_gather(void* buf, size_t bytes, hipStream_t s) = 0;
    // send / recv hold `world` blocks of `bytes`: block r of send goes to rank r, block p of
    // recv comes from rank p
    virtual int all_to_all(const void* send, void* recv, size_t bytes, hipStream_t s) = 0;
    // per-peer byte counts and offsets (host arrays of `world`)
    virtual int all_to_allv(const void* send, const size_t* sb, const size_t* so, void* recv, const size_t* rb,
                            const size_t* ro, hipStream_t s) = 0;
    // element-wise reduction over the ranks, in place (op: kRedSum / kRedMin / kRedMax)
    enum { kRedSum = 0, kRedMin = 1, kRedMax = 2 };
    virtual int all_reduce(int64_t* buf, size_t count, int op, hipStream_t s) = 0;
    int all_reduce_sum(int64_t* buf, size_t count, hipStream_t s) { return all_reduce(buf, count, kRedSum, s); }
    // a rank leaving the protocol early releases the peers waiting on it (in-process group)
    virtual void abort() {}
    std::string err;
    int64_t* pinned = nullptr;      // host counts of the driver (pinned once per exchange)
    int64_t* host_counts() {
        if (!pinned && hipHostMalloc(reinterpret_cast<void**>(&pinned), 8 * sizeof(int64_t), hipHostMallocDefault) != hipSuccess)
            pinned = nullptr;
        return pinned;
    }
    void release_pinned() {
        if (pinned) (void)hipHostFree(pinned);
        pinned = nullptr;
    }
};

namespace {

using tgo::copy_chunked;

// ------------------------------------------------------------------ RCCL (production)
struct RcclExchange : tgo_exchange {
    ncclComm_t comm = nullptr;
    bool aborted = false;
    ~RcclExchange() override {
        if (comm) (void)ncclCommDestroy(comm);
        release_pinned();
    }
    // A rank that fails between collectives (a local step's error, a HIP error) aborts its own
    // communicator and refuses further use here, so it returns the error at once instead of
    // entering another collective.  ncclCommAbort does NOT notify the peers: a peer already
    // in, or about to enter, a collective with this rank waits until its launcher ends it.
    // One process per GPU under torch.distributed.run provides that: the failed rank exits
    // with an error and the launcher terminates the rest of the group.
    void abort() override {
        if (comm) (void)ncclCommAbort(comm);
        comm = nullptr;
        aborted = true;
    }
    int check(ncclResult_t r, const char* what) {
        if (r == ncclSuccess) return TGO_OK;
        err = std::string(what) + ": " + ncclGetErrorString(r);
        return TGO_E_HIP;
    }
    bool usable() {
        if (!aborted) return true;
        err = "RCCL exchange aborted by an earlier failure";
        return false;
    }
    int all_gather(void* buf, size_t bytes, hipStream_t s) override {
        if (!usable()) return TGO_E_COMM;
        if (world == 1) return TGO_OK;
        char* b = static_cast<char*>(buf);
        return check(ncclAllGather(b + rank * bytes, b, bytes, ncclChar, comm, s), "ncclAllGather");
    }
    int all_to_all(const void* send, void* recv, size_t bytes, hipStream_t s) override {
        if (!usable()) return TGO_E_COMM;
        if (world == 1) return copy_on(send, recv, bytes, s);
        return check(ncclAllToAll(send, recv, bytes, ncclChar, comm, s), "ncclAllToAll");
    }
    int all_to_allv(const void* send, const size_t* sb, const size_t* so, void* recv, const size_t* rb,
                    const size_t* ro, hipStream_t s) override {
        if (!usable()) return TGO_E_COMM;
        if (world == 1) return copy_on(static_cast<const char*>(send) + so[0], static_cast<char*>(recv) + ro[0], sb[0], s);
        int rc = check(ncclGroupStart(), "ncclGroupStart");
        for (int p = 0; !rc && p < world; ++p) {
            if (sb[p]) rc = check(ncclSend(static_cast<const char*>(send) + so[p], sb[p], ncclChar, p, comm, s), "ncclSend");
            if (!rc && rb[p]) rc = check(ncclRecv(static_cast<char*>(recv) + ro[p], rb[p], ncclChar, p, comm, s), "ncclRecv");
        }
        const int rc2 = check(ncclGroupEnd(), "ncclGroupEnd");
        return rc ? rc : rc2;
    }
    int all_reduce(int64_t* buf, size_t count, int op, hipStream_t s) override {
        if (!usable()) return TGO_E_COMM;
        if (world == 1) return TGO_OK;
        const ncclRedOp_t o = op == kRedMin ? ncclMin : op == kRedMax ? ncclMax : ncclSum;
        return check(ncclAllReduce(buf, buf, count, ncclInt64, o, comm, s), "ncclAllReduce");
    }
    int copy_on(const void* src, void* dst, size_t bytes, hipStream_t s) {
        if (!bytes || src == dst) return TGO_OK;
        const hipError_t e = hipMemcpyAsync(dst, src, bytes, hipMemcpyDeviceToDevice, s);
        if (e == hipSuccess) return TGO_OK;
        err = hipGetErrorString(e);
        return TGO_E_HIP;
    }
};

// ------------------------------------------------------------------ in-process group (tests)
// Ranks are threads of one process; a collective is: finish the own stream, publish the
// buffer pointers, barrier, copy what this rank needs from the peers' buffers (device to
// device, own stream), finish, barrier (the peers' buffers may be reused afterwards).
struct LocalGroup {
    int world;
    std::mutex mu;
    std::condition_variable cv;
    int arrived = 0;
    long generation = 0;
    bool broken = false;
    struct Slot { const void* send; void* recv; const size_t* sb; const size_t* so; std::vector<int64_t> red; };
    std::vector<Slot> slot;
    explicit LocalGroup(int w) : world(w), slot(w) {}
    bool barrier() {
        std::unique_lock<std::mutex> lk(mu);
        if (broken) return false;
        const long gen = generation;
        if (++arrived == world) {
            arrived = 0;
            ++generation;
            cv.notify_all();
            return true;
        }
        const bool ok = cv.wait_for(lk, std::chrono::seconds(60), [&] { return generation != gen || broken; });
        if (!ok || broken) { broken = true; cv.notify_all(); return false; }
        return true;
    }
};

struct LocalExchange : tgo_exchange {
    std::shared_ptr<LocalGroup> g;
    ~LocalExchange() override { release_pinned(); }
    void abort() override {
        std::lock_guard<std::mutex> lk(g->mu);
        g->broken = true;
        g->cv.notify_all();
    }
    int fail_msg(const char* m) { err = m; return TGO_E_STATE; }
    int sync(hipStream_t s) {
        const hipError_t e = hipStreamSynchronize(s);
        if (e == hipSuccess) return TGO_OK;
        err = hipGetErrorString(e);
        return TGO_E_HIP;
    }
    int copy(void* dst, const void* src, size_t bytes, hipStream_t s) {
        if (!bytes || dst == src) return TGO_OK;
        const hipError_t e = hipMemcpyAsync(dst, src, bytes, hipMemcpyDeviceToDevice, s);
        if (e == hipSuccess) return TGO_OK;
        err = hipGetErrorString(e);
        return TGO_E_HIP;
    }
    template <class F>
    int collective(hipStream_t s, const LocalGroup::Slot& mine, F&& body) {
        int rc = sync(s);
        g->slot[rank] = mine;
        if (!g->barrier()) return fail_msg("local exchange: a rank failed or timed out");
        if (!rc) rc = body();
        if (!rc) rc = sync(s);
        if (!g->barrier()) return fail_msg("local exchange: a rank failed or timed out");
        return rc;
    }
    int all_gather(void* buf, size_t bytes, hipStream_t s) override {
        if (world == 1) return TGO_OK;                      // one rank: nothing to exchange (as RCCL)
        return collective(s, {buf, buf, nullptr, nullptr, {}}, [&]() -> int {
            for (int p = 0; p < world; ++p)
                if (p != rank) {
                    const char* src = static_cast<const char*>(g->slot[p].recv) + p * bytes;
                    if (int rc = copy(static_cast<char*>(buf) + p * bytes, src, bytes, s)) return rc;
                }
            return TGO_OK;
        });
    }
    int all_to_all(const void* send, void* recv, size_t bytes, hipStream_t s) override {
        if (world == 1) return copy(recv, send, bytes, s);
        return collective(s, {send, recv, nullptr, nullptr, {}}, [&]() -> int {
            for (int p = 0; p < world; ++p) {
                const char* src = static_cast<const char*>(g->slot[p].send) + rank * bytes;
                if (int rc = copy(static_cast<char*>(recv) + p * bytes, src, bytes, s)) return rc;
            }
            return TGO_OK;
        });
    }
    int all_to_allv(const void* send, const size_t* sb, const size_t* so, void* recv, const size_t* rb,
                    const size_t* ro, hipStream_t s) override {
        if (world == 1) {
            if (sb[0] != rb[0]) return fail_msg("local exchange: all_to_allv sizes do not match");
            return copy(static_cast<char*>(recv) + ro[0], static_cast<const char*>(send) + so[0], rb[0], s);
        }
        return collective(s, {send, recv, sb, so, {}}, [&]() -> int {
            for (int p = 0; p < world; ++p) {
                const LocalGroup::Slot& q = g->slot[p];
                if (q.sb[rank] != rb[p]) return fail_msg("local exchange: all_to_allv sizes do not match");
                const char* src = static_cast<const char*>(q.send) + q.so[rank];
                if (int rc = copy(static_cast<char*>(recv) + ro[p], src, rb[p], s)) return rc;
            }
            return TGO_OK;
        });
    }
    int all_reduce(int64_t* buf, size_t count, int op, hipStream_t s) override {
        if (world == 1) return TGO_OK;
        std::vector<int64_t> mine(count);
        int rc = sync(s);
        if (!rc) {
            const hipError_t e = hipMemcpy(mine.data(), buf, count * sizeof(int64_t), hipMemcpyDeviceToHost);
            if (e != hipSuccess) { err = hipGetErrorString(e); rc = TGO_E_HIP; }
        }
        g->slot[rank] = {nullptr, nullptr, nullptr, nullptr, mine};
        if (!g->barrier()) return fail_msg("local exchange: a rank failed or timed out");
        std::vector<int64_t> sum(mine);
        for (int p = 0; p < world; ++p) {
            if (p == rank) continue;
            for (size_t i = 0; i < count && i < g->slot[p].red.size(); ++i) {
                const int64_t v = g->slot[p].red[i];
                sum[i] = op == kRedMin ? std::min(sum[i], v) : op == kRedMax ? std::max(sum[i], v) : sum[i] + v;
            }
        }
        if (!g->barrier()) return fail_msg("local exchange: a rank failed or timed out");
        if (rc) return rc;
        const hipError_t e = hipMemcpyAsync(buf, sum.data(), count * sizeof(int64_t), hipMemcpyHostToDevice, s);
        if (e != hipSuccess) { err = hipGetErrorString(e); return TGO_E_HIP; }
        return sync(s);          // sum is a local: the copy must finish before it goes away
    }
};

}  // namespace

extern "C" {

int tgo_exchange_rccl_id(uint8_t* id_out) {
    if (!id_out) return TGO_E_INVALID;
    ncclUniqueId id;
    if (ncclGetUniqueId(&id) != ncclSuccess) return TGO_E_HIP;
    std::memcpy(id_out, &id, sizeof(id));
    return TGO_OK;
}

int tgo_exchange_rccl_create(int32_t world, int32_t rank, const uint8_t* id, int32_t device, tgo_exchange** out) {
    if (!id || !out || world < 1 || rank < 0 || rank >= world) return TGO_E_INVALID;
    *out = nullptr;
    if (hipSetDevice(device) != hipSuccess) return TGO_E_HIP;
    auto x = std::make_unique<RcclExchange>();
    x->world = world;
    x->rank = rank;
    ncclUniqueId uid;
    std::memcpy(&uid, id, sizeof(uid));
    if (ncclCommInitRank(&x->comm, world, uid, rank) != ncclSuccess) return TGO_E_HIP;
    *out = x.release();
    return TGO_OK;
}

int tgo_exchange_local_group(int32_t world, tgo_exchange** ranks_out) {
    if (!ranks_out || world < 1 || world > 64) return TGO_E_INVALID;
    auto g = std::make_shared<LocalGroup>(world);
    for (int r = 0; r < world; ++r) {
        auto* x = new LocalExchange();
        x->world = world;
        x->rank = r;
        x->g = g;
        ranks_out[r] = x;
    }
    return TGO_OK;
}

void tgo_exchange_destroy(tgo_exchange* x) { delete x; }

const char* tgo_exchange_last_error(const tgo_exchange* x) { return x ? x->err.c_str() : "null exchange"; }

}  // extern "C"

namespace tgo {

// ctx accessors (api.cpp): the ctx stream, partition dimensions, error text
hipStream_t part_stream(tgo_ctx* ctx);
int part_dims(tgo_ctx* ctx, int64_t* n_local, int64_t* lo, int64_t* n_global, int64_t* entries);
int part_fail(tgo_ctx* ctx, int code, const std::string& msg);
int part_scratch(tgo_ctx* ctx, void** p, int64_t bytes, int slot);
int64_t* part_dcounts_of(tgo_ctx* ctx);
// this rank's slice of the candidate words bypasses the pack / exchange (ORed in directly by the
// settle); (nullptr, -1) turns it off
void part_ms_bypass(tgo_ctx* ctx, uint64_t* cand_global, int self);
// the next settle sums its new frontier's push entries per source into out (one-shot)
int part_ms_settle_sums(tgo_ctx* ctx, int64_t* out, bool count_only = false);
// the next push writes its owned targets straight into next (bypass on); nullptr cancels
void part_ms_own_next(tgo_ctx* ctx, uint64_t* next);
// device words to the host through the mapped counter page (no stream synchronisation)
int part_read_words(tgo_ctx* ctx, const int64_t* dev, int count, int64_t* out);
int part_sssp_relax_dev(tgo_ctx* ctx, int64_t thr, int32_t nranks, int64_t* send, int64_t* sizes);
int part_sssp_header_fold(tgo_ctx* ctx, const int64_t* own, const int64_t* recv, int nranks, int64_t* out);
int part_sssp_split(tgo_ctx* ctx, int64_t delta, bool* on);
bool part_sssp_devloop(const tgo_ctx* ctx);
int part_sssp_dev_relax(tgo_ctx* ctx, int32_t nranks, int64_t* send, int64_t* sizes, int64_t* fold);
int part_sssp_header_read(tgo_ctx* ctx, const int64_t* own, const int64_t* recv, int nranks, int64_t* out,
                          int64_t* words);
int part_sssp_dev_apply(tgo_ctx* ctx, const int64_t* recv, int64_t npairs);
int part_sssp_dev_extract(tgo_ctx* ctx, int64_t thr);
double ms_split_of(const tgo_ctx* ctx);
std::shared_ptr<void>& part_state_of(tgo_ctx* ctx);
int part_in_list(tgo_ctx* ctx, const int32_t** adj, int64_t* nnz);
int part_out_list(tgo_ctx* ctx, const int32_t** adj, int64_t* nnz);
bool ms_ghost_of(const tgo_ctx* ctx);
int part_pr_layout_of(tgo_ctx* ctx, int32_t* world, int64_t* hot, int64_t* span);
int part_upload(tgo_ctx* ctx, HostGraph& h, int64_t n_global, int64_t lo);
int part_rows_take(tgo_ctx* ctx, RowStaging& st, std::string& err);
void part_drop_staging(tgo_ctx* ctx);
int part_threads(const tgo_ctx* ctx);
void part_set_live(tgo_ctx* ctx, int64_t live);
template <class T>
int scratch(tgo_ctx* ctx, T*& p, int64_t count, int slot) {
    void* q = nullptr;
    const int rc = part_scratch(ctx, &q, count * static_cast<int64_t>(sizeof(T)), slot);
    p = static_cast<T*>(q);
    return rc;
}

}  // namespace tgo

using namespace tgo;

namespace {

// Host-side helpers shared by the loops: small global reductions through a device buffer.
struct Driver {
    tgo_ctx* ctx;
    tgo_exchange* x;
    hipStream_t st;
    int64_t* dbuf = nullptr;        // device scalars (8)
    int64_t* hc = nullptr;          // pinned host view
    int xfail(int code) { return part_fail(ctx, code, "exchange: " + x->err); }
    int hip(const char* what) { return part_fail(ctx, TGO_E_HIP, what); }
    // out[i] = op over the ranks of vals[i], i < k <= 8 (one round trip)
    int reduce(const int64_t* vals, int k, int op, int64_t* out) {
        for (int i = 0; i < k; ++i) hc[i] = vals[i];
        if (hipMemcpyAsync(dbuf, hc, k * sizeof(int64_t), hipMemcpyHostToDevice, st) != hipSuccess) return hip("reduce upload");
        if (int r = x->all_reduce(dbuf, static_cast<size_t>(k), op, st)) return xfail(r);
        return part_read_words(ctx, dbuf, k, out);
    }
};

int driver_open(tgo_ctx* ctx, tgo_exchange* x, const char* name, int slot, Driver& d, int64_t& nl, int64_t& lo,
                int64_t& ng, int64_t& ent) {
    int rc = part_dims(ctx, &nl, &lo, &ng, &ent);
    if (rc) return rc;
    if (static_cast<int64_t>(x->world) * nl != ng || lo != static_cast<int64_t>(x->rank) * nl)
        return part_fail(ctx, TGO_E_INVALID, std::string(name) + ": the exchange's world / rank do not match the partition");
    d.ctx = ctx;
    d.x = x;
    d.st = part_stream(ctx);
    if ((rc = scratch(ctx, d.dbuf, 8, slot))) return rc;
    d.hc = x->host_counts();
    if (!d.hc) return part_fail(ctx, TGO_E_HIP, std::string(name) + ": pinned counts");
    return TGO_OK;
}

}  // namespace

namespace {

// Ghost lists (part_ghost.hip), kept with the graph: which of this rank's rows every peer
// reads (send_row) and where each value received from a peer goes (recv_pos).  PageRank reads
// over its in-lists into the blocked gathered vector; the multi-source sweep over both lists
// into the global mask vector (position = global id).
struct PrGhost {
    int world = 0, rank = -1;
    int64_t nl = 0, hot = 0, span = 0;
    int32_t* send_row = nullptr;    // local rows this rank sends, peer-major
    int32_t* recv_pos = nullptr;    // gathered-vector position of every received value
    double* sbuf = nullptr;
    double* rbuf = nullptr;
    int64_t nsend = 0, nrecv = 0;
    std::vector<size_t> sb, so, rb, ro;   // byte counts / offsets per peer (doubles)
    ~PrGhost() {
        for (void* p : {static_cast<void*>(send_row), static_cast<void*>(recv_pos), static_cast<void*>(sbuf),
                        static_cast<void*>(rbuf)})
            if (p) (void)hipFree(p);
    }
};

int build_ghost(tgo_ctx* ctx, tgo_exchange* x, Driver& d, int64_t nl, int64_t hot, int64_t span, bool both_lists,
                PrGhost& gh) {
    const int W = x->world, R = x->rank;
    hipStream_t st = d.st;
    const int32_t *adj = nullptr, *adj2 = nullptr;
    int64_t nnz = 0, nnz2 = 0;
    int rc = part_in_list(ctx, &adj, &nnz);
    if (!rc && both_lists) rc = part_out_list(ctx, &adj2, &nnz2);
    if (rc) return rc;
    std::string err;
    int32_t* need = nullptr;
    std::vector<int64_t> need_count;
    if ((rc = ghost_needs(adj, nnz, adj2, nnz2, nl, R, W, &need, need_count, st, err))) return part_fail(ctx, rc, err);
    struct Free { void* p; ~Free() { if (p) (void)hipFree(p); } } free_need{need};
    int64_t nneed = 0;
    for (int64_t c : need_count) nneed += c;
    // counts to the owners, then the ids (as int32 bytes)
    int64_t* sizes = nullptr;
    if ((rc = scratch(ctx, sizes, 2 * W, both_lists ? 7 : 21))) return rc;
    if (hipMemcpyAsync(sizes, need_count.data(), W * sizeof(int64_t), hipMemcpyHostToDevice, st) != hipSuccess)
        return d.hip("ghost counts upload");
    if (int r = x->all_to_all(sizes, sizes + W, 8, st)) return d.xfail(r);
    std::vector<int64_t> gives(W);
    if (hipMemcpyAsync(gives.data(), sizes + W, W * sizeof(int64_t), hipMemcpyDeviceToHost, st) != hipSuccess ||
        hipStreamSynchronize(st) != hipSuccess)
        return d.hip("ghost counts read");
    int64_t ngive = 0;
    for (int64_t c : gives) ngive += c;
    gh.world = W; gh.rank = R; gh.nl = nl; gh.hot = hot; gh.span = span;
    gh.nsend = ngive;
    gh.nrecv = nneed;
    if (hipMalloc(&gh.send_row, std::max<int64_t>(ngive, 1) * 4) != hipSuccess ||
        hipMalloc(&gh.recv_pos, std::max<int64_t>(nneed, 1) * 4) != hipSuccess ||
        hipMalloc(&gh.sbuf, std::max<int64_t>(ngive, 1) * 8) != hipSuccess ||
        hipMalloc(&gh.rbuf, std::max<int64_t>(nneed, 1) * 8) != hipSuccess)
        return part_fail(ctx, TGO_E_OOM, "ghost buffers");
    std::vector<size_t> ib(W), io(W), gb(W), go(W);
    gh.sb.assign(W, 0); gh.so.assign(W, 0); gh.rb.assign(W, 0); gh.ro.assign(W, 0);
    size_t a = 0, b = 0;
    for (int p = 0; p < W; ++p) {
        ib[p] = static_cast<size_t>(need_count[p]) * 4; io[p] = a; a += ib[p];       // my needs, to owner p
        gb[p] = static_cast<size_t>(gives[p]) * 4; go[p] = b; b += gb[p];            // p's needs of my rows
        gh.rb[p] = static_cast<size_t>(need_count[p]) * 8; gh.ro[p] = io[p] * 2;      // values received from p
        gh.sb[p] = static_cast<size_t>(gives[p]) * 8; gh.so[p] = go[p] * 2;           // values sent to p
    }
    if (int r = x->all_to_allv(need, ib.data(), io.data(), gh.send_row, gb.data(), go.data(), st)) return d.xfail(r);
    if (hipError_t e = k_sub_i32(gh.send_row, ngive, static_cast<int32_t>(static_cast<int64_t>(R) * nl), st))
        return part_fail(ctx, TGO_E_HIP, hipGetErrorString(e));
    if (hipError_t e = k_gathered_pos(need, nneed, nl, span, hot, W, gh.recv_pos, st))
        return part_fail(ctx, TGO_E_HIP, hipGetErrorString(e));
    if (hipStreamSynchronize(st) != hipSuccess) return d.hip("ghost lists");
    return TGO_OK;
}

// the ghost lists a driver keeps with the graph (part_state_of): PageRank's and the sweep's
struct GhostCache {
    std::shared_ptr<PrGhost> pr, ms;
};
GhostCache& ghost_cache(tgo_ctx* ctx) {
    std::shared_ptr<void>& st = part_state_of(ctx);
    if (!st) st = std::make_shared<GhostCache>();
    return *static_cast<GhostCache*>(st.get());
}

}  // namespace

extern "C" int tgo_part_msbfs_run(tgo_ctx* ctx, tgo_exchange* x, const int64_t* seeds, int32_t nseeds, int32_t max_depth,
                                  double ms_alpha, int64_t fixed_bytes, int64_t* reached, int64_t* entries,
                                  int32_t* levels_out) {
    if (!ctx) return TGO_E_INVALID;
    if (!x || !seeds || nseeds < 1 || nseeds > TGO_MAX_SOURCES || max_depth < 0)
        return part_fail(ctx, TGO_E_INVALID, "tgo_part_msbfs_run: bad arguments");
    int64_t nl = 0, lo = 0, ng = 0, ent = 0;
    int rc = part_dims(ctx, &nl, &lo, &ng, &ent);
    if (rc) return rc;
    const int W = x->world;
    if (static_cast<int64_t>(W) * nl != ng || lo != static_cast<int64_t>(x->rank) * nl)
        return part_fail(ctx, TGO_E_INVALID, "tgo_part_msbfs_run: the exchange's world / rank do not match the partition");
    hipStream_t st = part_stream(ctx);
    auto xfail = [&](int code) { return part_fail(ctx, code, "exchange: " + x->err); };
    // scratch (ctx-owned, reused): two alternating global mask buffers, the candidate masks,
    // the pair buffers, the device counts and the split sizes
    uint64_t *g0 = nullptr, *g1 = nullptr, *cand = nullptr;
    int64_t *send = nullptr, *recv = nullptr, *dc = nullptr, *sizes = nullptr;
    const int64_t pairs_cap = 2 * ng + 2 * W;
    if ((rc = scratch(ctx, g0, ng, 0)) || (rc = scratch(ctx, g1, ng, 1)) || (rc = scratch(ctx, cand, ng, 2)) ||
        (rc = scratch(ctx, send, pairs_cap, 3)) || (rc = scratch(ctx, recv, pairs_cap, 4)) ||
        (rc = scratch(ctx, dc, 3 + 2 * TGO_MAX_SOURCES, 5)) || (rc = scratch(ctx, sizes, 2 * W, 6)))
        return rc;
    int64_t* const caller_dc = part_dcounts_of(ctx);       // restored at the end
    // the rank's own candidate words never travel: the packs skip its slice and the settles OR
    // it in (the Python reference driver keeps packing every slice)
    struct Bypass {
        tgo_ctx* c;
        ~Bypass() { part_ms_bypass(c, nullptr, -1); }
    } bypass{ctx};
    part_ms_bypass(ctx, cand, x->rank);
    uint64_t* glob[2] = {g0, g1};
    // no clearing per sweep (as the Python driver): the buffers start zero (part_scratch), a
    // level rewrites the active rows of the next mask and the entry-less tail stays zero, the
    // pack clears the candidate masks it reads, and a dense level's all-gather overwrites the
    // peers' slices before the pull reads them.  A failed sweep re-zeroes all three.
    auto rezero = [&]() {
        (void)hipMemsetAsync(g0, 0, ng * 8, st);
        (void)hipMemsetAsync(g1, 0, ng * 8, st);
        (void)hipMemsetAsync(cand, 0, ng * 8, st);
    };
    int64_t* hc = x->host_counts();                         // pinned host view of the counts (kept)
    if (!hc) return part_fail(ctx, TGO_E_HIP, "tgo_part_msbfs_run: pinned counts");
    // dense levels: the ghost exchange (only the masks this rank's lists read, lists built once
    // per graph) unless TGO_TUNE_MS_GHOST = 0 or a single rank
    PrGhost* gh = nullptr;
    if (W > 1 && ms_ghost_of(ctx)) {
        Driver d{ctx, x, st, dc, hc};
        std::shared_ptr<PrGhost>& cached = ghost_cache(ctx).ms;
        gh = cached.get();
        if (!gh || gh->world != W || gh->rank != x->rank || gh->nl != nl) {
            auto fresh = std::make_shared<PrGhost>();
            if ((rc = build_ghost(ctx, x, d, nl, 0, nl, true, *fresh))) { x->abort(); return rc; }
            cached = fresh;
            gh = fresh.get();
        }
    }
    // global counts: write local {a, b} to dc, all-reduce, read back (one sync)
    auto global2 = [&](int64_t a, int64_t b, int64_t* out) -> int {
        hc[0] = a; hc[1] = b;
        if (hipMemcpyAsync(dc, hc, 2 * sizeof(int64_t), hipMemcpyHostToDevice, st) != hipSuccess)
            return part_fail(ctx, TGO_E_HIP, "counts upload");
        if (int r = x->all_reduce_sum(dc, 2, st)) return xfail(r);
        if (hipMemcpyAsync(hc, dc, 2 * sizeof(int64_t), hipMemcpyDeviceToHost, st) != hipSuccess ||
            hipStreamSynchronize(st) != hipSuccess)
            return part_fail(ctx, TGO_E_HIP, "counts read");
        out[0] = hc[0]; out[1] = hc[1];
        return TGO_OK;
    };
    int64_t tot[2];
    if ((rc = global2(ent, 0, tot))) return rc;
    const int64_t total = tot[0];
    uint64_t* fr = glob[0] + lo;
    uint64_t* frn = glob[1] + lo;
    int64_t c[2];
    if ((rc = tgo_part_ms_begin(ctx, seeds, nseeds, fr, c))) return rc;
    int64_t g[2];
    if ((rc = global2(c[0], c[1], g))) return rc;
    int64_t nf = g[0], mf = g[1];
    // level counts stay on the device: the steps publish {next queue, its entries, own queue}
    if ((rc = tgo_part_device_counts(ctx, dc))) return rc;
    int levels = 0;
    // source split of the first dense level of a run (tgo_bfs_multi's rule and budget)
    const double split_frac = ms_split_of(ctx);
    const uint64_t full = nseeds == 64 ? ~0ULL : ((1ULL << nseeds) - 1ULL);
    int64_t* sc64 = dc + 3;                                 // 64 per-source sums (free during the sweep)
    auto read64 = [&](int64_t* host) -> int {
        if (int r = x->all_reduce_sum(sc64, 64, st)) return xfail(r);
        if (hipMemcpyAsync(host, sc64, 64 * sizeof(int64_t), hipMemcpyDeviceToHost, st) != hipSuccess ||
            hipStreamSynchronize(st) != hipSuccess)
            return part_fail(ctx, TGO_E_HIP, "per-source sums read");
        return TGO_OK;
    };
    // pack + exchange the candidate masks of a push (fixed slots when cap bounds them), then
    // hand the received pairs to `fixed_fn` / `pairs_fn`
    // The own slice never travels (part_ms_bypass): its slot / split is empty, the settle ORs
    // it in; with one rank nothing is exchanged at all.
    auto exchange = [&](int64_t entries, auto&& fixed_fn, auto&& pairs_fn) -> int {
        const int64_t cap = std::min<int64_t>(entries, nl);
        if (W == 1) {
            const int64_t none = 0;
            return pairs_fn(&none);
        }
        if (cap > 0 && static_cast<int64_t>(W) * (cap + 1) * 16 <= fixed_bytes) {
            if (int r = tgo_part_ms_pack_fixed(ctx, cand, W, cap, send)) return r;
            // equal slots known on the host; the own slot is neither sent nor received (its
            // header in recv zeroed so the settle reads no pairs from it)
            const size_t slot = static_cast<size_t>(cap + 1) * 16;
            std::vector<size_t> sb(W, slot), so(W);
            for (int p = 0; p < W; ++p) so[p] = static_cast<size_t>(p) * slot;
            sb[x->rank] = 0;
            if (hipMemsetAsync(reinterpret_cast<char*>(recv) + so[x->rank], 0, 16, st) != hipSuccess)
                return part_fail(ctx, TGO_E_HIP, "own slot header");
            if (int r = x->all_to_allv(send, sb.data(), so.data(), recv, sb.data(), so.data(), st)) return xfail(r);
            return fixed_fn(cap);
        }
        // sized pairs: split sizes on the device, one all-to-all of them, one host read
        if (int r = tgo_part_ms_pack_dev(ctx, cand, W, send, sizes)) return r;
        if (int r = x->all_to_all(sizes, sizes + W, 8, st)) return xfail(r);
        std::vector<int64_t> both(2 * W);
        if (hipMemcpyAsync(both.data(), sizes, 2 * W * sizeof(int64_t), hipMemcpyDeviceToHost, st) != hipSuccess ||
            hipStreamSynchronize(st) != hipSuccess) return part_fail(ctx, TGO_E_HIP, "split sizes read");
        std::vector<size_t> sb(W), so(W), rb(W), ro(W);
        std::vector<int64_t> rpairs(W);
        size_t a = 0, b = 0;
        for (int p = 0; p < W; ++p) {
            sb[p] = static_cast<size_t>(both[p]) * 8; so[p] = a; a += sb[p];
            rb[p] = static_cast<size_t>(both[W + p]) * 8; ro[p] = b; b += rb[p];
            rpairs[p] = both[W + p] / 2;
        }
        if (int r = x->all_to_allv(send, sb.data(), so.data(), recv, rb.data(), ro.data(), st)) return xfail(r);
        return pairs_fn(rpairs.data());
    };
    bool prev_dense = false;
    bool sums = false;
    for (int level = 0; level < max_depth && nf > 0; ++level) {
        const bool dense = static_cast<double>(mf) * ms_alpha > static_cast<double>(total);
        DevSpan span(st, "part.msbfs.level", {"level", level}, {"dense", dense ? 1 : 0});
        const bool first_dense = dense && !prev_dense;
        prev_dense = dense;
        const bool sums_ready = sums;   // the previous level's settle summed the per-source entries
        sums = false;
        if (dense) {
            uint64_t sparse = 0;
            int32_t with_cand = 0;
            if (first_dense && split_frac > 0.0) {
                // every source's exact push entries (all-reduced), the smallest within the budget
                // after a push level its settle summed them (part_ms_settle_sums)
                int64_t se[64];
                if (!sums_ready && (rc = tgo_part_ms_source_entries(ctx, fr, full, sc64))) break;
                if ((rc = read64(se))) break;
                int order[64];
                for (int r = 0; r < nseeds; ++r) order[r] = r;
                std::sort(order, order + nseeds, [&](int a, int b) { return se[a] < se[b]; });
                int64_t used = 0;
                for (int i = 0; i < nseeds; ++i) {
                    const int r = order[i];
                    if (static_cast<double>(used + se[r]) > split_frac * static_cast<double>(total)) break;
                    used += se[r];
                    sparse |= 1ULL << r;
                }
                if (sparse == full) sparse = 0;
                if (sparse && used > 0) {               // push the sparse sources' frontiers
                    if ((rc = tgo_part_ms_push_masked(ctx, fr, cand, sparse))) break;
                    rc = exchange(used,
                                  [&](int64_t cap) { return tgo_part_ms_or_fixed(ctx, recv, W, cap, frn); },
                                  [&](const int64_t* rp) { return tgo_part_ms_or_pairs(ctx, recv, rp, W, frn); });
                    if (rc) break;
                    with_cand = 1;
                }
            }
            if (gh) {                                   // ghosts: pack -> all-to-allv -> unpack into glob[0]
                const uint64_t* own = glob[0] + lo;
                if (k_pack_u64(own, gh->send_row, gh->nsend, reinterpret_cast<uint64_t*>(gh->sbuf), st) != hipSuccess) {
                    rc = part_fail(ctx, TGO_E_HIP, "ghost pack");
                    break;
                }
                if (int r = x->all_to_allv(gh->sbuf, gh->sb.data(), gh->so.data(), gh->rbuf, gh->rb.data(), gh->ro.data(), st)) {
                    rc = xfail(r);
                    break;
                }
                if (k_unpack_u64(reinterpret_cast<const uint64_t*>(gh->rbuf), gh->recv_pos, gh->nrecv, glob[0], st) !=
                    hipSuccess) {
                    rc = part_fail(ctx, TGO_E_HIP, "ghost unpack");
                    break;
                }
            } else if (int r = x->all_gather(glob[0], static_cast<size_t>(nl) * 8, st)) {
                rc = xfail(r);
                break;
            }
            if ((rc = tgo_part_ms_pull_split(ctx, level, glob[0], frn, sparse, with_cand, nullptr))) break;
        } else {
            part_ms_own_next(ctx, frn);                 // owned candidates straight into frn
            if ((rc = tgo_part_ms_push(ctx, level, fr, cand))) break;
            // the settle sums the per-source entries when the next level may pull (this
            // frontier's entries within 64x of the pull threshold), as the one-GPU sweep
            sums = split_frac > 0.0 && static_cast<double>(mf) * ms_alpha * 64.0 > static_cast<double>(total);
            // and builds no queue when the next level will likely pull (within 8x of the threshold)
            const bool next_pull = static_cast<double>(mf) * ms_alpha * 8.0 > static_cast<double>(total);
            if ((sums || next_pull) && (rc = part_ms_settle_sums(ctx, sums ? sc64 : nullptr, next_pull))) break;
            rc = exchange(mf,
                          [&](int64_t cap) { return tgo_part_ms_settle_fixed(ctx, level, recv, W, cap, frn, nullptr); },
                          [&](const int64_t* rp) { return tgo_part_ms_settle_pairs(ctx, level, recv, rp, W, frn, nullptr); });
            if (rc) break;
        }
        std::swap(fr, frn);
        std::swap(glob[0], glob[1]);
        // global {next frontier, its entries}; this rank's queue length back to the engine
        if (int r = x->all_reduce_sum(dc, 2, st)) { rc = xfail(r); break; }
        if ((rc = part_read_words(ctx, dc, 3, hc))) break;
        nf = hc[0];
        mf = hc[1];
        if ((rc = tgo_part_set_local_qlen(ctx, hc[2]))) break;
        ++levels;
    }
    const int rc_off = tgo_part_device_counts(ctx, caller_dc);
    trace_resolve(st);
    (void)part_ms_settle_sums(ctx, nullptr);          // a failed level may have left it armed
    part_ms_own_next(ctx, nullptr);
    if (rc) {
        x->abort();
        rezero();
        return rc;
    }
    if (rc_off) return rc_off;
    std::vector<int64_t> r(nseeds), e(nseeds);
    const bool stats = reached || entries;           // the per-seed counts cost a pass over the masks
    if ((rc = tgo_part_ms_end(ctx, stats ? r.data() : nullptr, stats ? e.data() : nullptr))) return rc;
    if (stats) {
        std::vector<int64_t> both(2 * nseeds);
        std::copy(r.begin(), r.end(), both.begin());
        std::copy(e.begin(), e.end(), both.begin() + nseeds);
        int64_t* d = dc + 3;
        if (hipMemcpyAsync(d, both.data(), both.size() * 8, hipMemcpyHostToDevice, st) != hipSuccess)
            return part_fail(ctx, TGO_E_HIP, "stats upload");
        if (int q = x->all_reduce_sum(d, both.size(), st)) return xfail(q);
        if (hipMemcpyAsync(both.data(), d, both.size() * 8, hipMemcpyDeviceToHost, st) != hipSuccess ||
            hipStreamSynchronize(st) != hipSuccess)
            return part_fail(ctx, TGO_E_HIP, "stats read");
        for (int i = 0; i < nseeds; ++i) {
            if (reached) reached[i] = both[i];
            if (entries) entries[i] = both[nseeds + i];
        }
    }
    if (levels_out) *levels_out = levels;
    return TGO_OK;
}

// ======================================================================================
// Native loops of the other partitioned programs: single-source BFS, delta-stepping SSSP and
// PageRank, each ONE C-ABI call whose C++ loop issues its collectives through the exchange on
// the ctx stream (the protocols of titan_amd/distributed.py distributed_bfs / _sssp /
// _pagerank, which stay as the Python reference drivers).  They replace the per-superstep
// Python round trips of FulgoraGraphComputer's superstep loop (FulgoraGraphComputer.java:
// 151-189) in its multi-GPU form.


extern "C" int tgo_part_bfs_run(tgo_ctx* ctx, tgo_exchange* x, int64_t seed_global, int32_t max_depth, double alpha,
                                double beta, int64_t* dist_local, int64_t* reached, int32_t* levels_out) {
    if (!ctx) return TGO_E_INVALID;
    if (!x || max_depth < 0 || !(alpha > 0.0) || !(beta > 0.0))
        return part_fail(ctx, TGO_E_INVALID, "tgo_part_bfs_run: bad arguments");
    Driver d{};
    int64_t nl = 0, lo = 0, ng = 0, ent = 0;
    int rc = driver_open(ctx, x, "tgo_part_bfs_run", 12, d, nl, lo, ng, ent);
    if (rc) return rc;
    const int W = x->world;
    const int64_t nwl = nl / 64, nwg = ng / 64;
    hipStream_t st = d.st;
    // two alternating global frontier bitmaps (the owned next frontier is the rank's slice of
    // the other one, so the all-gather is in place), the discovered bitmap and its received
    // slices, the device level counts
    uint64_t *f0 = nullptr, *f1 = nullptr, *disc = nullptr, *recv = nullptr;
    int64_t* dc = nullptr;
    if ((rc = scratch(ctx, f0, nwg, 8)) || (rc = scratch(ctx, f1, nwg, 9)) || (rc = scratch(ctx, disc, nwg, 10)) ||
        (rc = scratch(ctx, recv, nwg, 11)) || (rc = scratch(ctx, dc, 4, 13)))
        return rc;
    int64_t* const caller_dc = part_dcounts_of(ctx);
    uint64_t* glob[2] = {f0, f1};
    int64_t c[2] = {0, 0};
    if ((rc = tgo_part_bfs_begin(ctx, seed_global, glob[0] + x->rank * nwl, c))) return rc;
    if (int r = x->all_gather(glob[0], static_cast<size_t>(nwl) * 8, st)) return d.xfail(r);
    // the seed level's counts and the graph's total entries in one reduction (one host round trip)
    int64_t v3[3] = {c[0], c[1], ent}, g[3] = {0, 0, 0};
    if ((rc = d.reduce(v3, 3, tgo_exchange::kRedSum, g))) return rc;
    int64_t nf = g[0], mf = g[1], mu = g[2] - mf;
    if ((rc = tgo_part_device_counts(ctx, dc))) return rc;
    bool bottom_up = false;
    int levels = 0;
    for (int level = 0; level < max_depth && nf > 0; ++level) {
        // direction-optimizing switch (Beamer et al.; the one-GPU rule, tgo_bfs)
        if (!bottom_up && static_cast<double>(mf) > static_cast<double>(mu) / alpha) bottom_up = true;
        else if (bottom_up && static_cast<double>(nf) < static_cast<double>(ng) / beta) bottom_up = false;
        uint64_t* nb = glob[1] + x->rank * nwl;
        DevSpan span(st, "part.bfs.level", {"level", level}, {"bottom_up", bottom_up ? 1 : 0});
        if (bottom_up) {
            if ((rc = tgo_part_bfs_bu(ctx, level, glob[0], nb, nullptr))) break;
        } else {
            // owned targets claimed during the expansion (tgo::part_bfs_td_fused); the remote
            // ones travel as discovered-bitmap slices and are claimed by their owners
            if (W > 1 && hipMemsetAsync(disc, 0, nwg * 8, st) != hipSuccess) { rc = d.hip("disc clear"); break; }
            if ((rc = tgo::part_bfs_td_fused(ctx, level, disc, nb))) break;
            if (W > 1) {
                if (int r = x->all_to_all(disc, recv, static_cast<size_t>(nwl) * 8, st)) { rc = d.xfail(r); break; }
                if ((rc = tgo::part_bfs_claim_remote(ctx, level, recv, W, nb))) break;
            }
            if ((rc = tgo::part_bfs_level_done(ctx))) break;
        }
        if (int r = x->all_gather(glob[1], static_cast<size_t>(nwl) * 8, st)) { rc = d.xfail(r); break; }
        std::swap(glob[0], glob[1]);
        if (int r = x->all_reduce_sum(dc, 2, st)) { rc = d.xfail(r); break; }
        if ((rc = part_read_words(ctx, dc, 3, d.hc))) break;
        nf = d.hc[0];
        mf = d.hc[1];
        mu -= mf;
        if ((rc = tgo_part_set_local_qlen(ctx, d.hc[2]))) break;
        ++levels;
    }
    const int rc_off = tgo_part_device_counts(ctx, caller_dc);
    trace_resolve(st);
    if (rc) { x->abort(); return rc; }
    if (rc_off) return rc_off;
    int64_t rl[2] = {0, 0};
    // the reach statistics (a pass over every list) only when asked for
    if ((rc = tgo_part_bfs_end(ctx, dist_local, reached ? rl : nullptr))) return rc;
    if (reached && (rc = d.reduce(rl, 2, tgo_exchange::kRedSum, reached))) return rc;
    if (levels_out) *levels_out = levels;
    return TGO_OK;
}

extern "C" int tgo_part_sssp_run(tgo_ctx* ctx, tgo_exchange* x, int64_t seed_global, int64_t delta, int64_t* dist_local,
                                 int64_t* reached, int32_t* phases_out) {
    if (!ctx) return TGO_E_INVALID;
    if (!x) return part_fail(ctx, TGO_E_INVALID, "tgo_part_sssp_run: bad arguments");
    Driver d{};
    int64_t nl = 0, lo = 0, ng = 0, ent = 0;
    int rc = driver_open(ctx, x, "tgo_part_sssp_run", 17, d, nl, lo, ng, ent);
    if (rc) return rc;
    const int W = x->world;
    hipStream_t st = d.st;
    int64_t *send = nullptr, *recv = nullptr, *sizes = nullptr;
    if ((rc = scratch(ctx, send, 2 * ng + 2, 14)) || (rc = scratch(ctx, recv, 2 * ng + 2, 15)) ||
        (rc = scratch(ctx, sizes, 11 * W + 3, 16)))
        return rc;
    // negative weights: every rank fails here, before any collective a peer could wait in
    int64_t wmin = 0, gmin = 0;
    if ((rc = tgo_part_weight_min(ctx, &wmin))) return rc;
    if ((rc = d.reduce(&wmin, 1, tgo_exchange::kRedMin, &gmin))) return rc;
    if (gmin < 0) return part_fail(ctx, TGO_E_INVALID, "delta-stepping needs non-negative weights (a rank holds a negative weight)");
    int64_t out[2] = {0, 0};
    if ((rc = tgo_part_sssp_begin(ctx, seed_global, delta, out))) return rc;
    if (delta <= 0) {           // the ranks' default widths follow their local mean weight: agree on one
        if ((rc = d.reduce(&out[1], 1, tgo_exchange::kRedMax, &delta))) return rc;
    }
    if (delta <= 0) return part_fail(ctx, TGO_E_INVALID, "tgo_part_sssp_run: bucket width");
    // light/heavy split (weighted loads): the same decision on every rank (the load's weights
    // and the agreed width); the loop below is the same either way
    bool split = false;
    if ((rc = part_sssp_split(ctx, delta, &split))) return rc;
    (void)split;
    // on the device-sized loop (delta_loop.hip) nothing but the header comes to the host
    const bool dev = part_sssp_devloop(ctx);
    int64_t thr = delta;
    int phases = 0;
    // per phase, ONE host read: the relax writes a 4-word header per peer on the device
    // {pair elements for it, near-queue length, pending minimum, members flag}; one all-to-all
    // moves the headers and a fold (2W + 3 words: sent / received sizes, global queue length,
    // pending minimum, members) comes back through the mapped counter page.  An empty global
    // near queue then moves straight to the next bucket: the pending minimum is kept on the
    // fly (delta.hip ds_track_reset), so no bitmap scan and no second collective.
    int64_t* hdr_recv = sizes + 4 * W;
    int64_t* fold = sizes + 8 * W;
    const int nf = 2 * W + 3;
    std::vector<int64_t> hf(nf);
    std::vector<size_t> sb(W), so(W), rb(W), ro(W);
    // One rank on the device loop: its header all-to-all is the identity, so the header kernel
    // folds and publishes it in one launch (3 launches and a copy fewer per phase).  Up to 14
    // ranks the fold publishes its own words (nf <= 32 counter-page words).
    const bool solo = dev && W == 1;
    for (;;) {
        DevSpan span(st, "part.sssp.phase", {"phase", phases}, {"threshold", thr});
        if (solo) {
            if ((rc = part_sssp_dev_relax(ctx, W, send, sizes, hf.data()))) break;
        } else {
            if ((rc = dev ? part_sssp_dev_relax(ctx, W, send, sizes, nullptr) : part_sssp_relax_dev(ctx, thr, W, send, sizes)))
                break;
            if (int r = x->all_to_all(sizes, hdr_recv, 32, st)) { rc = d.xfail(r); break; }
            if (nf <= 32) {                // through the mapped counter page (up to 14 ranks)
                if ((rc = part_sssp_header_read(ctx, sizes, hdr_recv, W, fold, hf.data()))) break;
            } else if ((rc = part_sssp_header_fold(ctx, sizes, hdr_recv, W, fold)) ||
                       hipMemcpyAsync(hf.data(), fold, nf * sizeof(int64_t), hipMemcpyDeviceToHost, st) != hipSuccess ||
                       hipStreamSynchronize(st) != hipSuccess) { if (!rc) rc = d.hip("header read"); break; }
        }
        if (hf[2 * W] == 0) {   // every near queue was empty (nothing was relaxed): the next non-empty bucket
            span.end();
            const int64_t mn = hf[2 * W + 1];
            if (mn == INT64_MAX && hf[2 * W + 2] == 0) break;   // converged: nothing pending, no members left
            if (mn != INT64_MAX && mn >= thr) thr = (mn / delta + 1) * delta;
            if ((rc = dev ? part_sssp_dev_extract(ctx, thr) : tgo_part_sssp_extract(ctx, thr, nullptr))) break;
            continue;
        }
        size_t a = 0, b = 0;
        for (int p = 0; p < W; ++p) {
            sb[p] = static_cast<size_t>(hf[p]) * 8; so[p] = a; a += sb[p];
            rb[p] = static_cast<size_t>(hf[W + p]) * 8; ro[p] = b; b += rb[p];
        }
        if (int r = x->all_to_allv(send, sb.data(), so.data(), recv, rb.data(), ro.data(), st)) { rc = d.xfail(r); break; }
        const int64_t np = static_cast<int64_t>(b / 16);
        if ((rc = dev ? part_sssp_dev_apply(ctx, recv, np) : tgo_part_sssp_apply(ctx, thr, recv, np, nullptr))) break;
        ++phases;
    }
    trace_resolve(st);
    if (rc) { x->abort(); return rc; }
    int64_t rl[2] = {0, 0};
    if ((rc = tgo_part_sssp_end(ctx, dist_local, rl))) return rc;
    if (reached && (rc = d.reduce(rl, 2, tgo_exchange::kRedSum, reached))) return rc;
    if (phases_out) *phases_out = phases;
    return TGO_OK;
}


extern "C" int tgo_part_pagerank_run(tgo_ctx* ctx, tgo_exchange* x, const tgo_pr_args* args, int32_t exchange_mode,
                                     double* pr_local, int64_t* exchanged_bytes) {
    if (!ctx) return TGO_E_INVALID;
    if (!x || !args || args->max_iterations < 1 || exchange_mode < 0 || exchange_mode > 1)
        return part_fail(ctx, TGO_E_INVALID, "tgo_part_pagerank_run: bad arguments");
    Driver d{};
    int64_t nl = 0, lo = 0, ng = 0, ent = 0;
    int rc = driver_open(ctx, x, "tgo_part_pagerank_run", 22, d, nl, lo, ng, ent);
    if (rc) return rc;
    const int W = x->world, R = x->rank;
    hipStream_t st = d.st;
    // layout: active span A = max active rows (every rank), the blocked hot-first layout
    int64_t act = 0, span = 0, hot = 0;
    if ((rc = tgo_part_active_rows(ctx, &act))) return rc;
    if ((rc = d.reduce(&act, 1, tgo_exchange::kRedMax, &span))) return rc;
    if ((rc = tgo_part_pr_blocked(ctx, W, span, &hot))) return rc;
    if (hot == 0) span = nl;                     // plain layout: rank-major n_local slices
    double *contrib = nullptr, *gath = nullptr;
    if ((rc = scratch(ctx, contrib, nl, 18)) || (rc = scratch(ctx, gath, static_cast<int64_t>(W) * span, 19))) return rc;
    PrGhost* gh = nullptr;
    if (exchange_mode == 1 && W > 1) {
        std::shared_ptr<PrGhost>& cached = ghost_cache(ctx).pr;
        gh = cached.get();
        if (!gh || gh->world != W || gh->rank != R || gh->hot != hot || gh->span != span || gh->nl != nl) {
            auto fresh = std::make_shared<PrGhost>();
            if ((rc = build_ghost(ctx, x, d, nl, hot, span, false, *fresh))) { x->abort(); return rc; }
            cached = fresh;
            gh = fresh.get();
        }
    }
    int64_t moved = 0;
  rerun:
    if ((rc = tgo_part_pr_begin(ctx, args, contrib))) return rc;
    for (int it = 2; it <= args->max_iterations; ++it) {
        DevSpan upd(st, "part.pagerank.update", {"iteration", it}, {"ghost", gh ? 1 : 0});
        // the rank's own slice into the gathered vector
        hipError_t e = hot == 0
            ? hipMemcpyAsync(gath + static_cast<int64_t>(R) * nl, contrib, nl * 8, hipMemcpyDeviceToDevice, st)
            : hipMemcpyAsync(gath + static_cast<int64_t>(R) * hot, contrib, hot * 8, hipMemcpyDeviceToDevice, st);
        if (e == hipSuccess && hot > 0 && span > hot)
            e = hipMemcpyAsync(gath + static_cast<int64_t>(W) * hot + static_cast<int64_t>(R) * (span - hot), contrib + hot,
                               (span - hot) * 8, hipMemcpyDeviceToDevice, st);
        if (e != hipSuccess) { rc = d.hip("own slice"); break; }
        if (W > 1 && gh) {                       // ghosts: exactly the remote values this rank reads
            if ((e = k_pack_f64(contrib, gh->send_row, gh->nsend, gh->sbuf, st)) != hipSuccess) { rc = d.hip("pack"); break; }
            if (int r = x->all_to_allv(gh->sbuf, gh->sb.data(), gh->so.data(), gh->rbuf, gh->rb.data(), gh->ro.data(), st)) {
                rc = d.xfail(r);
                break;
            }
            if ((e = k_unpack_f64(gh->rbuf, gh->recv_pos, gh->nrecv, gath, st)) != hipSuccess) { rc = d.hip("unpack"); break; }
            moved += gh->nrecv * 8;
        } else if (W > 1) {                      // all-gather of every rank's slices (in place)
            int r = hot == 0 ? x->all_gather(gath, static_cast<size_t>(nl) * 8, st)
                             : x->all_gather(gath, static_cast<size_t>(hot) * 8, st);
            if (!r && hot > 0 && span > hot)
                r = x->all_gather(gath + static_cast<int64_t>(W) * hot, static_cast<size_t>(span - hot) * 8, st);
            if (r) { rc = d.xfail(r); break; }
            moved += static_cast<int64_t>(W - 1) * (hot == 0 ? nl : span) * 8;
        }
        if ((rc = tgo_part_pr_step(ctx, gath, contrib))) break;
    }
    trace_resolve(st);
    if (rc) { x->abort(); tgo_part_pr_plain(ctx, 0); return rc; }
    if (hot > 0) {
        // a message outside the fixed-point passes' exact range on ANY rank (+inf from a vertex
        // whose row cut left it no OUT entry, NaN, ...): every rank re-runs the program on the
        // plain fp64 gather (rank-major all-gather layout), whose sums are Java double sums
        int32_t bad = 0;
        if ((rc = tgo_part_pr_exact_check(ctx, &bad))) { x->abort(); return rc; }
        int64_t b = bad, any = 0;
        if ((rc = d.reduce(&b, 1, tgo_exchange::kRedMax, &any))) return rc;
        if (any) {
            if ((rc = tgo_part_pr_plain(ctx, 1))) return rc;
            hot = 0;
            span = nl;
            gh = nullptr;
            if ((rc = scratch(ctx, gath, static_cast<int64_t>(W) * span, 19))) { tgo_part_pr_plain(ctx, 0); return rc; }
            goto rerun;
        }
    }
    rc = tgo_part_pr_end(ctx, pr_local);
    tgo_part_pr_plain(ctx, 0);
    if (rc) return rc;
    if (exchanged_bytes) *exchanged_bytes = moved;
    return TGO_OK;
}

// ======================================================================================
// The partitioned load from edgestore rows.  Rank r hands in the rows of its vertices (a row
// holds the vertex's OUT and IN entries, so a 1-D vertex partition is a row-range partition of
// the scan); the decode and the cut are the one-GPU rules per row (VertexJobConverter.java:
// 109-129, the 100 000 cap in column order: QueryContainer.java:28,122, ColumnValueStore.java:
// 47-69), so every rank's lists are exactly the lists tgo_load_rows would hold for those rows.
// Collectives (all on the exchange, every rank in the same order):
//   1. MAX of {decode failed, live rows}: a failure on any rank fails every rank here;
//      S = the largest live count rounded up to 64 (slot ids r * S + i, padding entry-less);
//   2. all-gather of the live Titan ids at their slots: the global id map;
//   3. (layout) all-gather of the degree-grouped slot layout;
//   4. SUM of the cut rows; when a single-direction scope cut any row, its push view is no
//      transpose of the stored opposite lists: the pull entries go to their sources' owners
//      (all-to-all of the counts, all-to-allv of the pairs) and become the push rows there.
namespace {
struct DevTmp {                 // a device temporary of the load (the ctx holds no graph yet)
    void* p = nullptr;
    ~DevTmp() { if (p) (void)hipFree(p); }
    hipError_t alloc(size_t bytes) { return hipMalloc(&p, std::max<size_t>(bytes, 8)); }
};
}  // namespace

// local_rc: a failure this rank met before the collective part (its staging is dropped); the
// ranks still agree on it, so every rank returns an error and none waits in an exchange.
static int finish_partition_rows(tgo_ctx* ctx, tgo_exchange* x, int32_t layout, int64_t* part_out, int local_rc,
                                 const std::string& local_err) {
    const int W = x->world, R = x->rank;
    hipStream_t st = part_stream(ctx);
    std::string err = local_err;
    auto xerr = [&](int code) { return part_fail(ctx, code, "exchange: " + x->err); };
    auto hip = [&](const char* what) { x->abort(); return part_fail(ctx, TGO_E_HIP, std::string("tgo_finish_partition_rows: ") + what); };
    DevTmp red;
    if (red.alloc(8 * sizeof(int64_t)) != hipSuccess) return hip("scratch");
    // element-wise reduction of k host words over the ranks
    auto reduce = [&](int64_t* v, int k, int op) -> int {
        if (hipMemcpyAsync(red.p, v, k * sizeof(int64_t), hipMemcpyHostToDevice, st) != hipSuccess) return hip("reduce upload");
        if (int r = x->all_reduce(static_cast<int64_t*>(red.p), static_cast<size_t>(k), op, st)) return xerr(r);
        if (hipMemcpyAsync(v, red.p, k * sizeof(int64_t), hipMemcpyDeviceToHost, st) != hipSuccess ||
            hipStreamSynchronize(st) != hipSuccess)
            return hip("reduce read");
        return TGO_OK;
    };
    // 1. decode, then agree on failure and on the slot size
    RowStaging stg;
    int drc = local_rc;
    if (drc) part_drop_staging(ctx);
    else drc = part_rows_take(ctx, stg, err);
    const int64_t count = drc ? 0 : static_cast<int64_t>(stg.vid.size());
    // a rank without staged rows (an empty range) takes the scope / weightedness of the others
    const bool staged = !drc && stg.active;
    int64_t v1[4] = {drc ? 1 : 0, count, staged ? stg.opts.scope + 1 : 0, staged && stg.opts.weight_key != 0 ? 1 : 0};
    const int64_t own_scope = v1[2], own_weighted = v1[3];
    if (int rc = reduce(v1, 4, tgo_exchange::kRedMax)) return rc;
    if (drc) return part_fail(ctx, drc, "tgo_finish_partition_rows: " + err);
    if (v1[0]) return part_fail(ctx, TGO_E_INVALID, "tgo_finish_partition_rows: another rank failed to decode its rows");
    if (!staged) {
        stg.opts.scope = static_cast<int32_t>(std::max<int64_t>(0, v1[2] - 1));
        stg.opts.weight_key = v1[3];
    }
    // ranks that disagree on the scope or the weight key fail below (agreed with the assembly)
    int mismatch = staged && (own_scope != v1[2] || own_weighted != v1[3]);
    const int64_t S = std::max<int64_t>(64, (v1[1] + 63) / 64 * 64), lo = static_cast<int64_t>(R) * S;
    const int64_t n_global = static_cast<int64_t>(W) * S;
    if (n_global >= INT32_MAX) return part_fail(ctx, TGO_E_UNSUPPORTED, "tgo_finish_partition_rows: more than 2^31 - 1 slots");
    // 2. the global id map: every rank's live ids at their slots
    std::vector<int64_t> slot_vid(static_cast<size_t>(n_global));
    {
        DevTmp buf;
        if (buf.alloc(n_global * sizeof(int64_t)) != hipSuccess) return hip("id buffer");
        std::vector<int64_t> own(static_cast<size_t>(S));
        for (int64_t i = 0; i < S; ++i) own[i] = i < count ? stg.vid[i] : -1 - (lo + i);   // padding: never a Titan id
        int64_t* b = static_cast<int64_t*>(buf.p);
        if (hipMemcpyAsync(b + lo, own.data(), S * sizeof(int64_t), hipMemcpyHostToDevice, st) != hipSuccess)
            return hip("id upload");
        if (int r = x->all_gather(b, static_cast<size_t>(S) * sizeof(int64_t), st)) return xerr(r);
        if (hipMemcpyAsync(slot_vid.data(), b, n_global * sizeof(int64_t), hipMemcpyDeviceToHost, st) != hipSuccess ||
            hipStreamSynchronize(st) != hipSuccess)
            return hip("id read");
    }
    HostGraph h;
    const int threads = part_threads(ctx);
    int arc = assemble_partition_rows(stg, slot_vid, S, R, h, threads, err);
    if (!arc && mismatch) {
        err = "the ranks staged rows with different scopes or weight keys";
        arc = TGO_E_INVALID;
    }
    std::vector<int64_t>().swap(slot_vid);
    // 3. the degree-grouped layout of every rank's slots (a rank whose assembly failed still
    //    takes part in the collective; the failure is agreed in step 4)
    if (layout) {
        DevTmp buf;
        if (buf.alloc(n_global * sizeof(int32_t)) != hipSuccess) return hip("layout buffer");
        std::vector<int32_t> lay(static_cast<size_t>(n_global));
        if (arc) for (int64_t i = 0; i < S; ++i) lay[lo + i] = static_cast<int32_t>(lo + i);
        else partition_rows_layout(h, lo, lay.data() + lo);
        int32_t* b = static_cast<int32_t*>(buf.p);
        if (hipMemcpyAsync(b + lo, lay.data() + lo, S * sizeof(int32_t), hipMemcpyHostToDevice, st) != hipSuccess)
            return hip("layout upload");
        if (int r = x->all_gather(b, static_cast<size_t>(S) * sizeof(int32_t), st)) return xerr(r);
        if (hipMemcpyAsync(lay.data(), b, n_global * sizeof(int32_t), hipMemcpyDeviceToHost, st) != hipSuccess ||
            hipStreamSynchronize(st) != hipSuccess)
            return hip("layout read");
        if (!arc) arc = apply_partition_layout(h, lo, lay.data(), threads, err);
    }
    // 4. cut rows anywhere: the push view from every rank's pull entries (and a last agreement
    //    on failure before the graph replaces the ctx's)
    int64_t v4[3] = {arc ? 1 : 0, h.truncated, count};
    if (int rc = reduce(v4, 3, tgo_exchange::kRedSum)) return rc;
    if (arc) return part_fail(ctx, arc, "tgo_finish_partition_rows: " + err);
    if (v4[0]) return part_fail(ctx, TGO_E_INVALID, "tgo_finish_partition_rows: another rank failed to assemble its rows");
    if (v4[1] > 0 && h.scope != TGO_SCOPE_BOTH_E) {
        std::vector<int64_t> cnt, pairs;
        partition_pull_pairs(h, lo, S, W, cnt, pairs);
        DevTmp dc, rc_, sbuf, rbuf;
        if (dc.alloc(W * sizeof(int64_t)) != hipSuccess || rc_.alloc(W * sizeof(int64_t)) != hipSuccess) return hip("count buffers");
        std::vector<int64_t> rcnt(W);
        if (hipMemcpyAsync(dc.p, cnt.data(), W * sizeof(int64_t), hipMemcpyHostToDevice, st) != hipSuccess) return hip("counts");
        if (int r = x->all_to_all(dc.p, rc_.p, sizeof(int64_t), st)) return xerr(r);
        if (hipMemcpyAsync(rcnt.data(), rc_.p, W * sizeof(int64_t), hipMemcpyDeviceToHost, st) != hipSuccess ||
            hipStreamSynchronize(st) != hipSuccess)
            return hip("count read");
        std::vector<size_t> sb(W), so(W), rb(W), ro(W);
        size_t a = 0, b = 0;
        for (int p = 0; p < W; ++p) {
            sb[p] = static_cast<size_t>(cnt[p]) * 16; so[p] = a; a += sb[p];
            rb[p] = static_cast<size_t>(rcnt[p]) * 16; ro[p] = b; b += rb[p];
        }
        if (sbuf.alloc(a) != hipSuccess || rbuf.alloc(b) != hipSuccess) return hip("pair buffers");
        if (a && hipMemcpyAsync(sbuf.p, pairs.data(), a, hipMemcpyHostToDevice, st) != hipSuccess) return hip("pairs");
        if (int r = x->all_to_allv(sbuf.p, sb.data(), so.data(), rbuf.p, rb.data(), ro.data(), st)) return xerr(r);
        std::vector<int64_t> recv(b / 8);
        if ((b && hipMemcpyAsync(recv.data(), rbuf.p, b, hipMemcpyDeviceToHost, st) != hipSuccess) ||
            hipStreamSynchronize(st) != hipSuccess)
            return hip("pair read");
        partition_push_from_pairs(h, recv.data(), static_cast<int64_t>(b / 16));
    }
    if (int rc = part_upload(ctx, h, n_global, lo)) return rc;
    part_set_live(ctx, count);
    part_out[0] = count;
    part_out[1] = S;
    part_out[2] = v4[2];
    return TGO_OK;
}

extern "C" int tgo_finish_partition_rows(tgo_ctx* ctx, tgo_exchange* x, int32_t layout, int64_t* part) {
    if (!ctx) return TGO_E_INVALID;
    if (!x || !part || x->world < 1 || x->rank < 0 || x->rank >= x->world)
        return part_fail(ctx, TGO_E_INVALID, "tgo_finish_partition_rows: bad arguments");
    return finish_partition_rows(ctx, x, layout, part, TGO_OK, std::string());
}

extern "C" int tgo_load_partition_rows(tgo_ctx* ctx, tgo_exchange* x, const tgo_rows* rows, const tgo_schema* schema,
                                       const tgo_load_opts* opts, int32_t layout, int64_t* part) {
    if (!ctx) return TGO_E_INVALID;
    if (!x || !part || x->world < 1 || x->rank < 0 || x->rank >= x->world)
        return part_fail(ctx, TGO_E_INVALID, "tgo_load_partition_rows: bad arguments");
    const int rc = tgo_load_rows(ctx, rows, schema, opts);
    return finish_partition_rows(ctx, x, layout, part, rc, rc ? std::string(tgo_last_error(ctx)) : std::string());
}

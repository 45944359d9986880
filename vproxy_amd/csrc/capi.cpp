// capi.cpp -- the C ABI (include/vclassify.h): contexts, snapshot
// publication, uploads, and the host-side control-plane mirrors.
#include <hip/hip_runtime.h>
#include <unistd.h>

#include <algorithm>
#include <atomic>
#include <condition_variable>
#include <cstdlib>
#include <cstring>
#include <map>
#include <memory>
#include <mutex>
#include <set>
#include <string>
#include <thread>
#include <vector>

#include "common/images.h"
#include "compile/compile.hpp"
#include "device/launch.h"
#include "host/mirror.hpp"
#include "host/net.hpp"
#include "host/prometheus.hpp"
#include "vclassify.h"

namespace {

thread_local std::string g_err;

int fail(int code, const std::string& msg) {
    g_err = msg;
    return code;
}

int hip_fail(hipError_t e, const char* what) {
    return fail(VC_EDEVICE, std::string(what) + ": " + hipGetErrorString(e));
}

// ---------------------------------------------------------------------------
// Retired device memory.  A snapshot's last reference can drop on any
// thread -- often an event-loop thread finishing a classify call that pinned
// the old tables -- and hipFree waits for the whole device.  Its buffers go
// here instead, and the control thread frees them (vc_compile_*,
// vc_servers_set_health, vc_counters_read after its device sync, vc_destroy):
// the thread that recompiles pays the wait, the classify threads never do.
// Retention: buffers whose last pin dropped after the publish that replaced
// them wait for the next of those calls.
// ---------------------------------------------------------------------------
struct Graveyard {
    std::mutex mu;
    std::vector<void*> ptrs;
    size_t bytes = 0;
    void bury(void* p, size_t n) {
        std::lock_guard<std::mutex> lk(mu);
        ptrs.push_back(p);
        bytes += n;
    }
    void drain() {
        std::vector<void*> v;
        {
            std::lock_guard<std::mutex> lk(mu);
            v.swap(ptrs);
            bytes = 0;
        }
        for (void* p : v) (void)hipFree(p);
    }
};

// Device allocation owned by a snapshot; retired through the graveyard.
struct DevBuf {
    void* p = nullptr;
    size_t n = 0;
    std::shared_ptr<Graveyard> grave;
    DevBuf() = default;
    DevBuf(const DevBuf&) = delete;
    DevBuf& operator=(const DevBuf&) = delete;
    ~DevBuf() {
        if (p) grave->bury(p, n);
    }
};

// A growable bump arena of device (hipMalloc) or page-locked host
// (hipHostMalloc) memory.  alloc never moves earlier allocations: a request
// that does not fit opens a new block; reset(), called only when nothing
// uses the arena, merges the blocks into one sized for the high-water mark,
// so a steady stream of calls allocates nothing.
class Arena {
public:
    explicit Arena(bool host) : host_(host) {}
    Arena(const Arena&) = delete;
    Arena& operator=(const Arena&) = delete;
    ~Arena() { release(); }
    void* alloc(size_t bytes, hipError_t* err) {
        const size_t b = (std::max<size_t>(bytes, 1) + 255) & ~size_t(255);
        if (blocks_.empty() || used_ + b > blocks_.back().second) {
            const size_t grow = blocks_.empty() ? 0 : 2 * blocks_.back().second;
            const size_t want = std::max(b, std::max(size_t(1) << 20, grow));
            void* p = nullptr;
            const hipError_t e = host_ ? hipHostMalloc(&p, want, hipHostMallocDefault)
                                       : hipMalloc(&p, want);
            if (e != hipSuccess) {
                *err = e;
                return nullptr;
            }
            blocks_.emplace_back(static_cast<uint8_t*>(p), want);
            used_ = 0;
        }
        uint8_t* p = blocks_.back().first + used_;
        used_ += b;
        return p;
    }
    hipError_t reset() {
        used_ = 0;
        if (blocks_.size() <= 1) return hipSuccess;
        size_t total = 0;
        for (auto& b : blocks_) total += b.second;
        release();
        void* p = nullptr;
        const hipError_t e = host_ ? hipHostMalloc(&p, total, hipHostMallocDefault)
                                   : hipMalloc(&p, total);
        if (e == hipSuccess) blocks_.emplace_back(static_cast<uint8_t*>(p), total);
        return e;
    }
    void release() {
        for (auto& b : blocks_) (void)(host_ ? hipHostFree(b.first) : hipFree(b.first));
        blocks_.clear();
        used_ = 0;
    }

private:
    bool host_;
    std::vector<std::pair<uint8_t*, size_t>> blocks_;
    size_t used_ = 0;
};

// One staging lane: a stream, device memory for a call's inputs and
// outputs, and a page-locked bounce buffer.  Every DMA of the host entry
// points runs between memory the library allocated itself: caller arrays
// are copied into the bounce buffer with memcpy on the calling thread, and
// results are copied out of it after the lane's stream has drained.  No
// pageable-memory DMA (which makes the runtime look up, pin or stage the
// caller's pages) and no stream-ordered pool allocation is on this path.
// Host memcpy for the staging copies.  One thread copies ~10 GB/s, a
// fifth of what PCIe moves, so copies of 4 MiB and more are split over a
// few worker threads (the calling thread takes a share too).  The workers
// start on first use and serve every lane of every stager.
class CopyPool {
public:
    static CopyPool& get() {
        static CopyPool pool;
        return pool;
    }
    void copy(void* dst, const void* src, size_t n) {
        const int parts = workers_ + 1;
        // a forked child has none of the parent's workers: copy alone there
        if (n < kMin || workers_ == 0 || ::getpid() != pid_) {
            std::memcpy(dst, src, n);
            return;
        }
        start();
        std::atomic<int> left{parts - 1};
        const size_t piece = (n / parts + 63) & ~size_t(63);
        {
            std::lock_guard<std::mutex> lk(mu_);
            for (int k = 1; k < parts; ++k) {
                const size_t a = std::min(n, piece * size_t(k));
                const size_t b = k + 1 == parts ? n : std::min(n, a + piece);
                jobs_.push_back(Job{static_cast<char*>(dst) + a, static_cast<const char*>(src) + a,
                                    b - a, &left});
            }
        }
        cv_.notify_all();
        std::memcpy(dst, src, std::min(n, piece));
        std::unique_lock<std::mutex> lk(mu_);
        done_.wait(lk, [&] { return left.load() == 0; });
    }
    ~CopyPool() {
        {
            std::lock_guard<std::mutex> lk(mu_);
            stop_ = true;
        }
        cv_.notify_all();
        for (auto& t : th_) t.join();
    }

private:
    static constexpr size_t kMin = size_t(4) << 20;
    struct Job {
        char* d;
        const char* s;
        size_t n;
        std::atomic<int>* left;
    };
    CopyPool() : pid_(::getpid()) {
        const unsigned hc = std::thread::hardware_concurrency();
        workers_ = int(std::min(7u, hc > 1 ? hc - 1 : 0u));
    }
    void start() {
        std::call_once(once_, [this] {
            for (int k = 0; k < workers_; ++k) th_.emplace_back([this] { run(); });
        });
    }
    void run() {
        for (;;) {
            Job j;
            {
                std::unique_lock<std::mutex> lk(mu_);
                cv_.wait(lk, [&] { return stop_ || !jobs_.empty(); });
                if (stop_ && jobs_.empty()) return;
                j = jobs_.back();
                jobs_.pop_back();
            }
            std::memcpy(j.d, j.s, j.n);
            if (j.left->fetch_sub(1) == 1) {
                std::lock_guard<std::mutex> lk(mu_);
                done_.notify_all();
            }
        }
    }
    int workers_ = 0;
    const pid_t pid_;
    std::once_flag once_;
    std::mutex mu_;
    std::condition_variable cv_, done_;
    std::vector<Job> jobs_;
    std::vector<std::thread> th_;
    bool stop_ = false;
};

// Copies of more than kPiece bytes go in pieces: piece k's host copy runs
// while piece k - 1's DMA is in flight (inputs), and piece k's results are
// copied out as soon as its D2H copy has landed, while the next lands.
constexpr size_t kPiece = size_t(16) << 20;

struct StageLane {
    hipStream_t s = nullptr;
    Arena dev{false}, host{true};
    struct Back {
        void* user;
        const void* pinned;
        size_t bytes;
        int ev;                 // index into evs: the piece's D2H has landed
    };
    std::vector<Back> backs;
    std::vector<hipEvent_t> evs;   // reused across calls
    int evs_used = 0;
    bool busy = false;      // copies or kernels issued since the last finish

    // an event recorded on the lane's stream now (-1: none available)
    int mark() {
        if (evs_used == int(evs.size())) {
            hipEvent_t e = nullptr;
            if (hipEventCreateWithFlags(&e, hipEventDisableTiming) != hipSuccess) return -1;
            evs.push_back(e);
        }
        if (hipEventRecord(evs[size_t(evs_used)], s) != hipSuccess) return -1;
        return evs_used++;
    }
    // wait for the lane's work without giving its memory back
    hipError_t wait() { return busy ? hipStreamSynchronize(s) : hipSuccess; }
    // wait, deliver the results to the caller's arrays (deliver), and reset
    // the arenas for the next user
    hipError_t finish(bool deliver) {
        hipError_t e = hipSuccess;
        if (deliver)
            for (const Back& b : backs) {
                if (e == hipSuccess && b.ev >= 0) e = hipEventSynchronize(evs[size_t(b.ev)]);
                if (e != hipSuccess) break;
                if (b.ev < 0 && (e = hipStreamSynchronize(s)) != hipSuccess) break;
                CopyPool::get().copy(b.user, b.pinned, b.bytes);
            }
        const hipError_t es = busy ? hipStreamSynchronize(s) : hipSuccess;
        if (e == hipSuccess) e = es;
        busy = false;
        backs.clear();
        evs_used = 0;
        const hipError_t r1 = dev.reset(), r2 = host.reset();
        return e != hipSuccess ? e : r1 != hipSuccess ? r1 : r2;
    }
    ~StageLane() {
        for (hipEvent_t e : evs) (void)hipEventDestroy(e);
    }
};

// Lanes 0 and 1 carry a chunked call's alternating chunks (host_chunks);
// lane 2 holds whole-call data (the pipeline's hostname-pool results) and
// the uploads of a compile.
struct Stager {
    StageLane lane[3];
};

struct Snapshot;
struct AclSnap;
struct RouteSnap;
struct HintSnap;
struct HostsSnap;
struct ServerSnap;
struct CertSnap;
struct MirrorSnap;
struct VniSnap;

// The published snapshot of every table kind, in VC_SNAP_* order.  A
// context holds the current set; a vc_pin holds a copy of the slots it
// pinned.
template <class S> struct snap_kind;
template <> struct snap_kind<AclSnap> { static constexpr int value = VC_SNAP_ACL; };
template <> struct snap_kind<RouteSnap> { static constexpr int value = VC_SNAP_ROUTE; };
template <> struct snap_kind<HintSnap> { static constexpr int value = VC_SNAP_UPSTREAM; };
template <> struct snap_kind<HostsSnap> { static constexpr int value = VC_SNAP_HOSTS; };
template <> struct snap_kind<ServerSnap> { static constexpr int value = VC_SNAP_SERVERS; };
template <> struct snap_kind<CertSnap> { static constexpr int value = VC_SNAP_CERTS; };
template <> struct snap_kind<MirrorSnap> { static constexpr int value = VC_SNAP_MIRROR; };
template <> struct snap_kind<VniSnap> { static constexpr int value = VC_SNAP_VNI; };

struct SnapSet {
    std::shared_ptr<const AclSnap> acl;
    std::shared_ptr<const RouteSnap> route;
    std::shared_ptr<const HintSnap> hint;
    std::shared_ptr<const HostsSnap> hosts;
    std::shared_ptr<const ServerSnap> servers;
    std::shared_ptr<const CertSnap> certs;
    std::shared_ptr<const MirrorSnap> mirror;
    std::shared_ptr<const VniSnap> vni;      // Switch.tables (vc_compile_vni_routes)

    template <class S> const std::shared_ptr<const S>& slot() const;
};
template <> const std::shared_ptr<const AclSnap>& SnapSet::slot<AclSnap>() const { return acl; }
template <> const std::shared_ptr<const RouteSnap>& SnapSet::slot<RouteSnap>() const { return route; }
template <> const std::shared_ptr<const HintSnap>& SnapSet::slot<HintSnap>() const { return hint; }
template <> const std::shared_ptr<const HostsSnap>& SnapSet::slot<HostsSnap>() const { return hosts; }
template <> const std::shared_ptr<const ServerSnap>& SnapSet::slot<ServerSnap>() const {
    return servers;
}
template <> const std::shared_ptr<const CertSnap>& SnapSet::slot<CertSnap>() const { return certs; }
template <> const std::shared_ptr<const MirrorSnap>& SnapSet::slot<MirrorSnap>() const {
    return mirror;
}
template <> const std::shared_ptr<const VniSnap>& SnapSet::slot<VniSnap>() const { return vni; }

}  // namespace

// A caller's pin (vc_pin_acquire): the snapshots of `kinds` that were
// current when it was taken.  Bound to a thread (vc_pin_bind), it is what
// that thread's classify calls on `ctx` use for those kinds.
struct vc_pin {
    vc_ctx* ctx = nullptr;
    uint32_t kinds = 0;
    SnapSet s;
};

namespace {
thread_local const vc_pin* t_pin = nullptr;
}  // namespace

struct vc_ctx : SnapSet {
    int device = 0;
    hipStream_t stream = nullptr;
    hipEvent_t handoff = nullptr;  // vc::Handoff: stream -> count_stream ordering
    std::mutex handoff_mu;
    vc::ScratchRing scratch;       // counter-pass scratch, reused across calls
    vc::ScratchRing http_scratch;  // vc_http_hint's rewrite space (best-fit, no grow-all)
    vc::TicketRing tickets;        // work counters of the string kernels
    int num_cus = 256;
    bool sync_check = false;       // VC_SYNC_CHECK: synchronise + check after every launch / copy
    std::atomic<bool> counters_on{false};
    std::mutex compile_mu;   // serialises compiles; classify never takes it
    std::shared_ptr<Graveyard> grave = std::make_shared<Graveyard>();
    std::mutex stage_mu;     // idle stagers (one per concurrent host-buffer call)
    std::vector<std::unique_ptr<Stager>> stagers;
    std::atomic<uint64_t> next_gen{1};       // generation of the next publish (any kind)
    std::mutex port_seen_mu;
    std::set<int32_t> acl_ports_seen;        // bind ports of switch calls (AclSnap::ports)

    // The snapshot a classify call uses: the calling thread's bound pin
    // when it pinned this kind (vc_pin_bind), else the current one.
    template <class S>
    std::shared_ptr<const S> get(const std::shared_ptr<const S>& p) const {
        const vc_pin* pin = t_pin;
        if (pin && pin->ctx == this && (pin->kinds >> snap_kind<S>::value & 1u))
            return pin->s.slot<S>();
        return std::atomic_load(&p);
    }
    // The current snapshot whatever the thread has bound (compiles).
    template <class S>
    std::shared_ptr<const S> current(const std::shared_ptr<const S>& p) const {
        return std::atomic_load(&p);
    }
    template <class S>
    void publish(std::shared_ptr<const S>& slot, std::shared_ptr<const S> v);
    template <class S>
    void publish_raw(std::shared_ptr<const S>& slot, std::shared_ptr<const S> v) {
        std::atomic_store(&slot, std::move(v));
        // the previous tables' buffers, if no call pins them any more
        grave->drain();
    }
    // `s` is the caller's hipStream_t; NULL is HIP's null stream, as in
    // every HIP API (torch's default stream reports itself as 0).
    // CUs a stream may run on: its CU mask (hipExtStreamCreateWithCUMask),
    // so grids sized to one resident round fill a partitioned stream's share
    int stream_cus(hipStream_t s) const {
        uint32_t m[32] = {};
        if (hipExtStreamGetCUMask(s, 32, m) != hipSuccess) return num_cus;
        int k = 0;
        for (uint32_t w : m) k += __builtin_popcount(w);
        return k > 0 && k < num_cus ? k : num_cus;
    }
    vc::LaunchCfg cfg(void* s) const {
        vc::LaunchCfg c;
        c.stream = static_cast<hipStream_t>(s);
        c.num_cus = stream_cus(c.stream);
        c.cu_masked = c.num_cus < num_cus;
        c.handoff = vc::Handoff{handoff, const_cast<std::mutex*>(&handoff_mu)};
        c.scratch = const_cast<vc::ScratchRing*>(&scratch);
        c.http_scratch = const_cast<vc::ScratchRing*>(&http_scratch);
        c.tickets = const_cast<vc::TicketRing*>(&tickets);
        return c;
    }
};

namespace {

int set_dev(vc_ctx* ctx) {
    if (!ctx) return fail(VC_EINVAL, "null context");
    hipError_t e = hipSetDevice(ctx->device);
    return e == hipSuccess ? VC_OK : hip_fail(e, "hipSetDevice");
}

// Device-side check flags of a VC_DEVCHECK build (dev_common.h): the first
// failing site per kernel file, read and cleared.  Always empty otherwise.
int devcheck_report(const char* what) {
    uint32_t f[4] = {};
    if (vc::devcheck_take(f) != hipSuccess || f[0] == 0) return VC_OK;
    return fail(VC_EDEVICE, std::string(what) + ": device check failed at site " +
                                std::to_string(f[0]) + " (" + std::to_string(f[1]) +
                                " hits, detail " + std::to_string(f[2]) + ", " +
                                std::to_string(f[3]) + ")");
}

// The status of a launch: its launch error, and under VC_SYNC_CHECK the
// stream's completion and the device check flags, named by the entry point.
int launched(vc_ctx* ctx, hipError_t e, void* stream, const char* what) {
    if (e != hipSuccess) {
        ctx->tickets.mark_dirty();
        return hip_fail(e, what);
    }
    if (!ctx->sync_check) return VC_OK;
    e = hipStreamSynchronize(static_cast<hipStream_t>(stream));
    if (e == hipSuccess) e = hipGetLastError();
    if (e != hipSuccess) {
        ctx->tickets.mark_dirty();
        return hip_fail(e, (std::string(what) + " (sync check)").c_str());
    }
    return devcheck_report(what);
}

// An idle stager for one host-buffer call, returned when the call ends.
class StagerLease {
public:
    explicit StagerLease(vc_ctx* ctx) : ctx_(ctx) {
        {
            std::lock_guard<std::mutex> lk(ctx->stage_mu);
            if (!ctx->stagers.empty()) {
                st_ = std::move(ctx->stagers.back());
                ctx->stagers.pop_back();
                return;
            }
        }
        auto st = std::make_unique<Stager>();
        for (StageLane& l : st->lane)
            if ((err_ = hipStreamCreateWithFlags(&l.s, hipStreamNonBlocking)) != hipSuccess) {
                destroy(st.get());
                return;
            }
        st_ = std::move(st);
    }
    StagerLease(const StagerLease&) = delete;
    StagerLease& operator=(const StagerLease&) = delete;
    ~StagerLease() {
        if (!st_) return;
        // a call that failed part-way may leave copies in flight into the
        // lane's memory: wait for them before the stager is reused
        for (StageLane& l : st_->lane) (void)l.finish(false);
        std::lock_guard<std::mutex> lk(ctx_->stage_mu);
        ctx_->stagers.push_back(std::move(st_));
    }
    explicit operator bool() const { return st_ != nullptr; }
    hipError_t err() const { return err_; }
    StageLane& lane(int k) { return st_->lane[k]; }
    static void destroy(Stager* st) {
        for (StageLane& l : st->lane) {
            if (!l.s) continue;
            (void)hipStreamSynchronize(l.s);
            (void)hipStreamDestroy(l.s);
            l.s = nullptr;
            l.dev.release();
            l.host.release();
        }
    }

private:
    vc_ctx* ctx_;
    std::unique_ptr<Stager> st_;
    hipError_t err_ = hipSuccess;
};

// One call's (or one chunk's) staging on a lane: inputs copied host ->
// bounce -> device, outputs allocated on the device and copied back into
// the bounce buffer; finish() hands them to the caller's arrays.
struct Staging {
    vc_ctx* ctx;
    StageLane& L;
    const char* what;
    hipError_t err = hipSuccess;
    Staging(vc_ctx* c, StageLane& l, const char* w) : ctx(c), L(l), what(w) {}
    Staging(const Staging&) = delete;
    Staging& operator=(const Staging&) = delete;
    hipStream_t stream() const { return L.s; }
    void copied() {
        L.busy = true;
        if (err == hipSuccess && ctx->sync_check) {
            err = hipStreamSynchronize(L.s);
            if (err == hipSuccess) err = hipGetLastError();
        }
    }
    void* in(const void* h, size_t bytes) {
        if (!h || err != hipSuccess) return nullptr;
        void* d = L.dev.alloc(bytes, &err);
        auto* p = static_cast<uint8_t*>(err == hipSuccess && bytes ? L.host.alloc(bytes, &err)
                                                                   : nullptr);
        if (err != hipSuccess || !bytes) return d;
        for (size_t a = 0; a < bytes && err == hipSuccess; a += kPiece) {
            const size_t m = std::min(kPiece, bytes - a);
            CopyPool::get().copy(p + a, static_cast<const uint8_t*>(h) + a, m);
            err = hipMemcpyAsync(static_cast<uint8_t*>(d) + a, p + a, m, hipMemcpyHostToDevice,
                                 L.s);
            copied();
        }
        return d;
    }
    void* out(const void* h, size_t bytes) {
        if (!h || err != hipSuccess) return nullptr;
        return L.dev.alloc(bytes, &err);
    }
    void back(void* h, const void* d, size_t bytes) {
        if (!h || !d || !bytes || err != hipSuccess) return;
        auto* p = static_cast<uint8_t*>(L.host.alloc(bytes, &err));
        for (size_t a = 0; a < bytes && err == hipSuccess; a += kPiece) {
            const size_t m = std::min(kPiece, bytes - a);
            err = hipMemcpyAsync(p + a, static_cast<const uint8_t*>(d) + a, m,
                                 hipMemcpyDeviceToHost, L.s);
            if (err == hipSuccess)
                L.backs.push_back(StageLane::Back{static_cast<uint8_t*>(h) + a, p + a, m,
                                                  bytes > kPiece ? L.mark() : -1});
            copied();
        }
    }
    // status of the call: wait for the lane and deliver the results
    int finish() {
        const hipError_t e = err != hipSuccess ? err : L.finish(true);
        if (e != hipSuccess) {
            ctx->tickets.mark_dirty();
            return hip_fail(e, what);
        }
        return ctx->sync_check ? devcheck_report(what) : VC_OK;
    }
};

// A compile's uploads: host vectors through a stager's bounce buffer into
// device buffers the snapshot owns, on lane 2's stream, waited for once.
struct Upload {
    vc_ctx* ctx;
    StagerLease lease;
    hipError_t err;
    explicit Upload(vc_ctx* c) : ctx(c), lease(c), err(lease.err()) {}
    StageLane& L() { return lease.lane(2); }
    void* dev(Snapshot& s, size_t bytes);
    template <class T>
    const T* operator()(Snapshot& s, const std::vector<T>& v) {
        void* d = dev(s, v.size() * sizeof(T));
        if (d && !v.empty() && err == hipSuccess) {
            const size_t bytes = v.size() * sizeof(T);
            void* p = L().host.alloc(bytes, &err);
            if (err != hipSuccess) return nullptr;
            CopyPool::get().copy(p, v.data(), bytes);
            L().busy = true;
            err = hipMemcpyAsync(d, p, bytes, hipMemcpyHostToDevice, L().s);
        }
        return static_cast<const T*>(d);
    }
    // zero-filled device counters
    unsigned long long* zeros(Snapshot& s, int64_t n) {
        const size_t bytes = size_t(std::max<int64_t>(n, 1)) * 8;
        void* d = dev(s, bytes);
        if (d && err == hipSuccess) {
            L().busy = true;
            err = hipMemsetAsync(d, 0, bytes, L().s);
        }
        return static_cast<unsigned long long*>(d);
    }
    hipError_t done() {
        if (!lease) return err;
        const hipError_t e = L().finish(false);
        return err != hipSuccess ? err : e;
    }
};

struct Snapshot {
    std::vector<std::unique_ptr<DevBuf>> bufs;
    unsigned long long* counters = nullptr;
    int64_t n_counters = 0;
    uint64_t digest = 0;           // vc::digest of the host-built image (vc_table_digest)
    mutable uint64_t gen = 0;      // set once by vc_ctx::publish (vc_pin_generation)

    void alloc_counters(Upload& up, int64_t n) {
        counters = up.zeros(*this, n);
        n_counters = n;
    }
};

void* Upload::dev(Snapshot& s, size_t bytes) {
    if (err != hipSuccess) return nullptr;
    auto b = std::make_unique<DevBuf>();
    b->n = std::max<size_t>(bytes, 16);
    b->grave = ctx->grave;
    err = hipMalloc(&b->p, b->n);
    if (err != hipSuccess) {
        b->p = nullptr;
        return nullptr;
    }
    void* p = b->p;
    s.bufs.push_back(std::move(b));
    return p;
}

// intervals of an AclPortImage the switch kernel copies into LDS
// (packet.hip kSwitchPortMax)
constexpr int kAclPortMax = 256;

struct AclSnap : Snapshot {
    AclImage img{};
    // The UDP list's IPv4 image at the Switch's VXLAN bind port
    // (images.h AclPortImage): built by a compile for every bind port a
    // switch call has used on this context, and on the first call with a new
    // one (acl_port_image); kept with the snapshot.
    std::shared_ptr<const vc::AclFamilyBuilt> udp4;   // the UDP list's IPv4 image, host side
    bool port_images = true;       // VC_ACL_PORT=0 at compile: general image only (A/B)
    mutable std::mutex port_mu;
    mutable std::map<int32_t, AclPortImage> ports;
    mutable std::vector<std::unique_ptr<DevBuf>> port_bufs;
};
struct RouteSnap : Snapshot {
    RouteImage img{};
    int32_t n4 = 0, n6 = 0;
};
struct VniSnap : Snapshot {
    VniImage img{};
};
struct HintSnap : Snapshot {
    HintImage img{};
};
struct HostsSnap : Snapshot {
    HostsImage img{};
};
struct CertSnap : Snapshot {
    CertImage img{};
};
struct MirrorSnap : Snapshot {
    MirrorImage img{};
    std::map<int32_t, MirrorSwImage> sw;   // per origin: switchPacket's bit-set image
};
struct ServerSnap : Snapshot {
    ServerImage img{};
    // A health update publishes a new snapshot that owns a fresh healthy[]
    // and shares the compiled lists of the snapshot vc_compile_servers made
    // (kept alive through `lists`), so a batch keeps one health view for all
    // of its chunks.
    std::shared_ptr<const ServerSnap> lists;
    // the host-built lists, for the pick table a health update rebuilds
    std::shared_ptr<const vc::ServersBuilt> host;
};

}  // namespace

// Every publish takes the context's next generation, so a pin can report
// which compile each of its snapshots came from (vc_pin_generation).
template <class S>
void vc_ctx::publish(std::shared_ptr<const S>& slot, std::shared_ptr<const S> v) {
    if (v) v->gen = next_gen.fetch_add(1, std::memory_order_relaxed);
    publish_raw(slot, std::move(v));
}

extern "C" {

const char* vc_version(void) { return "vclassify 0.1 (gfx950)"; }

const char* vc_last_error(void) { return g_err.c_str(); }

int vc_create(int device, vc_ctx** out) {
    if (!out) return fail(VC_EINVAL, "null out");
    *out = nullptr;
    int count = 0;
    hipError_t e = hipGetDeviceCount(&count);
    if (e != hipSuccess || count <= 0) return fail(VC_EDEVICE, "no HIP device available");
    if (device < 0 || device >= count) return fail(VC_EINVAL, "bad device ordinal");
    hipDeviceProp_t prop;
    e = hipGetDeviceProperties(&prop, device);
    if (e != hipSuccess) return hip_fail(e, "hipGetDeviceProperties");
    if (std::strncmp(prop.gcnArchName, "gfx950", 6) != 0)
        return fail(VC_EDEVICE, std::string("libvclassify is built for gfx950, device is ") +
                                    prop.gcnArchName);
    auto* c = new vc_ctx();
    c->device = device;
    c->num_cus = prop.multiProcessorCount;
    const char* sc = std::getenv("VC_SYNC_CHECK");
    c->sync_check = sc && *sc && std::strcmp(sc, "0") != 0;
    if ((e = hipSetDevice(device)) != hipSuccess ||
        (e = hipStreamCreateWithFlags(&c->stream, hipStreamNonBlocking)) != hipSuccess ||
        (e = hipEventCreateWithFlags(&c->handoff, hipEventDisableTiming)) != hipSuccess ||
        (e = c->scratch.init()) != hipSuccess || (e = c->http_scratch.init(false)) != hipSuccess ||
        (e = c->tickets.init()) != hipSuccess) {
        c->scratch.destroy();
        c->http_scratch.destroy();
        c->tickets.destroy();
        if (c->handoff) (void)hipEventDestroy(c->handoff);
        if (c->stream) (void)hipStreamDestroy(c->stream);
        delete c;
        return hip_fail(e, "context create");
    }
    *out = c;
    return VC_OK;
}

void vc_destroy(vc_ctx* ctx) {
    if (!ctx) return;
    (void)hipSetDevice(ctx->device);
    // batches may still run on callers' streams and read the tables
    (void)hipDeviceSynchronize();
    ctx->acl.reset();
    ctx->route.reset();
    ctx->hint.reset();
    ctx->hosts.reset();
    ctx->servers.reset();
    ctx->certs.reset();
    ctx->mirror.reset();
    ctx->vni.reset();
    if (t_pin && t_pin->ctx == ctx) t_pin = nullptr;
    ctx->grave->drain();
    for (auto& st : ctx->stagers) StagerLease::destroy(st.get());
    ctx->stagers.clear();
    (void)hipStreamDestroy(ctx->stream);
    if (ctx->handoff) (void)hipEventDestroy(ctx->handoff);
    ctx->scratch.destroy();
    ctx->http_scratch.destroy();
    ctx->tickets.destroy();
    delete ctx;
}

// ---------------------------------------------------------------------------
// Snapshot pins (SURVEY.md §8(b) "Threading")
// ---------------------------------------------------------------------------
static const Snapshot* slot_snap(const SnapSet& s, int kind) {
    switch (kind) {
    case VC_SNAP_ACL: return s.acl.get();
    case VC_SNAP_ROUTE: return s.route.get();
    case VC_SNAP_UPSTREAM: return s.hint.get();
    case VC_SNAP_HOSTS: return s.hosts.get();
    case VC_SNAP_SERVERS: return s.servers.get();
    case VC_SNAP_CERTS: return s.certs.get();
    case VC_SNAP_MIRROR: return s.mirror.get();
    case VC_SNAP_VNI: return s.vni.get();
    default: return nullptr;
    }
}

int vc_pin_acquire(vc_ctx* ctx, uint32_t kinds, vc_pin** out) {
    if (!ctx || !out) return fail(VC_EINVAL, "null argument");
    *out = nullptr;
    if (kinds & ~uint32_t(VC_SNAP_ALL)) return fail(VC_EINVAL, "unknown snapshot kind bits");
    auto* p = new (std::nothrow) vc_pin();
    if (!p) return fail(VC_ENOMEM, "pin");
    p->ctx = ctx;
    p->kinds = kinds;
    // each slot on its own atomic load: a compile of one kind publishes
    // one slot, so the set is what the calls of a batch would have seen
    // had they started now
    if (kinds >> VC_SNAP_ACL & 1) p->s.acl = ctx->current(ctx->acl);
    if (kinds >> VC_SNAP_ROUTE & 1) p->s.route = ctx->current(ctx->route);
    if (kinds >> VC_SNAP_UPSTREAM & 1) p->s.hint = ctx->current(ctx->hint);
    if (kinds >> VC_SNAP_HOSTS & 1) p->s.hosts = ctx->current(ctx->hosts);
    if (kinds >> VC_SNAP_SERVERS & 1) p->s.servers = ctx->current(ctx->servers);
    if (kinds >> VC_SNAP_CERTS & 1) p->s.certs = ctx->current(ctx->certs);
    if (kinds >> VC_SNAP_MIRROR & 1) p->s.mirror = ctx->current(ctx->mirror);
    if (kinds >> VC_SNAP_VNI & 1) p->s.vni = ctx->current(ctx->vni);
    *out = p;
    return VC_OK;
}

int vc_pin_bind(vc_ctx* ctx, const vc_pin* pin) {
    if (!ctx) return fail(VC_EINVAL, "null context");
    if (pin && pin->ctx != ctx) return fail(VC_EINVAL, "pin belongs to another context");
    t_pin = pin;
    return VC_OK;
}

int vc_pin_generation(const vc_pin* pin, int kind, uint64_t* gen) {
    if (!pin || !gen) return fail(VC_EINVAL, "null argument");
    if (kind < 0 || kind > VC_SNAP_VNI) return fail(VC_EINVAL, "bad snapshot kind");
    if (!(pin->kinds >> kind & 1)) return fail(VC_EINVAL, "kind not pinned");
    const Snapshot* s = slot_snap(pin->s, kind);
    *gen = s ? s->gen : 0;
    return VC_OK;
}

void vc_pin_release(vc_pin* pin) {
    if (!pin) return;
    if (t_pin == pin) t_pin = nullptr;
    // the last reference to a replaced snapshot sends its buffers to the
    // graveyard; the next compile frees them
    delete pin;
}

int vc_generation(vc_ctx* ctx, int kind, uint64_t* gen) {
    if (!ctx || !gen) return fail(VC_EINVAL, "null argument");
    if (kind < 0 || kind > VC_SNAP_VNI) return fail(VC_EINVAL, "bad snapshot kind");
    SnapSet cur;
    switch (kind) {
    case VC_SNAP_ACL: cur.acl = ctx->current(ctx->acl); break;
    case VC_SNAP_ROUTE: cur.route = ctx->current(ctx->route); break;
    case VC_SNAP_UPSTREAM: cur.hint = ctx->current(ctx->hint); break;
    case VC_SNAP_HOSTS: cur.hosts = ctx->current(ctx->hosts); break;
    case VC_SNAP_SERVERS: cur.servers = ctx->current(ctx->servers); break;
    case VC_SNAP_CERTS: cur.certs = ctx->current(ctx->certs); break;
    case VC_SNAP_MIRROR: cur.mirror = ctx->current(ctx->mirror); break;
    default: cur.vni = ctx->current(ctx->vni); break;
    }
    const Snapshot* s = slot_snap(cur, kind);
    *gen = s ? s->gen : 0;
    return VC_OK;
}

// ---------------------------------------------------------------------------
// Network helpers
// ---------------------------------------------------------------------------
int vc_net_parse(const char* s, vc_net* out) {
    if (!s || !out) return fail(VC_EINVAL, "null argument");
    if (!vc::net_parse(s, out)) return fail(VC_EINVAL, std::string("invalid network ") + s);
    return VC_OK;
}

int vc_net_from_prefix(const uint8_t* ip, int ip_len, int prefix, vc_net* out) {
    if (!ip || !out) return fail(VC_EINVAL, "null argument");
    if (!vc::net_from_prefix(ip, ip_len, prefix, out)) return fail(VC_EINVAL, "invalid network");
    return VC_OK;
}

int vc_net_contains_ip(const vc_net* net, const uint8_t* ip, int ip_len) {
    if (!net || !ip || (ip_len != 4 && ip_len != 16)) return fail(VC_EINVAL, "bad argument");
    return vc::net_contains_ip(*net, ip, ip_len) ? 1 : 0;
}

int vc_ip_parse(const char* s, uint8_t out[16]) {
    if (!s || !out) return fail(VC_EINVAL, "null argument");
    auto ip = vc::parse_ip(s);
    if (!ip) return fail(VC_EINVAL, std::string("not an ip literal: ") + s);
    std::memcpy(out, ip->b.data(), ip->len);
    return ip->len;
}

// ---------------------------------------------------------------------------
// ACL
// ---------------------------------------------------------------------------
int vc_compile_acl(vc_ctx* ctx, const vc_acl_rule* tcp, int n_tcp, const vc_acl_rule* udp,
                   int n_udp, int default_allow) {
    int rc = set_dev(ctx);
    if (rc) return rc;
    if ((n_tcp && !tcp) || (n_udp && !udp)) return fail(VC_EINVAL, "null rule array");
    vc::AclBuilt b;
    rc = vc::build_acl(tcp, n_tcp, udp, n_udp, default_allow, &b);
    if (rc) return fail(rc, "invalid SecurityGroup rule (network must be a valid Network)");
    std::lock_guard<std::mutex> lk(ctx->compile_mu);
    auto s = std::make_shared<AclSnap>();
    Upload up(ctx);
    for (int l = 0; l < 2; ++l)
        for (int f = 0; f < 2; ++f) {
            const vc::AclFamilyBuilt& fb = b.fam[l][f];
            AclFamilyImage& fi = s->img.fam[l][f];
            fi.bounds4 = f == 0 ? up(*s, fb.bounds4) : nullptr;
            fi.bounds6 = f == 1 ? up(*s, fb.bounds6) : nullptr;
            fi.rec = up(*s, fb.rec);
            fi.pieces = up(*s, fb.pieces);
            fi.dir4 = fb.dir4.empty() ? nullptr : up(*s, fb.dir4);
            fi.dir_bits = fb.dir4.empty() ? 0 : fb.dir_bits;
            fi.nb = fb.nb;
            fi.np = static_cast<int32_t>(fb.pieces.size() / 2);
            fi.v4_only = fb.v4_only;
        }
    s->img.allow = up(*s, b.allow);
    s->img.n_tcp = b.n_tcp;
    s->img.n_udp = b.n_udp;
    s->img.default_allow = b.default_allow;
    s->digest = vc::digest(b);
    s->alloc_counters(up, int64_t(n_tcp) + n_udp + 2);
    const char* env = std::getenv("VC_ACL_PORT");
    s->port_images = !(env && env[0] == '0');
    if (s->port_images) {
        std::set<int32_t> seen;
        {
            std::lock_guard<std::mutex> lk(ctx->port_seen_mu);
            seen = ctx->acl_ports_seen;
        }
        for (const int32_t port : seen) {
            std::vector<uint32_t> pb, pv;
            vc::build_acl_port(b.fam[1][0], uint32_t(port), &pb, &pv);
            AclPortImage im{nullptr, nullptr, 0, port};
            if (pb.size() <= size_t(kAclPortMax)) {
                im.bounds = up(*s, pb);
                im.value = up(*s, pv);
                im.nb = int32_t(pb.size());
            }
            s->ports[port] = im;
        }
    }
    if (const hipError_t e = up.done(); e != hipSuccess) return hip_fail(e, "ACL upload");
    if (s->port_images) s->udp4 = std::make_shared<const vc::AclFamilyBuilt>(std::move(b.fam[1][0]));
    ctx->publish(ctx->acl, std::shared_ptr<const AclSnap>(std::move(s)));
    return VC_OK;
}

// `pin`: the snapshot a chunked host call took once for all its chunks
// (a call classifies against the tables it started with).
static int acl_dev(vc_ctx* ctx, int fam, const uint8_t* proto, const void* src,
                   const uint16_t* port, int64_t n, int32_t* out_idx, uint8_t* out_allow,
                   void* stream, std::shared_ptr<const AclSnap> pin = nullptr) {
    int rc = set_dev(ctx);
    if (rc) return rc;
    if (n < 0 || (n > 0 && (!proto || !src || !port || !out_idx)))
        return fail(VC_EINVAL, "bad batch arguments");
    auto s = pin ? pin : ctx->get(ctx->acl);
    if (!s) return fail(VC_ESTATE, "no SecurityGroup compiled");
    unsigned long long* cnt = ctx->counters_on ? s->counters : nullptr;
    hipError_t e = fam == 4
        ? vc::launch_acl_v4(ctx->cfg(stream), s->img, proto, static_cast<const uint32_t*>(src),
                            port, n, out_idx, out_allow, cnt)
        : vc::launch_acl_v6(ctx->cfg(stream), s->img, proto, static_cast<const uint8_t*>(src),
                            port, n, out_idx, out_allow, cnt);
    return launched(ctx, e, stream, "ACL launch");
}

int vc_acl_classify_v4_dev(vc_ctx* ctx, const uint8_t* proto, const uint32_t* src4,
                           const uint16_t* port, int64_t n, int32_t* out_idx, uint8_t* out_allow,
                           void* stream) {
    return acl_dev(ctx, 4, proto, src4, port, n, out_idx, out_allow, stream);
}

int vc_acl_classify_v6_dev(vc_ctx* ctx, const uint8_t* proto, const uint8_t* src6,
                           const uint16_t* port, int64_t n, int32_t* out_idx, uint8_t* out_allow,
                           void* stream) {
    return acl_dev(ctx, 6, proto, src6, port, n, out_idx, out_allow, stream);
}

// Host-buffer batches of fixed-size items in chunks: chunk k's upload,
// kernel and download are ordered on lane k % 2, so one chunk's H2D copy,
// the next chunk's kernel and the previous chunk's D2H copy overlap (PCIe is
// full duplex).
constexpr int64_t kHostChunk = int64_t(4) << 20;

// Buffers registered through vc_host_register: base -> length.  A zero-copy
// call needs every array's whole extent [p, p + bytes) inside one of them; a
// short registration (or one made by someone else, whose extent we do not
// know) falls back to chunked staging instead of faulting on the device.
static std::mutex g_reg_mu;
static std::map<uintptr_t, size_t> g_reg;

// Device address of `bytes` bytes at h inside a page-locked, mapped host
// buffer (vc_host_register), or null -- ordinary pageable memory, a range
// the registration does not cover, or a device address that is not
// `align`-aligned (IPv6 arrays are read as 16-byte words).  Kernels then read
// their inputs and write their outputs across PCIe directly (both directions
// at once).
static void* mapped(const void* h, size_t bytes, uintptr_t align = 1) {
    if (!h) return nullptr;
    {
        const uintptr_t p = reinterpret_cast<uintptr_t>(h);
        std::lock_guard<std::mutex> lk(g_reg_mu);
        auto it = g_reg.upper_bound(p);
        if (it == g_reg.begin()) return nullptr;
        --it;
        if (p - it->first > it->second || bytes > it->second - (p - it->first)) return nullptr;
    }
    hipPointerAttribute_t a{};
    if (hipPointerGetAttributes(&a, h) != hipSuccess) {
        (void)hipGetLastError();
        return nullptr;
    }
    if (a.type != hipMemoryTypeHost || !a.devicePointer) return nullptr;
    if (reinterpret_cast<uintptr_t>(a.devicePointer) & (align - 1)) return nullptr;
    return a.devicePointer;
}

extern "C++" {
// Chunk k runs on lane k % 2 of one stager: its inputs are copied into the
// lane's bounce buffer and uploaded, the kernel runs, and its outputs come
// back into the bounce buffer, all in the lane's stream order.  Before a
// lane takes chunk k + 2 the host waits for chunk k and copies its results
// out, so one lane's transfers and kernel overlap the other lane's and the
// host copies.
template <class Body>   // int body(Staging&, int64_t lo, int64_t cnt, hipStream_t)
static int host_chunks(vc_ctx* ctx, StagerLease& lease, int64_t n, const char* what, Body body) {
    if (!lease) return hip_fail(lease.err(), what);
    int rc = VC_OK;
    for (int64_t lo = 0, k = 0; lo < n && rc == VC_OK; lo += kHostChunk, ++k) {
        StageLane& L = lease.lane(int(k & 1));
        const hipError_t e = L.finish(true);            // chunk k - 2's results
        if (e != hipSuccess) {
            rc = hip_fail(e, what);
            break;
        }
        Staging st(ctx, L, what);
        rc = body(st, lo, std::min(kHostChunk, n - lo), st.stream());
        if (rc == VC_OK && st.err != hipSuccess) rc = hip_fail(st.err, what);
    }
    for (int k = 0; k < 2; ++k) {
        const hipError_t e = lease.lane(k).finish(rc == VC_OK);
        if (rc == VC_OK && e != hipSuccess) rc = hip_fail(e, what);
    }
    if (rc == VC_OK && ctx->sync_check) rc = devcheck_report(what);
    return rc;
}
template <class Body>
static int host_chunks(vc_ctx* ctx, int64_t n, const char* what, Body body) {
    StagerLease lease(ctx);
    return host_chunks(ctx, lease, n, what, body);
}
}  // extern "C++"

static int acl_host(vc_ctx* ctx, int fam, const uint8_t* proto, const void* src,
                    const uint16_t* port, int64_t n, int32_t* out_idx, uint8_t* out_allow) {
    int rc = set_dev(ctx);
    if (rc) return rc;
    if (n <= 0) return n == 0 ? VC_OK : fail(VC_EINVAL, "negative n");
    if (!proto || !src || !port || !out_idx) return fail(VC_EINVAL, "bad batch arguments");
    const size_t sw = fam == 4 ? 4 : 16, un = size_t(n);
    void *mp = mapped(proto, un), *ms = mapped(src, un * sw, sw), *mq = mapped(port, un * 2);
    void *mi = mapped(out_idx, un * 4), *ma = mapped(out_allow, un);
    if (mp && ms && mq && mi && (!out_allow || ma)) {            // zero-copy
        rc = acl_dev(ctx, fam, static_cast<uint8_t*>(mp), ms, static_cast<uint16_t*>(mq), n,
                     static_cast<int32_t*>(mi), static_cast<uint8_t*>(ma), ctx->stream);
        if (rc) return rc;
        hipError_t e = hipStreamSynchronize(ctx->stream);
        if (e != hipSuccess) return hip_fail(e, "ACL classify");
        return ctx->sync_check ? devcheck_report("ACL classify") : VC_OK;
    }
    const auto pin = ctx->get(ctx->acl);
    return host_chunks(ctx, n, "ACL classify", [&](Staging& st, int64_t lo, int64_t c,
                                                   hipStream_t s) {
        const size_t u = size_t(lo), m = size_t(c);
        auto* dp = static_cast<uint8_t*>(st.in(proto + u, m));
        auto* ds = st.in(static_cast<const uint8_t*>(src) + u * sw, m * sw);
        auto* dq = static_cast<uint16_t*>(st.in(port + u, m * 2));
        auto* di = static_cast<int32_t*>(st.out(out_idx, m * 4));
        auto* da = static_cast<uint8_t*>(st.out(out_allow, m));
        if (st.err != hipSuccess) return VC_OK;               // reported by host_chunks
        int r = acl_dev(ctx, fam, dp, ds, dq, c, di, da, s, pin);
        if (r) return r;
        st.back(out_idx + u, di, m * 4);
        if (out_allow) st.back(out_allow + u, da, m);
        return VC_OK;
    });
}

int vc_acl_classify_v4(vc_ctx* ctx, const uint8_t* proto, const uint32_t* src4,
                       const uint16_t* port, int64_t n, int32_t* out_idx, uint8_t* out_allow) {
    return acl_host(ctx, 4, proto, src4, port, n, out_idx, out_allow);
}

int vc_acl_classify_v6(vc_ctx* ctx, const uint8_t* proto, const uint8_t* src6,
                       const uint16_t* port, int64_t n, int32_t* out_idx, uint8_t* out_allow) {
    return acl_host(ctx, 6, proto, src6, port, n, out_idx, out_allow);
}

// ---------------------------------------------------------------------------
// Routes
// ---------------------------------------------------------------------------
int vc_compile_routes(vc_ctx* ctx, const vc_net* v4, int n4, const vc_net* v6, int n6) {
    int rc = set_dev(ctx);
    if (rc) return rc;
    if ((n4 && !v4) || (n6 && !v6) || n4 < 0 || n6 < 0) return fail(VC_EINVAL, "bad rule arrays");
    vc::TrieBuilt t4, t6;
    if ((rc = vc::build_trie(v4, n4, 0, &t4)) != VC_OK) return fail(rc, "invalid IPv4 route rule");
    if ((rc = vc::build_trie(v6, n6, 1, &t6)) != VC_OK) return fail(rc, "invalid IPv6 route rule");
    std::lock_guard<std::mutex> lk(ctx->compile_mu);
    auto s = std::make_shared<RouteSnap>();
    Upload up(ctx);
    vc::TrieBuilt* tb[2] = {&t4, &t6};
    for (int f = 0; f < 2; ++f) {
        s->img.fam[f].nodes = up(*s, tb[f]->nodes);
        s->img.fam[f].root_bits = tb[f]->root_bits;
        s->img.fam[f].key_bits = tb[f]->key_bits;
        s->img.fam[f].n_rules = tb[f]->n_rules;
    }
    // the IPv6 wide root (images.h TrieImage.wide), expanded on the device
    // from the uploaded root and records; VC_ROUTE6_WIDE=0 leaves it out
    static const bool wide6 = [] {
        const char* w = std::getenv("VC_ROUTE6_WIDE");
        return !(w && std::strcmp(w, "0") == 0);
    }();
    if (wide6 && n6 > 0) {
        const size_t bytes = (size_t(1) << t6.root_bits) * 16;
        auto* w = static_cast<uint32_t*>(up.dev(*s, bytes));
        if (w && up.err == hipSuccess) {
            up.L().busy = true;
            up.err = vc::build_wide_root(s->img.fam[1].nodes, t6.root_bits, w, up.L().s);
            s->img.fam[1].wide = w;
        }
    }
    s->n4 = n4;
    s->n6 = n6;
    s->digest = vc::digest(t4, t6);
    s->alloc_counters(up, int64_t(n4) + n6 + 2);
    if (const hipError_t e = up.done(); e != hipSuccess) return hip_fail(e, "route upload");
    ctx->publish(ctx->route, std::shared_ptr<const RouteSnap>(std::move(s)));
    return VC_OK;
}

static int route_dev(vc_ctx* ctx, int fam, const void* dst, int64_t n, int32_t* out, void* stream,
                     std::shared_ptr<const RouteSnap> pin = nullptr) {
    int rc = set_dev(ctx);
    if (rc) return rc;
    if (n < 0 || (n > 0 && (!dst || !out))) return fail(VC_EINVAL, "bad batch arguments");
    auto s = pin ? pin : ctx->get(ctx->route);
    if (!s) return fail(VC_ESTATE, "no RouteTable compiled");
    unsigned long long* cnt = ctx->counters_on ? s->counters : nullptr;
    const int64_t nn = int64_t(s->n4) + s->n6;
    hipError_t e = fam == 4
        ? vc::launch_route_v4(ctx->cfg(stream), s->img.fam[0], static_cast<const uint32_t*>(dst),
                              n, out, cnt, 0, nn)
        : vc::launch_route_v6(ctx->cfg(stream), s->img.fam[1], static_cast<const uint8_t*>(dst),
                              n, out, cnt, s->n4, nn + 1);
    return launched(ctx, e, stream, "route launch");
}

int vc_route_lookup_v4_dev(vc_ctx* ctx, const uint32_t* dst4, int64_t n, int32_t* out,
                           void* stream) {
    return route_dev(ctx, 4, dst4, n, out, stream);
}

int vc_route_lookup_v6_dev(vc_ctx* ctx, const uint8_t* dst6, int64_t n, int32_t* out,
                           void* stream) {
    return route_dev(ctx, 6, dst6, n, out, stream);
}

static int route_host(vc_ctx* ctx, int fam, const void* dst, int64_t n, int32_t* out) {
    int rc = set_dev(ctx);
    if (rc) return rc;
    if (n <= 0) return n == 0 ? VC_OK : fail(VC_EINVAL, "negative n");
    if (!dst || !out) return fail(VC_EINVAL, "bad batch arguments");
    const size_t sw = fam == 4 ? 4 : 16;
    void *md = mapped(dst, size_t(n) * sw, sw), *mo = mapped(out, size_t(n) * 4);
    if (md && mo) {                                              // zero-copy
        rc = route_dev(ctx, fam, md, n, static_cast<int32_t*>(mo), ctx->stream);
        if (rc) return rc;
        hipError_t e = hipStreamSynchronize(ctx->stream);
        if (e != hipSuccess) return hip_fail(e, "route lookup");
        return ctx->sync_check ? devcheck_report("route lookup") : VC_OK;
    }
    const auto pin = ctx->get(ctx->route);
    return host_chunks(ctx, n, "route lookup", [&](Staging& st, int64_t lo, int64_t c,
                                                   hipStream_t s) {
        const size_t u = size_t(lo), m = size_t(c);
        void* dd = st.in(static_cast<const uint8_t*>(dst) + u * sw, m * sw);
        auto* dout = static_cast<int32_t*>(st.out(out, m * 4));
        if (st.err != hipSuccess) return VC_OK;
        int r = route_dev(ctx, fam, dd, c, dout, s, pin);
        if (r) return r;
        st.back(out + u, dout, m * 4);
        return VC_OK;
    });
}

int vc_route_lookup_v4(vc_ctx* ctx, const uint32_t* dst4, int64_t n, int32_t* out) {
    return route_host(ctx, 4, dst4, n, out);
}

int vc_route_lookup_v6(vc_ctx* ctx, const uint8_t* dst6, int64_t n, int32_t* out) {
    return route_host(ctx, 6, dst6, n, out);
}

int vc_compile_vni_routes(vc_ctx* ctx, const int32_t* vni, const vc_net* v4, const int32_t* v4_off,
                          const vc_net* v6, const int32_t* v6_off, int n_tables) {
    int rc = set_dev(ctx);
    if (rc) return rc;
    if (n_tables < 0 || (n_tables > 0 && (!vni || !v4_off || !v6_off)))
        return fail(VC_EINVAL, "bad table arrays");
    std::vector<int> order(static_cast<size_t>(n_tables));
    for (int t = 0; t < n_tables; ++t) {
        order[size_t(t)] = t;
        if (vni[t] < 0 || vni[t] > 0xFFFFFF) return fail(VC_EINVAL, "vni out of range");
        if (v4_off[t] < 0 || v4_off[t + 1] < v4_off[t] || v6_off[t] < 0 || v6_off[t + 1] < v6_off[t])
            return fail(VC_EINVAL, "bad rule offsets");
    }
    if (n_tables > 0 && ((v4_off[n_tables] > 0 && !v4) || (v6_off[n_tables] > 0 && !v6)))
        return fail(VC_EINVAL, "null rule array");
    std::sort(order.begin(), order.end(), [&](int a, int b) { return vni[a] < vni[b]; });
    for (int k = 1; k < n_tables; ++k)
        if (vni[order[size_t(k)]] == vni[order[size_t(k - 1)]])
            return fail(VC_EEXIST, "vni defined twice: " + std::to_string(vni[order[size_t(k)]]));
    std::vector<vc::TrieBuilt> tries(static_cast<size_t>(2 * n_tables));
    for (int k = 0; k < n_tables; ++k) {
        const int t = order[size_t(k)];
        if ((rc = vc::build_trie(v4 + v4_off[t], v4_off[t + 1] - v4_off[t], 0,
                                 &tries[size_t(2 * k)])) != VC_OK)
            return fail(rc, "invalid IPv4 route rule in vni " + std::to_string(vni[t]));
        if ((rc = vc::build_trie(v6 + v6_off[t], v6_off[t + 1] - v6_off[t], 1,
                                 &tries[size_t(2 * k + 1)])) != VC_OK)
            return fail(rc, "invalid IPv6 route rule in vni " + std::to_string(vni[t]));
    }
    std::lock_guard<std::mutex> lk(ctx->compile_mu);
    if (n_tables == 0) {
        ctx->publish(ctx->vni, std::shared_ptr<const VniSnap>());
        return VC_OK;
    }
    auto s = std::make_shared<VniSnap>();
    Upload up(ctx);
    std::vector<RouteImage> imgs(static_cast<size_t>(n_tables));
    std::vector<uint32_t> keys(static_cast<size_t>(n_tables));
    for (int k = 0; k < n_tables; ++k) {
        keys[size_t(k)] = uint32_t(vni[order[size_t(k)]]);
        for (int f = 0; f < 2; ++f) {
            const vc::TrieBuilt& tb = tries[size_t(2 * k + f)];
            TrieImage& ti = imgs[size_t(k)].fam[f];
            ti.nodes = up(*s, tb.nodes);
            ti.root_bits = tb.root_bits;
            ti.key_bits = tb.key_bits;
            ti.n_rules = tb.n_rules;
        }
    }
    s->img.vni = up(*s, keys);
    s->img.tables = up(*s, imgs);
    s->img.n = n_tables;
    if (const hipError_t e = up.done(); e != hipSuccess) return hip_fail(e, "vni route upload");
    ctx->publish(ctx->vni, std::shared_ptr<const VniSnap>(std::move(s)));
    return VC_OK;
}

// ---------------------------------------------------------------------------
// Upstream hints + DNS
// ---------------------------------------------------------------------------
int vc_compile_upstream(vc_ctx* ctx, const vc_group_annos* groups, int n) {
    int rc = set_dev(ctx);
    if (rc) return rc;
    if (n < 0 || (n && !groups)) return fail(VC_EINVAL, "bad group array");
    vc::HintBuilt b;
    if ((rc = vc::build_hints(groups, n, &b)) != VC_OK) return fail(rc, "invalid annotations");
    std::lock_guard<std::mutex> lk(ctx->compile_mu);
    auto s = std::make_shared<HintSnap>();
    Upload up(ctx);
    static_assert(sizeof(KeySlot) == sizeof(vc::KeySlotH), "slot layout");
    static_assert(sizeof(HostRec) == 64 && sizeof(HostExt) == 16, "record layout");
    s->img.blob = up(*s, b.blob);
    s->img.host_recs = up(*s, b.host.recs);
    s->img.host_ext = up(*s, b.host.ext);
    s->img.host_tags = up(*s, b.host.tags);
    s->img.uri_slots = reinterpret_cast<const KeySlot*>(up(*s, b.uri_slots));
    s->img.uri_tags = up(*s, b.uri_tags);
    s->img.lists = up(*s, b.lists);
    s->img.port_mins = reinterpret_cast<const PortMin*>(up(*s, b.port_mins));
    s->img.groups = reinterpret_cast<const GroupRec*>(up(*s, b.groups));
    s->img.host_mask = static_cast<uint32_t>(b.host.tags.size() - 1);
    s->img.uri_mask = static_cast<uint32_t>(b.uri_slots.size() - 1);
    s->img.n_groups = n;
    s->img.wildcard_slot = b.wildcard_slot;
    s->img.uri_star_slot = b.uri_star_slot;
    s->img.has_uri_keys = b.has_uri_keys;
    s->img.uri_len_lo = uint32_t(b.uri_len_mask);
    s->img.uri_len_hi = uint32_t(b.uri_len_mask >> 32);
    if (b.wildcard_slot >= 0) {
        const auto& w = b.host.recs[size_t(b.wildcard_slot)];
        s->img.wild_len_pm = w.len_pm;
        s->img.wild_a = w.a;
        s->img.wild_b = w.b;
    }
    s->digest = vc::digest(b);
    s->alloc_counters(up, int64_t(n) + 1);
    if (const hipError_t e = up.done(); e != hipSuccess) return hip_fail(e, "hint upload");
    ctx->publish(ctx->hint, std::shared_ptr<const HintSnap>(std::move(s)));
    return VC_OK;
}

int vc_hint_search_dev(vc_ctx* ctx, const uint8_t* host_blob, const uint32_t* host_off,
                       const uint8_t* host_null, const uint16_t* port, const uint8_t* uri_blob,
                       const uint32_t* uri_off, const uint8_t* uri_null, int64_t n,
                       int32_t* out_group, void* stream) {
    int rc = set_dev(ctx);
    if (rc) return rc;
    if (n < 0 || (n > 0 && !out_group) || (host_blob && !host_off) || (uri_blob && !uri_off))
        return fail(VC_EINVAL, "bad batch arguments");
    auto s = ctx->get(ctx->hint);
    if (!s) return fail(VC_ESTATE, "no Upstream compiled");
    hipError_t e = vc::launch_hint(ctx->cfg(stream), s->img, host_blob, host_off, host_null, port,
                                   uri_blob, uri_off, uri_null, n, out_group,
                                   ctx->counters_on ? s->counters : nullptr);
    return launched(ctx, e, stream, "hint launch");
}

int vc_hint_search(vc_ctx* ctx, const uint8_t* host_blob, const uint32_t* host_off,
                   const uint8_t* host_null, const uint16_t* port, const uint8_t* uri_blob,
                   const uint32_t* uri_off, const uint8_t* uri_null, int64_t n,
                   int32_t* out_group) {
    int rc = set_dev(ctx);
    if (rc) return rc;
    if (n <= 0) return n == 0 ? VC_OK : fail(VC_EINVAL, "negative n");
    if (!out_group || (host_blob && !host_off) || (uri_blob && !uri_off))
        return fail(VC_EINVAL, "bad batch arguments");
    StagerLease lease(ctx);
    if (!lease) return hip_fail(lease.err(), "hint search");
    Staging st(ctx, lease.lane(0), "hint search");
    hipStream_t s = st.stream();
    size_t hb = host_blob ? host_off[n] : 0, ub = uri_blob ? uri_off[n] : 0;
    auto* dhb = static_cast<uint8_t*>(host_blob ? st.in(host_blob, hb) : nullptr);
    auto* dho = static_cast<uint32_t*>(host_blob ? st.in(host_off, size_t(n + 1) * 4) : nullptr);
    auto* dhn = static_cast<uint8_t*>(st.in(host_null, size_t(n)));
    auto* dp = static_cast<uint16_t*>(st.in(port, size_t(n) * 2));
    auto* dub = static_cast<uint8_t*>(uri_blob ? st.in(uri_blob, ub) : nullptr);
    auto* duo = static_cast<uint32_t*>(uri_blob ? st.in(uri_off, size_t(n + 1) * 4) : nullptr);
    auto* dun = static_cast<uint8_t*>(st.in(uri_null, size_t(n)));
    auto* dout = static_cast<int32_t*>(st.out(out_group, size_t(n) * 4));
    if (st.err != hipSuccess) return hip_fail(st.err, "staging");
    rc = vc_hint_search_dev(ctx, dhb, dho, dhn, dp, dub, duo, dun, n, dout, s);
    if (rc) return rc;
    st.back(out_group, dout, size_t(n) * 4);
    return st.finish();
}

int vc_compile_hosts(vc_ctx* ctx, const char* const* keys, const int32_t* key_lens,
                     const int32_t* values, int n) {
    int rc = set_dev(ctx);
    if (rc) return rc;
    if (n < 0 || (n && (!keys || !key_lens || !values))) return fail(VC_EINVAL, "bad hosts arrays");
    vc::HostsBuilt b;
    if ((rc = vc::build_hosts(keys, key_lens, values, n, &b)) != VC_OK)
        return fail(rc, "invalid hosts entry");
    std::lock_guard<std::mutex> lk(ctx->compile_mu);
    auto s = std::make_shared<HostsSnap>();
    Upload up(ctx);
    s->img.blob = up(*s, b.blob);
    s->img.recs = up(*s, b.table.recs);
    s->img.tags = up(*s, b.table.tags);
    s->img.mask = static_cast<uint32_t>(b.table.tags.size() - 1);
    s->img.n = b.n;
    if (const hipError_t e = up.done(); e != hipSuccess) return hip_fail(e, "hosts upload");
    ctx->publish(ctx->hosts, std::shared_ptr<const HostsSnap>(std::move(s)));
    return VC_OK;
}

int vc_compile_hosts_text(vc_ctx* ctx, const char* text, int64_t len) {
    if (!text && len) return fail(VC_EINVAL, "null text");
    auto entries = vc::parse_hosts_text(std::string_view(text ? text : "", size_t(len)));
    std::vector<const char*> k;
    std::vector<int32_t> kl, v;
    for (auto& e : entries) {
        k.push_back(e.key.data());
        kl.push_back(static_cast<int32_t>(e.key.size()));
        v.push_back(e.value);
    }
    return vc_compile_hosts(ctx, k.data(), kl.data(), v.data(), static_cast<int>(k.size()));
}

int vc_dns_classify_dev(vc_ctx* ctx, const uint8_t* qblob, const uint32_t* qoff, int64_t n,
                        uint8_t* out_kind, int32_t* out_value, void* stream) {
    int rc = set_dev(ctx);
    if (rc) return rc;
    if (n < 0 || (n > 0 && (!qblob || !qoff || !out_kind || !out_value)))
        return fail(VC_EINVAL, "bad batch arguments");
    auto h = ctx->get(ctx->hint);
    if (!h) return fail(VC_ESTATE, "no Upstream (rrsets) compiled");
    auto ho = ctx->get(ctx->hosts);
    HostsImage hi{};
    if (ho) hi = ho->img;
    hipError_t e = vc::launch_dns(ctx->cfg(stream), hi, h->img, qblob, qoff, n, out_kind, out_value,
                                  ctx->counters_on ? h->counters : nullptr);
    return launched(ctx, e, stream, "dns launch");
}

int vc_dns_classify(vc_ctx* ctx, const uint8_t* qblob, const uint32_t* qoff, int64_t n,
                    uint8_t* out_kind, int32_t* out_value) {
    int rc = set_dev(ctx);
    if (rc) return rc;
    if (n <= 0) return n == 0 ? VC_OK : fail(VC_EINVAL, "negative n");
    if (!qblob || !qoff || !out_kind || !out_value) return fail(VC_EINVAL, "bad batch arguments");
    StagerLease lease(ctx);
    if (!lease) return hip_fail(lease.err(), "dns classify");
    Staging st(ctx, lease.lane(0), "dns classify");
    hipStream_t s = st.stream();
    auto* db = static_cast<uint8_t*>(st.in(qblob, qoff[n]));
    auto* dof = static_cast<uint32_t*>(st.in(qoff, size_t(n + 1) * 4));
    auto* dk = static_cast<uint8_t*>(st.out(out_kind, size_t(n)));
    auto* dv = static_cast<int32_t*>(st.out(out_value, size_t(n) * 4));
    if (st.err != hipSuccess) return hip_fail(st.err, "staging");
    rc = vc_dns_classify_dev(ctx, db, dof, n, dk, dv, s);
    if (rc) return rc;
    st.back(out_kind, dk, size_t(n));
    st.back(out_value, dv, size_t(n) * 4);
    return st.finish();
}

// ---------------------------------------------------------------------------
// HTTP/1 request heads -> HttpContext.connectionHint -> Upstream.searchForGroup
// ---------------------------------------------------------------------------
int vc_http_hint_dev(vc_ctx* ctx, const uint8_t* blob, int64_t blob_bytes, const uint32_t* off,
                     int64_t n, int32_t* out_group, uint8_t* out_kind, void* stream) {
    int rc = set_dev(ctx);
    if (rc) return rc;
    if (n < 0 || blob_bytes < 0 || (n > 0 && (!blob || !off || !out_group)))
        return fail(VC_EINVAL, "bad batch arguments");
    auto h = ctx->get(ctx->hint);
    if (!h) return fail(VC_ESTATE, "no Upstream compiled");
    hipError_t e = vc::launch_http_hint(ctx->cfg(stream), h->img, blob, blob_bytes, off, n,
                                        out_group, out_kind);
    return launched(ctx, e, stream, "http launch");
}

int vc_http_hint(vc_ctx* ctx, const uint8_t* blob, const uint32_t* off, int64_t n,
                 int32_t* out_group, uint8_t* out_kind) {
    int rc = set_dev(ctx);
    if (rc) return rc;
    if (n <= 0) return n == 0 ? VC_OK : fail(VC_EINVAL, "negative n");
    if (!blob || !off || !out_group) return fail(VC_EINVAL, "bad batch arguments");
    StagerLease lease(ctx);
    if (!lease) return hip_fail(lease.err(), "http hint");
    Staging st(ctx, lease.lane(0), "http hint");
    hipStream_t s = st.stream();
    auto* db = static_cast<uint8_t*>(st.in(blob, off[n]));
    auto* dof = static_cast<uint32_t*>(st.in(off, size_t(n + 1) * 4));
    auto* dg = static_cast<int32_t*>(st.out(out_group, size_t(n) * 4));
    auto* dk = out_kind ? static_cast<uint8_t*>(st.out(out_kind, size_t(n))) : nullptr;
    if (st.err != hipSuccess) return hip_fail(st.err, "staging");
    rc = vc_http_hint_dev(ctx, db, int64_t(off[n]), dof, n, dg, dk, s);
    if (rc) return rc;
    st.back(out_group, dg, size_t(n) * 4);
    if (dk) st.back(out_kind, dk, size_t(n));
    return st.finish();
}

// ---------------------------------------------------------------------------
// SSLContextHolder certificate choice by SNI
// ---------------------------------------------------------------------------
int vc_compile_certs(vc_ctx* ctx, const char* const* names, const int32_t* name_lens,
                     const int32_t* holder, int n_names, int n_holders) {
    int rc = set_dev(ctx);
    if (rc) return rc;
    if (n_names < 0 || n_holders < 0 || (n_names && (!names || !name_lens || !holder)))
        return fail(VC_EINVAL, "bad certificate name arrays");
    vc::HostsBuilt b;
    if ((rc = vc::build_certs(names, name_lens, holder, n_names, n_holders, &b)) != VC_OK)
        return fail(rc, "invalid certificate name or holder index");
    std::lock_guard<std::mutex> lk(ctx->compile_mu);
    auto s = std::make_shared<CertSnap>();
    Upload up(ctx);
    s->img.names.blob = up(*s, b.blob);
    s->img.names.recs = up(*s, b.table.recs);
    s->img.names.tags = up(*s, b.table.tags);
    s->img.names.mask = static_cast<uint32_t>(b.table.tags.size() - 1);
    s->img.names.n = b.n;
    s->img.n_holders = n_holders;
    if (const hipError_t e = up.done(); e != hipSuccess) return hip_fail(e, "certificate table upload");
    ctx->publish(ctx->certs, std::shared_ptr<const CertSnap>(std::move(s)));
    return VC_OK;
}

int vc_cert_choose_dev(vc_ctx* ctx, const uint8_t* sni_blob, const uint32_t* sni_off,
                       const uint8_t* sni_null, int64_t n, int32_t* out_holder, void* stream) {
    int rc = set_dev(ctx);
    if (rc) return rc;
    if (n < 0 || (n > 0 && (!sni_blob || !sni_off || !out_holder)))
        return fail(VC_EINVAL, "bad batch arguments");
    auto s = ctx->get(ctx->certs);
    if (!s) return fail(VC_ESTATE, "no certificate holders compiled");
    hipError_t e = vc::launch_certs(ctx->cfg(stream), s->img, sni_blob, sni_off, sni_null, n,
                                    out_holder);
    return launched(ctx, e, stream, "cert launch");
}

int vc_cert_choose(vc_ctx* ctx, const uint8_t* sni_blob, const uint32_t* sni_off,
                   const uint8_t* sni_null, int64_t n, int32_t* out_holder) {
    int rc = set_dev(ctx);
    if (rc) return rc;
    if (n <= 0) return n == 0 ? VC_OK : fail(VC_EINVAL, "negative n");
    if (!sni_blob || !sni_off || !out_holder) return fail(VC_EINVAL, "bad batch arguments");
    StagerLease lease(ctx);
    if (!lease) return hip_fail(lease.err(), "cert choose");
    Staging st(ctx, lease.lane(0), "cert choose");
    hipStream_t s = st.stream();
    auto* db = static_cast<uint8_t*>(st.in(sni_blob, sni_off[n]));
    auto* dof = static_cast<uint32_t*>(st.in(sni_off, size_t(n + 1) * 4));
    auto* dn = static_cast<uint8_t*>(st.in(sni_null, size_t(n)));
    auto* dout = static_cast<int32_t*>(st.out(out_holder, size_t(n) * 4));
    if (st.err != hipSuccess) return hip_fail(st.err, "staging");
    rc = vc_cert_choose_dev(ctx, db, dof, dn, n, dout, s);
    if (rc) return rc;
    st.back(out_holder, dout, size_t(n) * 4);
    return st.finish();
}

int vc_host_register(void* p, int64_t bytes) {
    if (!p || bytes <= 0) return fail(VC_EINVAL, "bad host buffer");
    hipError_t e = hipHostRegister(p, size_t(bytes), hipHostRegisterMapped);
    if (e != hipSuccess) return hip_fail(e, "hipHostRegister");
    std::lock_guard<std::mutex> lk(g_reg_mu);
    g_reg[reinterpret_cast<uintptr_t>(p)] = size_t(bytes);
    return VC_OK;
}

int vc_host_unregister(void* p) {
    if (!p) return fail(VC_EINVAL, "bad host buffer");
    {
        std::lock_guard<std::mutex> lk(g_reg_mu);
        g_reg.erase(reinterpret_cast<uintptr_t>(p));
    }
    hipError_t e = hipHostUnregister(p);
    return e == hipSuccess ? VC_OK : hip_fail(e, "hipHostUnregister");
}

// ---------------------------------------------------------------------------
// Mirror filters
// ---------------------------------------------------------------------------
int vc_compile_mirror(vc_ctx* ctx, const vc_mirror_filter* filters, int n) {
    int rc = set_dev(ctx);
    if (rc) return rc;
    if (n < 0 || (n && !filters)) return fail(VC_EINVAL, "bad filter array");
    std::vector<MirrorRec> recs;
    if ((rc = vc::build_mirror(filters, n, &recs)) != VC_OK)
        return fail(rc, "invalid mirror filter (mirror index, port range or network)");
    std::lock_guard<std::mutex> lk(ctx->compile_mu);
    auto s = std::make_shared<MirrorSnap>();
    Upload up(ctx);
    s->img.f = up(*s, recs);
    s->img.n = n;
    // switchPacket's bit-set image of every origin that has one (compile.hpp
    // build_mirror_switch), its interval tables copied into LDS by the kernel.
    // A/B switches (every form gives the same answers): VC_MIRROR_SW=0 keeps
    // every origin on the per-filter kernel, =1 reads the interval tables
    // from global memory.
    const char* env = std::getenv("VC_MIRROR_SW");
    std::vector<vc::MirrorSwBuilt> built;
    if (!(env && env[0] == '0')) {
        std::set<int32_t> origins;
        for (const MirrorRec& r : recs) origins.insert(r.origin);
        built.reserve(origins.size());
        for (const int32_t o : origins) {
            built.emplace_back();
            vc::MirrorSwBuilt& b = built.back();
            if (!vc::build_mirror_switch(recs, o, &b)) {
                built.pop_back();
                continue;
            }
            b.img.macs = up(*s, b.macs);
            b.img.mirs = up(*s, b.mirs);
            b.img.b4 = up(*s, b.b4);
            b.img.p4 = up(*s, b.p4);
            b.img.b6 = up(*s, b.b6);
            b.img.p6 = up(*s, b.p6);
            b.img.tids = up(*s, b.tids);
            b.img.aids = up(*s, b.aids);
            b.img.bp = up(*s, b.bp);
            b.img.pp = up(*s, b.pp);
            b.img.bm = up(*s, b.bm);
            b.img.pm = up(*s, b.pm);
            b.img.lds = !(env && env[0] == '1');
            s->sw[o] = b.img;
        }
    }
    if (const hipError_t e = up.done(); e != hipSuccess) return hip_fail(e, "mirror filter upload");
    ctx->publish(ctx->mirror, std::shared_ptr<const MirrorSnap>(std::move(s)));
    return VC_OK;
}

static bool al16(const void* p) { return (reinterpret_cast<uintptr_t>(p) & 15) == 0; }

int vc_mirror_match_dev(vc_ctx* ctx, int32_t origin, const vc_mirror_items* items, int64_t n,
                        uint64_t* out_mirrors, void* stream) {
    int rc = set_dev(ctx);
    if (rc) return rc;
    if (n < 0 || (n > 0 && (!items || !out_mirrors))) return fail(VC_EINVAL, "bad batch arguments");
    if (n == 0) return VC_OK;
    if ((items->ip_src && !al16(items->ip_src)) || (items->ip_dst && !al16(items->ip_dst)))
        return fail(VC_EINVAL, "ip_src / ip_dst must be 16-byte aligned");
    if ((reinterpret_cast<uintptr_t>(items->mac_src) | reinterpret_cast<uintptr_t>(items->mac_dst)) & 1)
        return fail(VC_EINVAL, "mac_src / mac_dst must be 2-byte aligned");
    auto s = ctx->get(ctx->mirror);
    if (!s) return fail(VC_ESTATE, "no mirror filters compiled");
    const auto sw = s->sw.find(origin);
    hipError_t e = vc::launch_mirror_match(ctx->cfg(stream), s->img,
                                           sw == s->sw.end() ? nullptr : &sw->second, origin,
                                           *items, n, out_mirrors);
    return launched(ctx, e, stream, "mirror launch");
}

int vc_mirror_match(vc_ctx* ctx, int32_t origin, const vc_mirror_items* items, int64_t n,
                    uint64_t* out_mirrors) {
    int rc = set_dev(ctx);
    if (rc) return rc;
    if (n <= 0) return n == 0 ? VC_OK : fail(VC_EINVAL, "negative n");
    if (!items || !out_mirrors) return fail(VC_EINVAL, "bad batch arguments");
    StagerLease lease(ctx);
    if (!lease) return hip_fail(lease.err(), "mirror match");
    Staging st(ctx, lease.lane(0), "mirror match");
    hipStream_t s = st.stream();
    const size_t un = size_t(n);
    vc_mirror_items d{};
    d.mac_src = static_cast<const uint8_t*>(st.in(items->mac_src, un * 6));
    d.mac_dst = static_cast<const uint8_t*>(st.in(items->mac_dst, un * 6));
    d.ip_src_len = static_cast<const uint8_t*>(st.in(items->ip_src_len, un));
    d.ip_dst_len = static_cast<const uint8_t*>(st.in(items->ip_dst_len, un));
    d.ip_src = static_cast<const uint8_t*>(st.in(items->ip_src, un * 16));
    d.ip_dst = static_cast<const uint8_t*>(st.in(items->ip_dst, un * 16));
    d.transport = static_cast<const int32_t*>(st.in(items->transport, un * 4));
    d.port_src = static_cast<const int32_t*>(st.in(items->port_src, un * 4));
    d.port_dst = static_cast<const int32_t*>(st.in(items->port_dst, un * 4));
    d.app = static_cast<const int32_t*>(st.in(items->app, un * 4));
    auto* dout = static_cast<uint64_t*>(st.out(out_mirrors, un * 8));
    if (st.err != hipSuccess) return hip_fail(st.err, "staging");
    rc = vc_mirror_match_dev(ctx, origin, &d, n, dout, s);
    if (rc) return rc;
    st.back(out_mirrors, dout, un * 8);
    return st.finish();
}

int vc_mirror_switch_dev(vc_ctx* ctx, int32_t origin, const uint8_t* blob, const uint32_t* off,
                         int64_t n, int layer, uint64_t* out_mirrors, void* stream) {
    int rc = set_dev(ctx);
    if (rc) return rc;
    if (n < 0 || (n > 0 && (!blob || !off || !out_mirrors)))
        return fail(VC_EINVAL, "bad batch arguments");
    if (layer != VC_LAYER_VXLAN && layer != VC_LAYER_ETHER)
        return fail(VC_EINVAL, "switchPacket takes VXLAN or Ethernet frames");
    auto s = ctx->get(ctx->mirror);
    if (!s) return fail(VC_ESTATE, "no mirror filters compiled");
    const auto sw = s->sw.find(origin);
    hipError_t e = vc::launch_mirror_switch(ctx->cfg(stream), s->img,
                                            sw == s->sw.end() ? nullptr : &sw->second, origin,
                                            blob, off, n, layer, out_mirrors);
    return launched(ctx, e, stream, "mirror switch launch");
}

int vc_mirror_switch(vc_ctx* ctx, int32_t origin, const uint8_t* blob, const uint32_t* off,
                     int64_t n, int layer, uint64_t* out_mirrors) {
    int rc = set_dev(ctx);
    if (rc) return rc;
    if (n <= 0) return n == 0 ? VC_OK : fail(VC_EINVAL, "negative n");
    if (!blob || !off || !out_mirrors) return fail(VC_EINVAL, "bad batch arguments");
    StagerLease lease(ctx);
    if (!lease) return hip_fail(lease.err(), "mirror switch");
    Staging st(ctx, lease.lane(0), "mirror switch");
    hipStream_t s = st.stream();
    auto* db = static_cast<uint8_t*>(st.in(blob, off[n]));
    auto* dof = static_cast<uint32_t*>(st.in(off, size_t(n + 1) * 4));
    auto* dout = static_cast<uint64_t*>(st.out(out_mirrors, size_t(n) * 8));
    if (st.err != hipSuccess) return hip_fail(st.err, "staging");
    rc = vc_mirror_switch_dev(ctx, origin, db, dof, n, layer, dout, s);
    if (rc) return rc;
    st.back(out_mirrors, dout, size_t(n) * 8);
    return st.finish();
}

// ---------------------------------------------------------------------------
// ServerGroup source hashing
// ---------------------------------------------------------------------------
int vc_compile_servers(vc_ctx* ctx, const vc_server* servers, const int32_t* group_off,
                       int n_groups) {
    int rc = set_dev(ctx);
    if (rc) return rc;
    vc::ServersBuilt b;
    if ((rc = vc::build_servers(servers, group_off, n_groups, &b)) != VC_OK)
        return fail(rc, "invalid server lists");
    std::lock_guard<std::mutex> lk(ctx->compile_mu);
    auto s = std::make_shared<ServerSnap>();
    Upload up(ctx);
    s->img.view_off = up(*s, b.view_off);
    s->img.order = up(*s, b.order);
    s->img.healthy = up(*s, b.healthy);
    s->img.group_base = up(*s, b.group_base);
    s->img.pick = up(*s, b.pick);
    s->img.view_pk = up(*s, b.view_pk);
    s->img.n_groups = b.n_groups;
    s->img.n_servers = b.n_servers;
    s->img.pk_ok = b.pk_ok ? 1 : 0;
    if (const hipError_t e = up.done(); e != hipSuccess) return hip_fail(e, "server upload");
    s->host = std::make_shared<const vc::ServersBuilt>(std::move(b));
    ctx->publish(ctx->servers, std::shared_ptr<const ServerSnap>(std::move(s)));
    return VC_OK;
}

int vc_servers_set_health(vc_ctx* ctx, const uint8_t* healthy, int64_t n_servers) {
    int rc = set_dev(ctx);
    if (rc) return rc;
    std::lock_guard<std::mutex> lk(ctx->compile_mu);
    auto s = ctx->current(ctx->servers);
    if (!s) return fail(VC_ESTATE, "no servers compiled");
    if (n_servers != s->img.n_servers || (n_servers > 0 && !healthy))
        return fail(VC_EINVAL, "health array does not match the compiled servers");
    std::vector<uint8_t> h(healthy, healthy + n_servers);
    for (auto& x : h) x = x ? 1 : 0;
    // copy-on-write: batches in flight keep the snapshot (and health) they pinned
    auto ns = std::make_shared<ServerSnap>();
    ns->img = s->img;
    ns->lists = s->lists ? s->lists : s;
    ns->host = s->host;
    std::vector<int32_t> pick;
    vc::source_pick_table(*s->host, h.data(), &pick);
    Upload up(ctx);
    ns->img.healthy = up(*ns, h);
    ns->img.pick = up(*ns, pick);
    if (const hipError_t e = up.done(); e != hipSuccess) return hip_fail(e, "health upload");
    ctx->publish(ctx->servers, std::shared_ptr<const ServerSnap>(std::move(ns)));
    return VC_OK;
}

static int source_dev(vc_ctx* ctx, int fam, const int32_t* group, const void* src, int64_t n,
                      int view, int32_t* out, void* stream,
                      std::shared_ptr<const ServerSnap> pin = nullptr) {
    int rc = set_dev(ctx);
    if (rc) return rc;
    if (n < 0 || (n > 0 && (!group || !src || !out))) return fail(VC_EINVAL, "bad batch arguments");
    if (view != VC_SOURCE_ALL && view != VC_SOURCE_IPV4 && view != VC_SOURCE_IPV6)
        return fail(VC_EINVAL, "view must be VC_SOURCE_ALL, _IPV4 or _IPV6");
    if (fam == 6 && (reinterpret_cast<uintptr_t>(src) & 15))
        return fail(VC_EINVAL, "IPv6 addresses must be 16-byte aligned");
    auto s = pin ? pin : ctx->get(ctx->servers);
    if (!s) return fail(VC_ESTATE, "no servers compiled");
    hipError_t e = vc::launch_source(ctx->cfg(stream), s->img, group, src, fam, n, view, out);
    return launched(ctx, e, stream, "source launch");
}

static int source_host(vc_ctx* ctx, int fam, const int32_t* group, const void* src, int64_t n,
                       int view, int32_t* out) {
    int rc = set_dev(ctx);
    if (rc) return rc;
    if (n <= 0) return n == 0 ? VC_OK : fail(VC_EINVAL, "negative n");
    if (!group || !src || !out) return fail(VC_EINVAL, "bad batch arguments");
    const size_t sw = fam == 4 ? 4 : 16, un = size_t(n);
    void *mg = mapped(group, un * 4), *ms = mapped(src, un * sw, sw), *mo = mapped(out, un * 4);
    if (mg && ms && mo) {                                        // zero-copy
        rc = source_dev(ctx, fam, static_cast<int32_t*>(mg), ms, n, view,
                        static_cast<int32_t*>(mo), ctx->stream);
        if (rc) return rc;
        hipError_t e = hipStreamSynchronize(ctx->stream);
        if (e != hipSuccess) return hip_fail(e, "source select");
        return ctx->sync_check ? devcheck_report("source select") : VC_OK;
    }
    const auto pin = ctx->get(ctx->servers);
    return host_chunks(ctx, n, "source select", [&](Staging& st, int64_t lo, int64_t c,
                                                    hipStream_t s) {
        const size_t u = size_t(lo), m = size_t(c);
        auto* dg = static_cast<int32_t*>(st.in(group + u, m * 4));
        void* ds = st.in(static_cast<const uint8_t*>(src) + u * sw, m * sw);
        auto* dout = static_cast<int32_t*>(st.out(out, m * 4));
        if (st.err != hipSuccess) return VC_OK;
        int r = source_dev(ctx, fam, dg, ds, c, view, dout, s, pin);
        if (r) return r;
        st.back(out + u, dout, m * 4);
        return VC_OK;
    });
}

int vc_source_select_v4_dev(vc_ctx* ctx, const int32_t* group, const uint32_t* src4, int64_t n,
                            int view, int32_t* out_server, void* stream) {
    return source_dev(ctx, 4, group, src4, n, view, out_server, stream);
}
int vc_source_select_v6_dev(vc_ctx* ctx, const int32_t* group, const uint8_t* src6, int64_t n,
                            int view, int32_t* out_server, void* stream) {
    return source_dev(ctx, 6, group, src6, n, view, out_server, stream);
}
int vc_source_select_v4(vc_ctx* ctx, const int32_t* group, const uint32_t* src4, int64_t n,
                        int view, int32_t* out_server) {
    return source_host(ctx, 4, group, src4, n, view, out_server);
}
int vc_source_select_v6(vc_ctx* ctx, const int32_t* group, const uint8_t* src6, int64_t n,
                        int view, int32_t* out_server) {
    return source_host(ctx, 6, group, src6, n, view, out_server);
}

// ---------------------------------------------------------------------------
// Header extraction
// ---------------------------------------------------------------------------
int vc_parse_packets_dev(vc_ctx* ctx, const uint8_t* blob, const uint32_t* off, int64_t n,
                         int layer, const vc_pkt_out* out, void* stream) {
    int rc = set_dev(ctx);
    if (rc) return rc;
    if (n < 0 || (n > 0 && (!blob || !off || !out))) return fail(VC_EINVAL, "bad batch arguments");
    if (layer != VC_LAYER_VXLAN && layer != VC_LAYER_ETHER && layer != VC_LAYER_IPV4 &&
        layer != VC_LAYER_IPV6)
        return fail(VC_EINVAL, "layer must be VC_LAYER_VXLAN, _ETHER, _IPV4 or _IPV6");
    if (n > 0 && ((reinterpret_cast<uintptr_t>(out->src6) & 15) ||
                  (reinterpret_cast<uintptr_t>(out->dst6) & 15)))
        return fail(VC_EINVAL, "src6/dst6 must be 16-byte aligned");
    hipError_t e = vc::launch_packets(ctx->cfg(stream), blob, off, n, layer, *out);
    return launched(ctx, e, stream, "packet launch");
}

int vc_dns_datagrams_dev(vc_ctx* ctx, const uint8_t* blob, const uint32_t* off, int64_t n,
                         const uint8_t* remote_family, const uint32_t* remote4,
                         const uint8_t* remote6, const uint16_t* remote_port,
                         const vc_dnsd_out* out, void* stream) {
    int rc = set_dev(ctx);
    if (rc) return rc;
    if (n < 0 || (n > 0 && (!blob || !off || !remote4 || !remote_port || !out || !out->status ||
                            !out->kind || !out->value || (remote_family && !remote6))))
        return fail(VC_EINVAL, "bad batch arguments");
    if (reinterpret_cast<uintptr_t>(remote6) & 15)
        return fail(VC_EINVAL, "remote6 must be 16-byte aligned");
    auto a = ctx->get(ctx->acl);
    auto h = ctx->get(ctx->hint);
    if (!a || !h) return fail(VC_ESTATE, "SecurityGroup and Upstream (rrsets) must be compiled");
    auto ho = ctx->get(ctx->hosts);
    HostsImage hi{};
    if (ho) hi = ho->img;
    const vc::LaunchCfg c = ctx->cfg(stream);
    hipError_t e = vc::launch_dns_datagrams(c, hi, h->img, a->img, blob, off, n, remote_family,
                                            remote4, remote6, remote_port, out->status, out->acl,
                                            out->nq, out->qtype, out->kind, out->value);
    if (e == hipSuccess && ctx->counters_on) {
        // hit counters: the UDP rule matched for every datagram (when the
        // caller asks for the rule indices: no aux = the UDP list), and the
        // group of every question classified VC_DNS_GROUP
        const int64_t nr = int64_t(a->img.n_tcp) + a->img.n_udp;
        if (out->acl)
            e = vc::launch_hist(c, VC_HIST_ACL, out->acl, nullptr, n, nr, 0, nr, a->img.n_tcp,
                                a->counters);
        if (e == hipSuccess)
            e = vc::launch_hist(c, VC_HIST_DNS, out->value, out->kind, n * VC_DNSD_MAXQ,
                                h->img.n_groups, 0, h->img.n_groups, 0, h->counters);
    }
    return launched(ctx, e, stream, "dns datagram launch");
}

int vc_dns_datagrams(vc_ctx* ctx, const uint8_t* blob, const uint32_t* off, int64_t n,
                     const uint8_t* remote_family, const uint32_t* remote4,
                     const uint8_t* remote6, const uint16_t* remote_port,
                     const vc_dnsd_out* out) {
    int rc = set_dev(ctx);
    if (rc) return rc;
    if (n <= 0) return n == 0 ? VC_OK : fail(VC_EINVAL, "negative n");
    if (!blob || !off || !remote4 || !remote_port || !out || !out->status || !out->kind ||
        !out->value || (remote_family && !remote6))
        return fail(VC_EINVAL, "bad batch arguments");
    StagerLease lease(ctx);
    if (!lease) return hip_fail(lease.err(), "dns datagrams");
    Staging st(ctx, lease.lane(0), "dns datagrams");
    hipStream_t s = st.stream();
    const size_t un = size_t(n), uq = un * VC_DNSD_MAXQ;
    auto* db = static_cast<uint8_t*>(st.in(blob, off[n]));
    auto* doff = static_cast<uint32_t*>(st.in(off, (un + 1) * 4));
    auto* dfam = static_cast<uint8_t*>(st.in(remote_family, un));
    auto* d4 = static_cast<uint32_t*>(st.in(remote4, un * 4));
    auto* d6 = static_cast<uint8_t*>(st.in(remote6, un * 16));
    auto* dp = static_cast<uint16_t*>(st.in(remote_port, un * 2));
    vc_dnsd_out d{};
    d.status = static_cast<uint8_t*>(st.out(out->status, un));
    d.acl = static_cast<int32_t*>(st.out(out->acl, un * 4));
    d.nq = static_cast<uint8_t*>(st.out(out->nq, un));
    d.qtype = static_cast<uint16_t*>(st.out(out->qtype, uq * 2));
    d.kind = static_cast<uint8_t*>(st.out(out->kind, uq));
    d.value = static_cast<int32_t*>(st.out(out->value, uq * 4));
    if (st.err != hipSuccess) return hip_fail(st.err, "staging");
    rc = vc_dns_datagrams_dev(ctx, db, doff, n, dfam, d4, d6, dp, &d, s);
    if (rc) return rc;
    st.back(out->status, d.status, un);
    st.back(out->acl, d.acl, un * 4);
    st.back(out->nq, d.nq, un);
    st.back(out->qtype, d.qtype, uq * 2);
    st.back(out->kind, d.kind, uq);
    st.back(out->value, d.value, uq * 4);
    return st.finish();
}

// The UDP v4 image of `s` at `port` (the Switch's VXLAN bind port): from
// the snapshot when its compile built it, else built now and kept with the
// snapshot (the first switch call with a new port on each snapshot pays one
// small host build and a synchronous upload).  nb == 0: the general image
// (too many intervals for the kernel's LDS copy, VC_ACL_PORT=0, or a failed
// upload).
static AclPortImage acl_port_image(vc_ctx* ctx, const AclSnap& s, int32_t port) {
    AclPortImage im{nullptr, nullptr, 0, port};
    if (!s.port_images || !s.udp4 || port < 0 || port > 65535) return im;
    std::lock_guard<std::mutex> lk(s.port_mu);
    const auto it = s.ports.find(port);
    if (it != s.ports.end()) return it->second;
    {
        // later compiles build this port's image ahead
        std::lock_guard<std::mutex> seen(ctx->port_seen_mu);
        ctx->acl_ports_seen.insert(port);
    }
    std::vector<uint32_t> pb, pv;
    vc::build_acl_port(*s.udp4, uint32_t(port), &pb, &pv);
    if (pb.size() <= size_t(kAclPortMax)) {
        // through a stager's page-locked bounce buffer, as every upload
        Snapshot own;
        Upload up(ctx);
        const uint32_t* b = up(own, pb);
        const uint32_t* v = up(own, pv);
        if (up.done() == hipSuccess && b && v) {
            im.bounds = b;
            im.value = v;
            im.nb = int32_t(pb.size());
        }
        for (auto& d : own.bufs) s.port_bufs.push_back(std::move(d));
    }
    s.ports[port] = im;
    return im;
}

int vc_switch_classify_dev(vc_ctx* ctx, const uint8_t* blob, const uint32_t* off, int64_t n,
                           int layer, const uint8_t* remote_family, const uint32_t* remote4,
                           const uint8_t* remote6, int bind_port, const vc_pkt_out* out,
                           int32_t* out_acl, uint8_t* out_allow, int32_t* out_route,
                           void* stream) {
    int rc = set_dev(ctx);
    if (rc) return rc;
    if (n < 0 || (n > 0 && (!blob || !off || !out_route || !remote4 ||
                            (remote_family && !remote6))))
        return fail(VC_EINVAL, "bad batch arguments");
    if (layer != VC_LAYER_VXLAN && layer != VC_LAYER_ETHER && layer != VC_LAYER_IPV4 &&
        layer != VC_LAYER_IPV6)
        return fail(VC_EINVAL, "layer must be VC_LAYER_VXLAN, _ETHER, _IPV4 or _IPV6");
    const vc_pkt_out none{};
    const vc_pkt_out& o = out ? *out : none;
    if ((reinterpret_cast<uintptr_t>(o.src6) & 15) || (reinterpret_cast<uintptr_t>(o.dst6) & 15) ||
        (reinterpret_cast<uintptr_t>(remote6) & 15))
        return fail(VC_EINVAL, "src6 / dst6 / remote6 must be 16-byte aligned");
    auto a = ctx->get(ctx->acl);
    auto r = ctx->get(ctx->route);
    auto vt = ctx->get(ctx->vni);
    if (!a || (!r && !vt))
        return fail(VC_ESTATE, "SecurityGroup and RouteTable (or per-VNI tables) must be compiled");
    const AclPortImage ap = acl_port_image(ctx, *a, bind_port);
    hipError_t e = vc::launch_switch(ctx->cfg(stream), a->img, r ? r->img : RouteImage{},
                                     vt ? vt->img : VniImage{}, blob, off, n, layer, o,
                                     remote_family, remote4, remote6, bind_port, ap, out_acl,
                                     out_allow, out_route);
    return launched(ctx, e, stream, "switch launch");
}

// Device copies of the host arrays of a vc_pkt_out (NULL stays NULL).
static vc_pkt_out stage_pkt_out(Staging& st, const vc_pkt_out& out, size_t un) {
    vc_pkt_out d{};
    d.status = static_cast<uint8_t*>(st.out(out.status, un));
    d.l3 = static_cast<uint8_t*>(st.out(out.l3, un));
    d.l4 = static_cast<uint8_t*>(st.out(out.l4, un));
    d.proto = static_cast<uint8_t*>(st.out(out.proto, un));
    d.vni = static_cast<uint32_t*>(st.out(out.vni, un * 4));
    d.ether_type = static_cast<uint16_t*>(st.out(out.ether_type, un * 2));
    d.src4 = static_cast<uint32_t*>(st.out(out.src4, un * 4));
    d.dst4 = static_cast<uint32_t*>(st.out(out.dst4, un * 4));
    d.src6 = static_cast<uint8_t*>(st.out(out.src6, un * 16));
    d.dst6 = static_cast<uint8_t*>(st.out(out.dst6, un * 16));
    d.sport = static_cast<uint16_t*>(st.out(out.sport, un * 2));
    d.dport = static_cast<uint16_t*>(st.out(out.dport, un * 2));
    return d;
}

static void back_pkt_out(Staging& st, const vc_pkt_out& out, const vc_pkt_out& d, size_t un) {
    st.back(out.status, d.status, un);
    st.back(out.l3, d.l3, un);
    st.back(out.l4, d.l4, un);
    st.back(out.proto, d.proto, un);
    st.back(out.vni, d.vni, un * 4);
    st.back(out.ether_type, d.ether_type, un * 2);
    st.back(out.src4, d.src4, un * 4);
    st.back(out.dst4, d.dst4, un * 4);
    st.back(out.src6, d.src6, un * 16);
    st.back(out.dst6, d.dst6, un * 16);
    st.back(out.sport, d.sport, un * 2);
    st.back(out.dport, d.dport, un * 2);
}

int vc_switch_classify(vc_ctx* ctx, const uint8_t* blob, const uint32_t* off, int64_t n, int layer,
                       const uint8_t* remote_family, const uint32_t* remote4,
                       const uint8_t* remote6, int bind_port, const vc_pkt_out* out,
                       int32_t* out_acl, uint8_t* out_allow, int32_t* out_route) {
    int rc = set_dev(ctx);
    if (rc) return rc;
    if (n <= 0) return n == 0 ? VC_OK : fail(VC_EINVAL, "negative n");
    if (!blob || !off || !out_route || !remote4 || (remote_family && !remote6))
        return fail(VC_EINVAL, "bad batch arguments");
    StagerLease lease(ctx);
    if (!lease) return hip_fail(lease.err(), "switch classify");
    Staging st(ctx, lease.lane(0), "switch classify");
    hipStream_t s = st.stream();
    const size_t un = size_t(n);
    const vc_pkt_out none{};
    const vc_pkt_out& o = out ? *out : none;
    auto* db = static_cast<uint8_t*>(st.in(blob, off[n]));
    auto* doff = static_cast<uint32_t*>(st.in(off, (un + 1) * 4));
    auto* dfam = static_cast<uint8_t*>(st.in(remote_family, un));
    auto* d4 = static_cast<uint32_t*>(st.in(remote4, un * 4));
    auto* d6 = static_cast<uint8_t*>(st.in(remote6, un * 16));
    const vc_pkt_out d = stage_pkt_out(st, o, un);
    auto* dacl = static_cast<int32_t*>(st.out(out_acl, un * 4));
    auto* dal = static_cast<uint8_t*>(st.out(out_allow, un));
    auto* dr = static_cast<int32_t*>(st.out(out_route, un * 4));
    if (st.err != hipSuccess) return hip_fail(st.err, "staging");
    rc = vc_switch_classify_dev(ctx, db, doff, n, layer, dfam, d4, d6, bind_port, &d, dacl, dal, dr,
                                s);
    if (rc) return rc;
    back_pkt_out(st, o, d, un);
    st.back(out_acl, dacl, un * 4);
    st.back(out_allow, dal, un);
    st.back(out_route, dr, un * 4);
    return st.finish();
}

int vc_parse_packets(vc_ctx* ctx, const uint8_t* blob, const uint32_t* off, int64_t n, int layer,
                     const vc_pkt_out* out) {
    int rc = set_dev(ctx);
    if (rc) return rc;
    if (n <= 0) return n == 0 ? VC_OK : fail(VC_EINVAL, "negative n");
    if (!blob || !off || !out) return fail(VC_EINVAL, "bad batch arguments");
    StagerLease lease(ctx);
    if (!lease) return hip_fail(lease.err(), "parse packets");
    Staging st(ctx, lease.lane(0), "parse packets");
    hipStream_t s = st.stream();
    auto* db = static_cast<uint8_t*>(st.in(blob, off[n]));
    auto* doff = static_cast<uint32_t*>(st.in(off, size_t(n + 1) * 4));
    vc_pkt_out d{};
    const size_t un = size_t(n);
    d.status = static_cast<uint8_t*>(st.out(out->status, un));
    d.l3 = static_cast<uint8_t*>(st.out(out->l3, un));
    d.l4 = static_cast<uint8_t*>(st.out(out->l4, un));
    d.proto = static_cast<uint8_t*>(st.out(out->proto, un));
    d.vni = static_cast<uint32_t*>(st.out(out->vni, un * 4));
    d.ether_type = static_cast<uint16_t*>(st.out(out->ether_type, un * 2));
    d.src4 = static_cast<uint32_t*>(st.out(out->src4, un * 4));
    d.dst4 = static_cast<uint32_t*>(st.out(out->dst4, un * 4));
    d.src6 = static_cast<uint8_t*>(st.out(out->src6, un * 16));
    d.dst6 = static_cast<uint8_t*>(st.out(out->dst6, un * 16));
    d.sport = static_cast<uint16_t*>(st.out(out->sport, un * 2));
    d.dport = static_cast<uint16_t*>(st.out(out->dport, un * 2));
    if (st.err != hipSuccess) return hip_fail(st.err, "staging");
    rc = vc_parse_packets_dev(ctx, db, doff, n, layer, &d, s);
    if (rc) return rc;
    st.back(out->status, d.status, un);
    st.back(out->l3, d.l3, un);
    st.back(out->l4, d.l4, un);
    st.back(out->proto, d.proto, un);
    st.back(out->vni, d.vni, un * 4);
    st.back(out->ether_type, d.ether_type, un * 2);
    st.back(out->src4, d.src4, un * 4);
    st.back(out->dst4, d.dst4, un * 4);
    st.back(out->src6, d.src6, un * 16);
    st.back(out->dst6, d.dst6, un * 16);
    st.back(out->sport, d.sport, un * 2);
    st.back(out->dport, d.dport, un * 2);
    return st.finish();
}

// ---------------------------------------------------------------------------
// Pipeline
// ---------------------------------------------------------------------------
int vc_pipeline_v4_dev(vc_ctx* ctx, const uint8_t* proto, const uint32_t* src4,
                       const uint32_t* dst4, const uint16_t* dport, const uint32_t* host_id,
                       const int32_t* pool_group, int64_t n_pool, int64_t n, int32_t* out_acl,
                       int32_t* out_route,
                       int32_t* out_group, uint8_t* out_allow, void* stream) {
    return vc_pipeline_v4_dev_ex(ctx, proto, src4, dst4, dport, host_id, pool_group, n_pool, n,
                                 out_acl, out_route, out_group, out_allow, stream, nullptr);
}

int vc_pipeline_v4_dev_ex(vc_ctx* ctx, const uint8_t* proto, const uint32_t* src4,
                          const uint32_t* dst4, const uint16_t* dport, const uint32_t* host_id,
                          const int32_t* pool_group, int64_t n_pool, int64_t n, int32_t* out_acl,
                          int32_t* out_route, int32_t* out_group, uint8_t* out_allow, void* stream,
                          void* kernel_done_event) {
    if (n > 0 && !host_id) return fail(VC_EINVAL, "bad batch arguments");
    const vc_packets in{nullptr, proto, src4, dst4, nullptr, nullptr, dport, host_id};
    const vc_pipeline_out out{out_acl, out_route, out_group, out_allow};
    return vc_pipeline_dev(ctx, &in, n, pool_group, n_pool, &out, stream, nullptr,
                           kernel_done_event);
}

namespace {
struct PipePins {                  // the snapshots one pipeline call classifies against
    std::shared_ptr<const AclSnap> a;
    std::shared_ptr<const RouteSnap> r;
    std::shared_ptr<const HintSnap> h;
};
}  // namespace

static int pipeline_check(const vc_packets* in, int64_t n, const int32_t* pool_group,
                          int64_t n_pool, const vc_pipeline_out* out) {
    if (n < 0 || n_pool < 0 || !in || !out) return fail(VC_EINVAL, "bad batch arguments");
    if (n == 0) return VC_OK;
    if (!in->proto || !in->src4 || !in->dst4 || !in->dport || !out->acl || !out->route ||
        !out->group || (in->host_id && n_pool > 0 && !pool_group))
        return fail(VC_EINVAL, "bad batch arguments");
    if (in->family && (!in->src6 || !in->dst6))
        return fail(VC_EINVAL, "a batch with a family array needs src6 and dst6");
    return VC_OK;
}

static int pipeline_dev(vc_ctx* ctx, const vc_packets& in, int64_t n, const int32_t* pool_group,
                        int64_t n_pool, const vc_pipeline_out& out, void* stream,
                        void* count_stream, void* kernel_done, const PipePins& pin,
                        int64_t n6c = -1) {
    if ((in.src6 && (reinterpret_cast<uintptr_t>(in.src6) & 15)) ||
        (in.dst6 && (reinterpret_cast<uintptr_t>(in.dst6) & 15)))
        return fail(VC_EINVAL, "src6 / dst6 must be 16-byte aligned");
    if (!pin.a || !pin.r) return fail(VC_ESTATE, "SecurityGroup and RouteTable must be compiled");
    const bool on = ctx->counters_on;
    vc::PipeArgs p{in.family, in.proto, in.src4, in.dst4, in.src6, in.dst6, in.dport, in.host_id,
                   pool_group, in.host_id ? n_pool : 0, n, out.acl, out.route, out.group,
                   out.allow, n6c};
    vc::PipeCounters cnt{on ? pin.a->counters : nullptr, on ? pin.r->counters : nullptr,
                         on && pin.h && in.host_id ? pin.h->counters : nullptr,
                         pin.h ? pin.h->img.n_groups : 0};
    hipError_t e = vc::launch_pipeline(ctx->cfg(stream), pin.a->img, pin.r->img, pin.r->n4,
                                       pin.r->n6, p, cnt, static_cast<hipEvent_t>(kernel_done),
                                       static_cast<hipStream_t>(count_stream));
    return launched(ctx, e, stream, "pipeline launch");
}

int vc_pipeline_dev(vc_ctx* ctx, const vc_packets* in, int64_t n, const int32_t* pool_group,
                    int64_t n_pool, const vc_pipeline_out* out, void* stream, void* count_stream,
                    void* kernel_done_event) {
    int rc = set_dev(ctx);
    if (rc) return rc;
    if ((rc = pipeline_check(in, n, pool_group, n_pool, out)) != VC_OK) return rc;
    const PipePins pin{ctx->get(ctx->acl), ctx->get(ctx->route), ctx->get(ctx->hint)};
    return pipeline_dev(ctx, *in, n, pool_group, n_pool, *out, stream, count_stream,
                        kernel_done_event, pin);
}

// the alignment the compact-row kernel's vector loads need
static bool c6_aligned(const vc_packets& in, const vc_pipeline_out& out) {
    auto al = [](const void* p, uintptr_t a) { return !p || (reinterpret_cast<uintptr_t>(p) & (a - 1)) == 0; };
    return al(in.family, 4) && al(in.proto, 4) && al(in.src4, 16) && al(in.dst4, 16) &&
           al(in.dport, 8) && al(in.host_id, 16) && al(out.acl, 16) && al(out.route, 16) &&
           al(out.group, 16) && al(out.allow, 4);
}

int vc_pipeline_c6_dev(vc_ctx* ctx, const vc_packets* in, int64_t n, int64_t n6,
                       const int32_t* pool_group, int64_t n_pool, const vc_pipeline_out* out,
                       void* stream, void* count_stream, void* kernel_done_event) {
    int rc = set_dev(ctx);
    if (rc) return rc;
    // no IPv6 rows: the kernel reads none (pipe_mix_c6), so any aligned
    // non-null pointer stands in for the empty arrays
    alignas(16) static const uint8_t kNoRows[16] = {};
    vc_packets m = in ? *in : vc_packets{};
    if (in && n6 == 0) m.src6 = m.dst6 = kNoRows;
    in = in ? &m : nullptr;
    if ((rc = pipeline_check(in, n, pool_group, n_pool, out)) != VC_OK) return rc;
    if (n == 0) return kernel_done_event ? (hipEventRecord(static_cast<hipEvent_t>(kernel_done_event),
                                                           static_cast<hipStream_t>(stream)) == hipSuccess
                                                ? VC_OK : fail(VC_EDEVICE, "event record"))
                                         : VC_OK;
    if (!in->family || n6 < 0 || (n6 > 0 && (!in->src6 || !in->dst6)))
        return fail(VC_EINVAL, "compact IPv6 rows need the family array and n6 >= 0 rows");
    if (!c6_aligned(*in, *out))
        return fail(VC_EINVAL, "vc_pipeline_c6_dev needs 16-byte aligned 4-byte fields (4-byte "
                               "aligned family / proto / allow, 8-byte aligned dport)");
    const PipePins pin{ctx->get(ctx->acl), ctx->get(ctx->route), ctx->get(ctx->hint)};
    return pipeline_dev(ctx, *in, n, pool_group, n_pool, *out, stream, count_stream,
                        kernel_done_event, pin, n6);
}

// The host entry points: vc_pipeline (n6 < 0: src6 / dst6 hold n rows) and
// vc_pipeline_c6 (n6 >= 0: one row per IPv6 packet, packet order).
static int pipeline_host(vc_ctx* ctx, const vc_packets* in, int64_t n, int64_t n6,
                         const int32_t* pool_group, int64_t n_pool, const vc_pipeline_out* out) {
    const PipePins pin{ctx->get(ctx->acl), ctx->get(ctx->route), ctx->get(ctx->hint)};
    if (!pin.a || !pin.r) return fail(VC_ESTATE, "SecurityGroup and RouteTable must be compiled");
    const size_t un = size_t(n);
    const bool six = in->family != nullptr;
    const size_t pool_bytes = in->host_id ? size_t(n_pool) * 4 : 0;
    // zero-copy when every array lies inside a registered buffer
    vc_packets m{};
    vc_pipeline_out mo{};
    bool zc = true;
    auto map = [&](const void* h, size_t bytes, uintptr_t al) -> void* {
        if (!h || !bytes) return nullptr;
        void* d = mapped(h, bytes, al);
        if (!d) zc = false;
        return d;
    };
    m.family = static_cast<const uint8_t*>(map(in->family, un, 1));
    m.proto = static_cast<const uint8_t*>(map(in->proto, un, 1));
    m.src4 = static_cast<const uint32_t*>(map(in->src4, un * 4, 4));
    m.dst4 = static_cast<const uint32_t*>(map(in->dst4, un * 4, 4));
    const bool c6 = n6 >= 0;
    const size_t rows = c6 ? size_t(n6) : un;
    m.src6 = static_cast<const uint8_t*>(map(six ? in->src6 : nullptr, rows * 16, 16));
    m.dst6 = static_cast<const uint8_t*>(map(six ? in->dst6 : nullptr, rows * 16, 16));
    if (c6 && !rows) m.src6 = m.dst6 = in->src6;                // never read
    m.dport = static_cast<const uint16_t*>(map(in->dport, un * 2, 2));
    m.host_id = static_cast<const uint32_t*>(map(in->host_id, un * 4, 4));
    mo.acl = static_cast<int32_t*>(map(out->acl, un * 4, 4));
    mo.route = static_cast<int32_t*>(map(out->route, un * 4, 4));
    mo.group = static_cast<int32_t*>(map(out->group, un * 4, 4));
    mo.allow = static_cast<uint8_t*>(map(out->allow, un, 1));
    // The hostname pool results are uploaded once, on the stager's whole-call
    // lane, and stay there for the call: pool_group[host_id] is a random
    // 4-byte gather per packet, which across PCIe (a registered pool read
    // zero-copy) held a compact-row batch to 8.8 GB/s.
    StagerLease lease(ctx);
    if (!lease) return hip_fail(lease.err(), "pipeline");
    Staging pst(ctx, lease.lane(2), "pool upload");
    const int32_t* dpool = pool_bytes
        ? static_cast<const int32_t*>(pst.in(pool_group, pool_bytes)) : nullptr;
    if (pst.err == hipSuccess) pst.err = lease.lane(2).wait();
    if (pst.err != hipSuccess) return hip_fail(pst.err, "pool upload");
    // Zero-copy for IPv4-only batches and for compact IPv6 rows: their reads
    // are coalesced.  A mixed batch with n rows reads 16-byte IPv6 addresses
    // for a scattered 15 % of its packets, which across PCIe ran at 7 GB/s;
    // staging it with DMA copies (registered memory copies at full rate) is
    // faster.  The compact kernel's vector loads need the alignment
    // vc_pipeline_c6_dev asks for; a batch without it is staged.
    if (zc && c6) zc = c6_aligned(m, mo);
    if (zc && (!six || c6)) {
        int rc = pipeline_dev(ctx, m, n, dpool, n_pool, mo, ctx->stream, nullptr, nullptr, pin,
                              n6);
        if (rc) return rc;
        hipError_t e = hipStreamSynchronize(ctx->stream);
        if (e != hipSuccess) return hip_fail(e, "pipeline");
        return ctx->sync_check ? devcheck_report("pipeline") : VC_OK;
    }
    // chunked staging
    int64_t row = 0;                                // compact rows: the chunk's first row
    const int rc = host_chunks(ctx, lease, n, "pipeline", [&](Staging& st, int64_t lo, int64_t c,
                                                              hipStream_t s) {
        const size_t u = size_t(lo), k = size_t(c);
        vc_packets d{};
        vc_pipeline_out o{};
        // compact rows: the chunk's IPv6 packets are the next k6 rows (the
        // count overlaps the previous chunk's copies and kernel)
        int64_t k6 = 0;
        if (c6) {
            for (size_t i = 0; i < k; ++i) k6 += in->family[u + i] == 6;
            if (row + k6 > n6) return fail(VC_EINVAL, "the family array has more IPv6 packets "
                                                      "than n6 rows");
        }
        const size_t r0 = c6 ? size_t(row) : u, rk = c6 ? size_t(k6) : k;
        d.family = six ? static_cast<const uint8_t*>(st.in(in->family + u, k)) : nullptr;
        d.proto = static_cast<const uint8_t*>(st.in(in->proto + u, k));
        d.src4 = static_cast<const uint32_t*>(st.in(in->src4 + u, k * 4));
        d.dst4 = static_cast<const uint32_t*>(st.in(in->dst4 + u, k * 4));
        d.src6 = six && rk ? static_cast<const uint8_t*>(st.in(in->src6 + r0 * 16, rk * 16))
                           : nullptr;
        d.dst6 = six && rk ? static_cast<const uint8_t*>(st.in(in->dst6 + r0 * 16, rk * 16))
                           : nullptr;
        if (six && !rk) d.src6 = d.dst6 = d.family;             // no rows: never read
        row += k6;
        d.dport = static_cast<const uint16_t*>(st.in(in->dport + u, k * 2));
        d.host_id = in->host_id ? static_cast<const uint32_t*>(st.in(in->host_id + u, k * 4))
                                : nullptr;
        o.acl = static_cast<int32_t*>(st.out(out->acl, k * 4));
        o.route = static_cast<int32_t*>(st.out(out->route, k * 4));
        o.group = static_cast<int32_t*>(st.out(out->group, k * 4));
        o.allow = static_cast<uint8_t*>(st.out(out->allow, k));
        if (st.err != hipSuccess) return VC_OK;               // reported by host_chunks
        int r = pipeline_dev(ctx, d, c, dpool, n_pool, o, s, nullptr, nullptr, pin,
                             c6 ? k6 : -1);
        if (r) return r;
        st.back(out->acl + u, o.acl, k * 4);
        st.back(out->route + u, o.route, k * 4);
        st.back(out->group + u, o.group, k * 4);
        if (out->allow) st.back(out->allow + u, o.allow, k);
        return VC_OK;
    });
    if (rc == VC_OK && c6 && row != n6)
        return fail(VC_EINVAL, "the family array has fewer IPv6 packets than n6 rows");
    return rc;
}

int vc_pipeline(vc_ctx* ctx, const vc_packets* in, int64_t n, const int32_t* pool_group,
                int64_t n_pool, const vc_pipeline_out* out) {
    int rc = set_dev(ctx);
    if (rc) return rc;
    if ((rc = pipeline_check(in, n, pool_group, n_pool, out)) != VC_OK) return rc;
    if (n == 0) return VC_OK;
    return pipeline_host(ctx, in, n, -1, pool_group, n_pool, out);
}

int vc_pipeline_c6(vc_ctx* ctx, const vc_packets* in, int64_t n, int64_t n6,
                   const int32_t* pool_group, int64_t n_pool, const vc_pipeline_out* out) {
    int rc = set_dev(ctx);
    if (rc) return rc;
    alignas(16) static const uint8_t kNoRows[16] = {};
    vc_packets m = in ? *in : vc_packets{};
    if (in && n6 == 0) m.src6 = m.dst6 = kNoRows;
    in = in ? &m : nullptr;
    if ((rc = pipeline_check(in, n, pool_group, n_pool, out)) != VC_OK) return rc;
    if (n == 0) return VC_OK;
    if (!in->family || n6 < 0 || n6 > n)
        return fail(VC_EINVAL, "compact IPv6 rows need the family array and 0 <= n6 <= n rows");
    // One rule for both host paths (zero-copy and staged), checked before any
    // output is written: n6 is the number of IPv6 packets.  A vectorised
    // byte count over the host family array, small beside the batch's PCIe
    // traffic.
    int64_t six = 0;
    const uint8_t* fam = in->family;
    for (int64_t i = 0; i < n; ++i) six += fam[i] == 6;
    if (six != n6)
        return fail(VC_EINVAL, "the family array has " + std::to_string(six) +
                                   " IPv6 packets but n6 = " + std::to_string(n6) + " rows");
    return pipeline_host(ctx, in, n, n6, pool_group, n_pool, out);
}

// ---------------------------------------------------------------------------
// Counters
// ---------------------------------------------------------------------------
int vc_counters_enable(vc_ctx* ctx, int on) {
    if (!ctx) return fail(VC_EINVAL, "null context");
    ctx->counters_on = on != 0;
    return VC_OK;
}

static const Snapshot* counter_snap(vc_ctx* ctx, int kind, std::shared_ptr<const void>* keep) {
    switch (kind) {
    case VC_COUNTERS_ACL: { auto s = ctx->get(ctx->acl); *keep = s; return s.get(); }
    case VC_COUNTERS_ROUTE: { auto s = ctx->get(ctx->route); *keep = s; return s.get(); }
    case VC_COUNTERS_GROUP: { auto s = ctx->get(ctx->hint); *keep = s; return s.get(); }
    default: return nullptr;
    }
}

int vc_counters_device(vc_ctx* ctx, int kind, uint64_t** dev_ptr, int64_t* n) {
    int rc = set_dev(ctx);
    if (rc) return rc;
    std::shared_ptr<const void> keep;
    const Snapshot* s = counter_snap(ctx, kind, &keep);
    if (!s) return fail(VC_ESTATE, "no table compiled for this counter kind");
    if (dev_ptr) *dev_ptr = reinterpret_cast<uint64_t*>(s->counters);
    if (n) *n = s->n_counters;
    return VC_OK;
}

int vc_counters_read(vc_ctx* ctx, int kind, uint64_t* host, int64_t n) {
    int rc = set_dev(ctx);
    if (rc) return rc;
    std::shared_ptr<const void> keep;
    const Snapshot* s = counter_snap(ctx, kind, &keep);
    if (!s) return fail(VC_ESTATE, "no table compiled for this counter kind");
    if (!host || n < s->n_counters) return fail(VC_EINVAL, "host buffer too small");
    hipError_t e = hipStreamSynchronize(ctx->stream);
    if (e == hipSuccess) e = hipDeviceSynchronize();
    if (e == hipSuccess)
        e = hipMemcpy(host, s->counters, size_t(s->n_counters) * 8, hipMemcpyDeviceToHost);
    // the device is idle here, so freeing retired snapshot buffers costs no
    // wait: a deployment that rarely recompiles but reads its counters
    // (Prometheus scrapes) does not keep superseded tables alive
    if (e == hipSuccess) ctx->grave->drain();
    return e == hipSuccess ? VC_OK : hip_fail(e, "counter read");
}

int vc_table_digest(vc_ctx* ctx, int kind, uint64_t* digest) {
    int rc = set_dev(ctx);
    if (rc) return rc;
    if (!digest) return fail(VC_EINVAL, "null digest");
    std::shared_ptr<const void> keep;
    const Snapshot* s = counter_snap(ctx, kind, &keep);
    if (!s) return fail(VC_ESTATE, "no table compiled for this kind");
    *digest = s->digest;
    return VC_OK;
}

// Host-only digests: the same builds as the compile calls, no device.
int vc_digest_acl(const vc_acl_rule* tcp, int n_tcp, const vc_acl_rule* udp, int n_udp,
                  int default_allow, uint64_t* digest) {
    if ((n_tcp && !tcp) || (n_udp && !udp) || !digest) return fail(VC_EINVAL, "null argument");
    vc::AclBuilt b;
    if (int rc = vc::build_acl(tcp, n_tcp, udp, n_udp, default_allow, &b)) return fail(rc, "invalid rule");
    *digest = vc::digest(b);
    return VC_OK;
}

int vc_digest_routes(const vc_net* v4, int n4, const vc_net* v6, int n6, uint64_t* digest) {
    if ((n4 && !v4) || (n6 && !v6) || n4 < 0 || n6 < 0 || !digest)
        return fail(VC_EINVAL, "bad rule arrays");
    vc::TrieBuilt t4, t6;
    int rc;
    if ((rc = vc::build_trie(v4, n4, 0, &t4)) != VC_OK) return fail(rc, "invalid IPv4 route rule");
    if ((rc = vc::build_trie(v6, n6, 1, &t6)) != VC_OK) return fail(rc, "invalid IPv6 route rule");
    *digest = vc::digest(t4, t6);
    return VC_OK;
}

int vc_digest_upstream(const vc_group_annos* groups, int n, uint64_t* digest) {
    if (n < 0 || (n && !groups) || !digest) return fail(VC_EINVAL, "bad group array");
    vc::HintBuilt b;
    if (int rc = vc::build_hints(groups, n, &b)) return fail(rc, "invalid annotations");
    *digest = vc::digest(b);
    return VC_OK;
}

int vc_counters_reset(vc_ctx* ctx) {
    int rc = set_dev(ctx);
    if (rc) return rc;
    for (int k = 0; k < 3; ++k) {
        std::shared_ptr<const void> keep;
        const Snapshot* s = counter_snap(ctx, k, &keep);
        if (!s) continue;
        hipError_t e = hipMemsetAsync(s->counters, 0, size_t(std::max<int64_t>(s->n_counters, 1)) * 8,
                                      ctx->stream);
        if (e != hipSuccess) return hip_fail(e, "counter reset");
    }
    hipError_t e = hipStreamSynchronize(ctx->stream);
    return e == hipSuccess ? VC_OK : hip_fail(e, "counter reset");
}

int vc_counters_add_dev(vc_ctx* ctx, int kind, const int32_t* out, const uint8_t* aux, int family,
                        int64_t n, void* stream) {
    int rc = set_dev(ctx);
    if (rc) return rc;
    if (n < 0 || (n > 0 && !out)) return fail(VC_EINVAL, "bad batch arguments");
    if (n == 0) return VC_OK;
    hipError_t e = hipSuccess;
    vc::LaunchCfg c = ctx->cfg(stream);
    if (kind == VC_COUNTERS_ACL) {
        auto s = ctx->get(ctx->acl);
        if (!s) return fail(VC_ESTATE, "no SecurityGroup compiled");
        if (!aux) return fail(VC_EINVAL, "ACL counters need the proto array");
        const int64_t nr = int64_t(s->img.n_tcp) + s->img.n_udp;
        e = vc::launch_hist(c, VC_HIST_ACL, out, aux, n, nr, 0, nr, s->img.n_tcp, s->counters);
    } else if (kind == VC_COUNTERS_ROUTE) {
        auto s = ctx->get(ctx->route);
        if (!s) return fail(VC_ESTATE, "no RouteTable compiled");
        if (family != 4 && family != 6) return fail(VC_EINVAL, "family must be 4 or 6");
        const int64_t nn = int64_t(s->n4) + s->n6;
        e = family == 4 ? vc::launch_hist(c, VC_HIST_PLAIN, out, nullptr, n, s->n4, 0, nn, 0,
                                          s->counters)
                        : vc::launch_hist(c, VC_HIST_PLAIN, out, nullptr, n, s->n6, s->n4, nn + 1,
                                          0, s->counters);
    } else if (kind == VC_COUNTERS_GROUP) {
        auto s = ctx->get(ctx->hint);
        if (!s) return fail(VC_ESTATE, "no Upstream compiled");
        const int32_t ng = s->img.n_groups;
        e = vc::launch_hist(c, aux ? VC_HIST_DNS : VC_HIST_PLAIN, out, aux, n, ng, 0, ng, 0,
                            s->counters);
    } else {
        return fail(VC_EINVAL, "unknown counter kind");
    }
    return launched(ctx, e, stream, "counter pass");
}

// ---------------------------------------------------------------------------
// Prometheus text (host/prometheus.cpp)
// ---------------------------------------------------------------------------
static int text_out(const std::string& text, char* buf, int64_t cap, int64_t* len) {
    int rc = vc::copy_text(text, buf, cap, len);
    return rc == VC_OK ? rc : fail(rc, "buffer too small for the exposition text");
}

int vc_prometheus_format(const vc_metric* metrics, int32_t n, const char* const* help_metric,
                         const char* const* help_text, int32_t n_help, char* buf, int64_t cap,
                         int64_t* len) {
    if (n < 0 || n_help < 0 || (n && !metrics) || (n_help && (!help_metric || !help_text)))
        return fail(VC_EINVAL, "bad metric arrays");
    std::vector<vc::PromMetric> ms;
    ms.reserve(size_t(n));
    for (int32_t i = 0; i < n; ++i) {
        const vc_metric& m = metrics[i];
        if (!m.metric || m.n_labels < 0 || (m.n_labels && (!m.label_keys || !m.label_values)))
            return fail(VC_EINVAL, "bad metric " + std::to_string(i));
        if (m.type != VC_METRIC_COUNTER && m.type != VC_METRIC_GAUGE)
            return fail(VC_EINVAL, "unknown metric type");
        vc::PromMetric p{m.metric, m.type == VC_METRIC_COUNTER ? "counter" : "gauge", {}, m.value};
        for (int32_t k = 0; k < m.n_labels; ++k) {
            if (!m.label_keys[k] || !m.label_values[k]) return fail(VC_EINVAL, "null label");
            p.labels[m.label_keys[k]] = m.label_values[k];
        }
        ms.push_back(std::move(p));
    }
    std::map<std::string, std::string> help;
    for (int32_t i = 0; i < n_help; ++i) {
        if (!help_metric[i] || !help_text[i]) return fail(VC_EINVAL, "null help message");
        help[help_metric[i]] = help_text[i];
    }
    return text_out(vc::prometheus_text(ms, help), buf, cap, len);
}

int vc_prometheus_hits(const uint64_t* acl, int n_tcp, int n_udp, const uint64_t* route, int n4,
                       int n6, const uint64_t* group, int n_groups, const char* extra_labels,
                       char* buf, int64_t cap, int64_t* len) {
    if (n_tcp < 0 || n_udp < 0 || n4 < 0 || n6 < 0 || n_groups < 0)
        return fail(VC_EINVAL, "negative counter size");
    std::map<std::string, std::string> extra;
    if (vc::parse_extra_labels(extra_labels, &extra) != VC_OK)
        return fail(VC_EINVAL, "invalid format, expecting k=v");
    std::vector<vc::PromMetric> ms;
    std::map<std::string, std::string> help;
    vc::hit_metrics(acl, n_tcp, n_udp, route, n4, n6, group, n_groups, extra, &ms, &help);
    return text_out(vc::prometheus_text(ms, help), buf, cap, len);
}

int vc_counters_prometheus(vc_ctx* ctx, const char* extra_labels, char* buf, int64_t cap,
                           int64_t* len) {
    int rc = set_dev(ctx);
    if (rc) return rc;
    auto a = ctx->get(ctx->acl);
    auto r = ctx->get(ctx->route);
    auto h = ctx->get(ctx->hint);
    std::vector<uint64_t> ha, hr, hg;
    hipError_t e = hipStreamSynchronize(ctx->stream);
    if (e == hipSuccess) e = hipDeviceSynchronize();
    auto fetch = [&](const Snapshot* s, std::vector<uint64_t>* v) {
        if (!s || e != hipSuccess) return;
        v->resize(size_t(std::max<int64_t>(s->n_counters, 1)));
        e = hipMemcpy(v->data(), s->counters, size_t(s->n_counters) * 8, hipMemcpyDeviceToHost);
    };
    fetch(a.get(), &ha);
    fetch(r.get(), &hr);
    fetch(h.get(), &hg);
    if (e != hipSuccess) return hip_fail(e, "counter read");
    return vc_prometheus_hits(a ? ha.data() : nullptr, a ? a->img.n_tcp : 0, a ? a->img.n_udp : 0,
                              r ? hr.data() : nullptr, r ? r->n4 : 0, r ? r->n6 : 0,
                              h ? hg.data() : nullptr, h ? h->img.n_groups : 0, extra_labels, buf,
                              cap, len);
}

// ---------------------------------------------------------------------------
// Control-plane mirrors
// ---------------------------------------------------------------------------
}  // extern "C"

struct vc_secgroup {
    vc::SecurityGroup sg;
};
struct vc_routetable {
    vc::RouteTable rt;
};

extern "C" {

int vc_secgroup_new(const char* alias, int default_allow, vc_secgroup** out) {
    if (!alias || !out) return fail(VC_EINVAL, "null argument");
    *out = new vc_secgroup{vc::SecurityGroup(alias, default_allow != 0)};
    return VC_OK;
}

void vc_secgroup_free(vc_secgroup* sg) { delete sg; }

int vc_secgroup_set_default(vc_secgroup* sg, int default_allow) {
    if (!sg) return fail(VC_EINVAL, "null argument");
    sg->sg.set_default_allow(default_allow != 0);
    return VC_OK;
}

int vc_secgroup_add_rule(vc_secgroup* sg, const char* alias, const vc_net* net, int proto,
                         int min_port, int max_port, int allow) {
    if (!sg || !alias || !net) return fail(VC_EINVAL, "null argument");
    vc::SecurityGroupRule r{alias, *net, proto == VC_PROTO_TCP ? VC_PROTO_TCP : VC_PROTO_UDP,
                            min_port, max_port, allow != 0};
    int rc = sg->sg.add_rule(std::move(r));
    return rc ? fail(rc, std::string("security-group-rule already exists: ") + alias) : VC_OK;
}

int vc_secgroup_remove_rule(vc_secgroup* sg, const char* alias) {
    if (!sg || !alias) return fail(VC_EINVAL, "null argument");
    int rc = sg->sg.remove_rule(alias);
    return rc ? fail(rc, std::string("security-group-rule not found: ") + alias) : VC_OK;
}

int vc_secgroup_rules(const vc_secgroup* sg, int proto, vc_acl_rule* out, int cap) {
    if (!sg) return fail(VC_EINVAL, "null argument");
    const auto& l = proto == VC_PROTO_TCP ? sg->sg.tcp() : sg->sg.udp();
    for (int i = 0; i < cap && i < static_cast<int>(l.size()); ++i)
        out[i] = vc_acl_rule{l[i].network, l[i].min_port, l[i].max_port, l[i].allow ? 1 : 0};
    return static_cast<int>(l.size());
}

int vc_secgroup_compile(vc_ctx* ctx, const vc_secgroup* sg) {
    if (!sg) return fail(VC_EINVAL, "null argument");
    std::vector<vc_acl_rule> t(sg->sg.tcp().size()), u(sg->sg.udp().size());
    vc_secgroup_rules(sg, VC_PROTO_TCP, t.data(), static_cast<int>(t.size()));
    vc_secgroup_rules(sg, VC_PROTO_UDP, u.data(), static_cast<int>(u.size()));
    return vc_compile_acl(ctx, t.data(), static_cast<int>(t.size()), u.data(),
                          static_cast<int>(u.size()), sg->sg.default_allow() ? 1 : 0);
}

int vc_routetable_new(const vc_net* v4net, const vc_net* v6net, int vni, vc_routetable** out) {
    if (!out) return fail(VC_EINVAL, "null argument");
    if (!v4net && v6net) return fail(VC_EINVAL, "v6 network needs a v4 network");
    *out = v4net ? new vc_routetable{vc::RouteTable(*v4net, v6net, vni)} : new vc_routetable{};
    return VC_OK;
}

void vc_routetable_free(vc_routetable* rt) { delete rt; }

int vc_routetable_add_rule(vc_routetable* rt, const char* alias, const vc_net* net, int to_vni,
                           const uint8_t* via_ip, int via_len) {
    if (!rt || !alias || !net) return fail(VC_EINVAL, "null argument");
    vc::RouteRule r;
    r.alias = alias;
    r.rule = *net;
    if (via_ip) {
        if (via_len != 4 && via_len != 16) return fail(VC_EINVAL, "bad via ip");
        r.has_ip = true;
        std::memcpy(r.ip, via_ip, via_len);
        r.ip_len = via_len;
    } else {
        r.to_vni = to_vni;
    }
    int rc = rt->rt.add_rule(r);
    return rc ? fail(rc, std::string("cannot add route ") + alias) : VC_OK;
}

int vc_routetable_add_rules(vc_routetable* rt, const char* alias_prefix, const vc_net* nets, int n,
                            int to_vni) {
    if (!rt || !alias_prefix || (n && !nets) || n < 0) return fail(VC_EINVAL, "bad arguments");
    std::vector<vc::RouteRule> v(n);
    for (int i = 0; i < n; ++i) {
        v[i].alias = std::string(alias_prefix) + std::to_string(i);
        v[i].rule = nets[i];
        v[i].to_vni = to_vni;
    }
    int rc = rt->rt.add_rules_bulk(std::move(v));
    return rc < 0 ? fail(rc, "cannot add routes") : rc;
}

int vc_routetable_del_rule(vc_routetable* rt, const char* alias) {
    if (!rt || !alias) return fail(VC_EINVAL, "null argument");
    int rc = rt->rt.del_rule(alias);
    return rc ? fail(rc, std::string("route not found: ") + alias) : VC_OK;
}

int vc_routetable_rules(const vc_routetable* rt, int family, vc_net* out, int cap) {
    if (!rt) return fail(VC_EINVAL, "null argument");
    const auto& l = family == 4 ? rt->rt.v4() : rt->rt.v6();
    for (int i = 0; i < cap && i < static_cast<int>(l.size()); ++i) out[i] = l[i].rule;
    return static_cast<int>(l.size());
}

int vc_routetable_compile(vc_ctx* ctx, const vc_routetable* rt) {
    if (!rt) return fail(VC_EINVAL, "null argument");
    std::vector<vc_net> a(rt->rt.v4().size()), b(rt->rt.v6().size());
    vc_routetable_rules(rt, 4, a.data(), static_cast<int>(a.size()));
    vc_routetable_rules(rt, 6, b.data(), static_cast<int>(b.size()));
    return vc_compile_routes(ctx, a.data(), static_cast<int>(a.size()), b.data(),
                             static_cast<int>(b.size()));
}

int vc_routetables_compile_vni(vc_ctx* ctx, const vc_routetable* const* tables, int n) {
    if (n < 0 || (n && !tables)) return fail(VC_EINVAL, "bad table array");
    std::vector<int32_t> vni, o4{0}, o6{0};
    std::vector<vc_net> a, b;
    for (int t = 0; t < n; ++t) {
        if (!tables[t]) return fail(VC_EINVAL, "null table");
        vni.push_back(tables[t]->rt.vni());
        for (const auto& r : tables[t]->rt.v4()) a.push_back(r.rule);
        for (const auto& r : tables[t]->rt.v6()) b.push_back(r.rule);
        o4.push_back(static_cast<int32_t>(a.size()));
        o6.push_back(static_cast<int32_t>(b.size()));
    }
    return vc_compile_vni_routes(ctx, vni.data(), a.data(), o4.data(), b.data(), o6.data(), n);
}

}  // extern "C"

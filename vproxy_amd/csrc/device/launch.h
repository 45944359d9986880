// launch.h -- host-callable launchers for the classifier kernels.
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

#include <atomic>
#include <condition_variable>
#include <mutex>

#include "../common/images.h"
#include "vclassify.h"

namespace vc {

// hit-counter histogram modes (counters.hip)
#define VC_HIST_PLAIN 0   // v >= 0 -> base + v, v < 0 -> null_bin
#define VC_HIST_ACL 1     // aux = proto: tcp v -> v, udp v -> nt + v, -1 -> null_bin (+1 udp)
#define VC_HIST_DNS 2     // aux = kind: counted only where kind == VC_DNS_GROUP
#define VC_HIST_ROUTE 3   // aux = family: v4 v -> v, v6 v -> nt + v; -1 -> null_bin (+1 for v6)

// A context-owned event for handing work from the caller's stream to a
// second one (record + wait under the mutex).  One event re-recorded per
// call: creating and destroying an event per call made hipEventDestroy wait
// for the pending record, which blocked the host until the kernel ended.
struct Handoff {
    hipEvent_t ev = nullptr;
    std::mutex* mu = nullptr;
    // `to` waits for everything issued on `from` so far
    hipError_t operator()(hipStream_t from, hipStream_t to) const {
        std::lock_guard<std::mutex> lk(*mu);
        hipError_t e = hipEventRecord(ev, from);
        return e == hipSuccess ? hipStreamWaitEvent(to, ev, 0) : e;
    }
};

// Device scratch owned by a context and reused across calls: a few arenas,
// each ordered by an event recorded where its last user finished with it.
// A lease makes the caller's stream wait (in stream order, not on the host)
// for the arena's previous user; releasing records the event on the stream
// that used it last.  Replaces stream-ordered pool allocations, whose
// hipFreeAsync blocked the calling thread for milliseconds on this runtime
// (profiles/r02_hip_api_free_async.txt).
class ScratchRing {
public:
    static constexpr int kSlots = 4;
    // grow_all (the counter passes): a batch larger than any before grows
    // every idle arena at once.  Off (the HTTP rewrite space): a call takes
    // an idle arena that already fits, else grows only the largest idle one,
    // so a steady stream of calls keeps one large arena, not four.
    hipError_t init(bool grow_all = true);
    void destroy();           // after the device is idle
    hipError_t acquire(size_t bytes, hipStream_t s, int* slot, uint8_t** base);
    hipError_t release(int slot, hipStream_t s);

private:
    struct Slot {
        uint8_t* p = nullptr;
        size_t cap = 0;
        hipEvent_t ev = nullptr;
        bool busy = false;
        bool used = false;
    };
    std::mutex mu_;
    std::condition_variable cv_;
    Slot slots_[kSlots];
    int next_ = 0;
    bool grow_all_ = true;
};

// Work counters of the dynamically scheduled string kernels (hint, DNS,
// SNI): the waves of a launch take 64-item chunks from one device counter,
// so workgroups that become resident late -- beside another stream's kernel
// -- do not hold back a fixed share of the work.  The wave that takes the
// launch's last ticket resets the counter to zero, so a slot needs no
// memset before reuse; slots go round-robin (kSlots launches in flight, far
// more than the context's streams ever queue).  A launch that fails or
// faults part-way can leave its slot nonzero, and every later launch on
// that slot would skip work.  The context bumps the ring's error epoch on
// any device error (capi.cpp `launched`); a slot handed out afterwards whose
// own epoch is older is zeroed first, with a 4-byte memset on the launching
// stream, so it is ordered before the kernel that uses it and touches no
// other slot: zeroing the whole ring instead could reset the counter of a
// ticketed kernel still running on another stream (the pool pass beside the
// pipeline, another caller's DNS launch), which would then hand its tickets
// out twice and leave its slot nonzero.  A slot comes round again only
// kSlots launches later, long after its previous kernel ended.
class TicketRing {
public:
    static constexpr uint32_t kSlots = 4096;
    // words per slot: [0] the work counter; [1], [2] a follow-up kernel's
    // (hint_defer_kernel: deferred lanes, workgroups done); [3] spare
    static constexpr uint32_t kWords = 4;
    hipError_t init() {
        hipError_t e = hipMalloc(reinterpret_cast<void**>(&d_), kSlots * kWords * sizeof(uint32_t));
        if (e == hipSuccess) e = hipMemset(d_, 0, kSlots * kWords * sizeof(uint32_t));
        for (uint32_t k = 0; k < kSlots; ++k) epoch_of_[k].store(0);
        return e;
    }
    void destroy() {            // after the device is idle
        if (d_) (void)hipFree(d_);
        d_ = nullptr;
    }
    void mark_dirty() { epoch_.fetch_add(1); }
    uint32_t* next(hipStream_t s) {
        if (!d_) return nullptr;
        const uint32_t k = next_.fetch_add(1) % kSlots;
        const uint32_t e = epoch_.load();
        if (epoch_of_[k].load() != e) {
            // a slot that cannot be zeroed is not used: null = the static split
            if (hipMemsetAsync(d_ + kWords * k, 0, kWords * sizeof(uint32_t), s) != hipSuccess)
                return nullptr;
            epoch_of_[k].store(e);
        }
        return d_ + kWords * k;
    }

private:
    uint32_t* d_ = nullptr;
    std::atomic<uint32_t> next_{0};
    std::atomic<uint32_t> epoch_{0};
    std::atomic<uint32_t> epoch_of_[kSlots];
};

struct LaunchCfg {
    int num_cus = 256;        // CUs the stream may use (its CU mask, else all)
    bool cu_masked = false;   // the stream has a CU mask narrower than the device
    hipStream_t stream = nullptr;
    Handoff handoff;
    ScratchRing* scratch = nullptr;   // counter-pass scratch (required by the launchers)
    ScratchRing* http_scratch = nullptr;   // the HTTP rewrite space (launch_http_hint)
    TicketRing* tickets = nullptr;    // work counters; null: static grid-stride split
};

// Device-side check flags of a VC_DEVCHECK build (dev_common.h VC_CHECK):
// the first failing site of any kernel file, its hit count and two detail
// words, read and cleared.  A normal build reports nothing.
hipError_t devcheck_take(uint32_t out[4]);

// Workgroups per CU that can be resident at once for `kernel` (occupancy
// query, cached per kernel).
int resident_per_cu(const void* kernel, int block, size_t shmem);

// Grid of a grid-stride kernel: as many workgroups as fit the device at
// once (every workgroup starts in the first round; a larger grid leaves a
// partial second round), and no more than the work needs.
inline int resident_grid(const LaunchCfg& c, const void* kernel, int block, size_t shmem,
                         int64_t want_blocks) {
    const int64_t cap = int64_t(c.num_cus) * resident_per_cu(kernel, block, shmem);
    if (want_blocks < 1) want_blocks = 1;
    return int(want_blocks < cap ? want_blocks : cap);
}


hipError_t launch_acl_v4(const LaunchCfg& c, const AclImage& img, const uint8_t* proto,
                         const uint32_t* src4, const uint16_t* port, int64_t n, int32_t* out,
                         uint8_t* allow, unsigned long long* counters);
hipError_t launch_acl_v6(const LaunchCfg& c, const AclImage& img, const uint8_t* proto,
                         const uint8_t* src6, const uint16_t* port, int64_t n, int32_t* out,
                         uint8_t* allow, unsigned long long* counters);
// counters (optional): rule i -> counters[rule_base + i], null -> counters[none_at]
hipError_t launch_route_v4(const LaunchCfg& c, const TrieImage& t, const uint32_t* dst4, int64_t n,
                           int32_t* out, unsigned long long* counters, int64_t rule_base,
                           int64_t none_at);
hipError_t launch_route_v6(const LaunchCfg& c, const TrieImage& t, const uint8_t* dst6, int64_t n,
                           int32_t* out, unsigned long long* counters, int64_t rule_base,
                           int64_t none_at);
// images.h TrieImage.wide from a device copy of the trie (root + records):
// 4 words per root slot, on `stream`
hipError_t build_wide_root(const uint32_t* nodes, int root_bits, uint32_t* wide,
                           hipStream_t stream);
hipError_t launch_hint(const LaunchCfg& c, const HintImage& img, const uint8_t* host_blob,
                       const uint32_t* host_off, const uint8_t* host_null, const uint16_t* port,
                       const uint8_t* uri_blob, const uint32_t* uri_off, const uint8_t* uri_null,
                       int64_t n, int32_t* out, unsigned long long* counters);
hipError_t launch_dns(const LaunchCfg& c, const HostsImage& hosts, const HintImage& hints,
                      const uint8_t* qblob, const uint32_t* qoff, int64_t n, uint8_t* kind,
                      int32_t* value, unsigned long long* group_counters);
// HttpContext.connectionHint + Upstream.searchForGroup over HTTP/1 request
// heads (http.hip); blob_bytes >= off[n] sizes the launch's scratch
hipError_t launch_http_hint(const LaunchCfg& c, const HintImage& img, const uint8_t* blob,
                            int64_t blob_bytes, const uint32_t* off, int64_t n, int32_t* out_group,
                            uint8_t* out_kind);
// SSLContextHolder.choose over a batch of SNI names (hint.hip)
hipError_t launch_certs(const LaunchCfg& c, const CertImage& certs, const uint8_t* blob,
                        const uint32_t* off, const uint8_t* null, int64_t n, int32_t* out);
// Mirror filters (mirror.hip)
hipError_t launch_mirror_match(const LaunchCfg& c, const MirrorImage& img,
                               const MirrorSwImage* sw, int32_t origin, const vc_mirror_items& in,
                               int64_t n, uint64_t* out);
hipError_t launch_mirror_switch(const LaunchCfg& c, const MirrorImage& img,
                                const MirrorSwImage* sw, int32_t origin, const uint8_t* blob,
                                const uint32_t* off, int64_t n, int layer, uint64_t* out);
// Combined ACL -> route -> host pipeline (classify.hip).  Device pointers;
// family null = every packet IPv4, host_id null = no hostname stage.
struct PipeArgs {
    const uint8_t* family;
    const uint8_t* proto;
    const uint32_t* src4;
    const uint32_t* dst4;
    const uint8_t* src6;           // 16-byte aligned
    const uint8_t* dst6;
    const uint16_t* dport;
    const uint32_t* host_id;
    const int32_t* pool_group;
    int64_t n_pool;
    int64_t n;
    int32_t* out_acl;
    int32_t* out_route;
    int32_t* out_group;
    uint8_t* out_allow;
    // -1: src6 / dst6 have a row per packet; >= 0: they hold only the IPv6
    // packets' addresses, n6c rows in packet order (vc_pipeline_c6_dev)
    int64_t n6c = -1;
};
// Counter arrays of the pinned snapshots (null = not counted): ACL
// [tcp][udp][tcp default][udp default], route [v4][v6][v4 null][v6 null],
// group [handles][null].
struct PipeCounters {
    unsigned long long* acl;
    unsigned long long* route;
    unsigned long long* group;
    int32_t n_groups;
};
// kernel_done (optional) is recorded right after the classify kernel; the
// counter finish passes run on count_stream (after the kernel) when it is
// given, else on c.stream.
hipError_t launch_pipeline(const LaunchCfg& c, const AclImage& acl, const RouteImage& route,
                           int32_t n4, int32_t n6, const PipeArgs& p, const PipeCounters& cnt,
                           hipEvent_t kernel_done, hipStream_t count_stream);

// ServerGroup source hashing (select.hip); family 4: src = uint32 v4 keys,
// 6: 16-byte addresses (16-byte aligned); view = VC_SOURCE_*.
hipError_t launch_source(const LaunchCfg& c, const ServerImage& img, const int32_t* group,
                         const void* src, int family, int64_t n, int view, int32_t* out);

// Header extraction (packet.hip); out arrays are device pointers, src6/dst6
// 16-byte aligned.
hipError_t launch_packets(const LaunchCfg& c, const uint8_t* blob, const uint32_t* off, int64_t n,
                          int layer, const vc_pkt_out& out);
// Parse + bare-VXLAN ACL on the sender + inner route in one pass (packet.hip)
hipError_t launch_dns_datagrams(const LaunchCfg& c, const HostsImage& hosts,
                                const HintImage& hints, const AclImage& acl, const uint8_t* blob,
                                const uint32_t* off, int64_t n, const uint8_t* rfam,
                                const uint32_t* r4, const uint8_t* r6, const uint16_t* rport,
                                uint8_t* status, int32_t* out_acl, uint8_t* nq, uint16_t* qtype,
                                uint8_t* kind, int32_t* value);
hipError_t launch_switch(const LaunchCfg& c, const AclImage& acl, const RouteImage& rt,
                         const VniImage& vt, const uint8_t* blob, const uint32_t* off, int64_t n, int layer,
                         const vc_pkt_out& out, const uint8_t* rfam, const uint32_t* r4,
                         const uint8_t* r6, int bind_port, const AclPortImage& ap,
                         int32_t* out_acl, uint8_t* out_allow, int32_t* out_route);

// Large counter spaces (counters.hip): bucket partition + per-bucket LDS
// histograms, split so a producer kernel (the pipeline) can supply the
// per-workgroup bucket counts itself: begin (carve the arrays out of leased
// scratch), producer writes counts[bucket * nblk + block] over pipe_slice()
// slices of nblk workgroups, finish (scan, scatter, histogram).
struct BigHist {
    int nbk = 0, nblk = 0;
    uint32_t* counts = nullptr;
    uint32_t* offsets = nullptr;
    uint32_t* seg_off = nullptr;
    uint16_t* tmp = nullptr;       // bucket-partitioned bins (within-bucket index)
};
bool big_hist_applies(int64_t n, int64_t nval);
int big_hist_bucket_shift();
size_t big_hist_bytes(int64_t n, int64_t nval, int nblk);
void big_hist_begin(uint8_t* scratch, int64_t n, int64_t nval, int nblk, BigHist* h);
hipError_t big_hist_finish(const LaunchCfg& c, BigHist* h, int mode, const int32_t* idx,
                           const uint8_t* aux, int64_t n, int32_t nt, int64_t nval, int64_t base,
                           unsigned long long* counters, bool run);

// Histogram a classify output array into uint64 hit counters.  Values in
// [0, nval) land at counters[base + v]; nulls at counters[null_bin].
hipError_t launch_hist(const LaunchCfg& c, int mode, const int32_t* idx, const uint8_t* aux,
                       int64_t n, int64_t nval, int64_t base, int64_t null_bin, int32_t nt,
                       unsigned long long* counters);

}  // namespace vc

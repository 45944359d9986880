// hint.hip -- Upstream.searchForGroup(Hint) and DNSServer classification.
//
//   Hint.formatHost / formatUri      base/.../processor/Hint.java:57-90
//   Hint.matchLevel                  Hint.java:100-160
//   Upstream.searchForGroup          core/.../svrgroup/Upstream.java:187-198
//   IP.isIpv6 / isIpLiteral          base/src/main/java/vfd/IP.java:158-300
//   DNSServer.handleRequest (class.) core/src/main/java/vproxy/dns/DNSServer.java:116-166
//
// One lane per hint.  The linear argmax over all groups becomes a handful of
// hash probes: the query host is scanned right-to-left once, producing the
// reversed-FNV hash of every dot-suffix ("." + annoHost candidates) and of
// the whole host; each probe is confirmed by a byte compare.
#include "acl_dev.h"
#include "hint_dev.h"
#include "launch.h"
#include "chunks.h"
#include "stage.h"

namespace vcd {

constexpr int kHintBlock = 256;
constexpr int kWaves = kHintBlock / 64;
constexpr uint32_t kStageBytes = 4096;   // per wave: 64 names of up to 64 B on average
constexpr uint32_t kStageWords = (kStageBytes + 2 * kApron) / 4;
// Minimum waves per SIMD.  hint_kernel: 7 holds it at 72 VGPRs: C4 0.866 ->
// 0.817 ms against 5 waves at 96 VGPRs (profiles/r02_ab_hint_occupancy.txt);
// the call-free kernel at 8 (64 VGPRs) spills 20 and loses (0.833 against
// 0.772 ms, profiles/r04_ab_minw.txt).  dns_kernel: 7 (72 VGPRs, no spills)
// since its loop has no call (0.913 against 0.928 ms at 6); with the calls
// it spilled in the hot path at 7 (1.26 against 1.07 ms, round 2).  On
// chunk pairs (VC_DNS_PAIR): 6 (80 VGPRs): 0.78 ms against 0.78 at 7 (72
// VGPRs, 11 spilled) and 0.83 at 5 (90, none), against 0.807 on single
// chunks (profiles/r04_ab_dns_pair.txt); with its results stored in item
// order (VC_DNS_ORDERED) it keeps nothing in scratch and runs 0.764 against
// 0.776 ms (profiles/r04_ab_dns_ordered.txt).
#ifndef VC_HINT_MINW
#define VC_HINT_MINW 7
#endif
#ifndef VC_HINT_SWAP
#define VC_HINT_SWAP 1
#endif
#ifndef VC_CERT_SWAP
#define VC_CERT_SWAP 1
#endif
#ifndef VC_DNS_PAIR
#define VC_DNS_PAIR 1
#endif
#ifndef VC_DNS_PRE
#define VC_DNS_PRE 2
#endif
// VC_DNS_ORDERED: dns_kernel's results stored in item order (chunk_loop store)
#ifndef VC_DNS_ORDERED
#define VC_DNS_ORDERED 1
#endif
#ifndef VC_CERT_ORDERED
#define VC_CERT_ORDERED 1
#endif
// hint_kernel's and dns_kernel's static shares (chunks.h ChunksT S)
#ifndef VC_HINT_STATIC
#define VC_HINT_STATIC 60
#endif
#ifndef VC_DNS_STATIC
#define VC_DNS_STATIC 50
#endif
#ifndef VC_DNS_SWAP
#define VC_DNS_SWAP VC_HINT_SWAP
#endif
#ifndef VC_HINT_PRE
#define VC_HINT_PRE 2
#endif
#ifndef VC_HINT_TICKETS                 // 0: static split (A/B only)
#define VC_HINT_TICKETS 1
#endif
#ifndef VC_HINT_DEFER
#define VC_HINT_DEFER 1
#endif
#ifndef VC_DNS_DEFER
#define VC_DNS_DEFER 1
#endif
// Workgroups of the follow-up (deferred-lane) kernels.  Each reads the
// launch's deferred count and adds one to its done count, so with nothing
// deferred the launch costs those loads and same-address atomics; with many
// deferred lanes the grid strides over the batch.  With nothing deferred
// the C4 follow-up takes 4.4 us at 64 workgroups, 11.7 us at 512
// (profiles/r04_ab_defer_grid.txt); 128 keeps a heavily deferred batch (an
// IPv6-literal Host header on every packet) on half the CUs.
#ifndef VC_DEFER_GRID
#define VC_DEFER_GRID 128
#endif
#ifndef VC_DNS_MINW
#define VC_DNS_MINW 6
#endif


#if defined(VC_HINT_PROF)
// Profiling build: phase cycles summed over the waves of every launch
// (0 stage, 1 scan, 2 tag groups, 3 records, 4 DNS hosts, 5 output), [6] waves.
__device__ unsigned long long vc_hint_prof[kProfPhases + 1];
__device__ __forceinline__ void prof_begin() {
    uint64_t* t = vc_prof_lds + (threadIdx.x >> 6) * (kProfPhases + 1);
    if ((threadIdx.x & 63) < kProfPhases) t[threadIdx.x & 63] = 0;
    if ((threadIdx.x & 63) == 0) t[kProfPhases] = clock64();
    __builtin_amdgcn_wave_barrier();
}
__device__ __forceinline__ void prof_end() {
    const uint64_t* t = vc_prof_lds + (threadIdx.x >> 6) * (kProfPhases + 1);
    const int l = int(threadIdx.x & 63);
    if (l < kProfPhases) atomicAdd(&vc_hint_prof[l], (unsigned long long)t[l]);
    if (l == kProfPhases) atomicAdd(&vc_hint_prof[l], 1ull);
}
constexpr size_t kProfLds = size_t(kWaves) * (kProfPhases + 1) * 8;
#define VC_PBEGIN() prof_begin()
#define VC_PEND() prof_end()
#else
constexpr size_t kProfLds = 0;
#define VC_PBEGIN() ((void)0)
#define VC_PEND() ((void)0)
#endif

// The chunk loop of the string kernels.  A wave stages its chunk's items
// (contiguous in the blob) into LDS with one coalesced copy; when the next
// chunk is also this wave's and both fit the stage, it stages the two
// together and runs body(c, staged, a0, a, e) for each from one copy.
// kPre 2: every offset the two chunks need (the staged span, and each
// lane's [a, e)) is loaded together up front, so a pair costs one offset and
// one blob round trip before its first scan instead of four dependent ones
// (SNI 0.638 -> 0.624 ms; the call-free hint kernel 0.769 -> 0.761 ms,
// profiles/r04_ab_hint_pre.txt -- with the slow-path calls in its loop the
// live offsets spilled: 0.81 -> 0.92 ms).  kPre 0: each chunk's [a, e) is
// loaded at its body.
// kPre 3: as 2, and the next pair's offsets are loaded before this pair is
// staged, so they arrive with this pair's bytes: a pair costs one blob round
// trip before its first scan (the ticket counter is read one pair early).
// A lane's starts in the two chunks; its ends are the next lane's starts
// (lane 63: the spans' ends o1, o2), taken by a lane shift when used, so the
// prefetched pair holds two VGPRs and three SGPRs.
// VC_OFF_NT: the chunk loop's offset loads carry the nontemporal hint (a
// streamed array, like the staged blob).  Off: each offset is read twice (a
// lane's start and the previous lane's end, a chunk's span ends), and the
// hinted lines are gone before the second read -- C4 0.598 -> 0.607 ms, DNS
// 0.745 -> 0.757, SNI 0.521 -> 0.532 (profiles/r05_ab_off_nt_rejected.jsonl)
#ifndef VC_OFF_NT
#define VC_OFF_NT 0
#endif
__device__ __forceinline__ uint32_t off_ld(const uint32_t* p) {
#if VC_OFF_NT
    return __builtin_nontemporal_load(p);
#else
    return *p;
#endif
}

struct PairOffs {
    uint32_t A0 = 0, A1 = 0, o0 = 0, o1 = 0, o2 = 0;
};

__device__ __forceinline__ PairOffs pair_offs(const uint32_t* off, int64_t base, int64_t n) {
    PairOffs r;
    const int64_t i0 = base + int(threadIdx.x & 63), i1 = i0 + 64;
    r.A0 = off[i0 < n ? i0 : n];
    r.A1 = off[i1 < n ? i1 : n];
    r.o0 = uint32_t(__builtin_amdgcn_readfirstlane(int(off[base])));
    r.o1 = uint32_t(__builtin_amdgcn_readfirstlane(int(off[base + 64 < n ? base + 64 : n])));
    r.o2 = uint32_t(__builtin_amdgcn_readfirstlane(int(off[base + 128 < n ? base + 128 : n])));
    VC_CHECK(r.o0 <= r.o1 && r.o1 <= r.o2 && r.o2 <= off[n], 301, base, r.o2);
    return r;
}

// kSwap (kPre 2): each lane runs the shorter of its two items in the pair's
// first body call and the longer in the second.  A body's scan runs to its
// wave's longest name, so the first call ends near the lanes' upper
// quantile of the shorter names instead of the longest of 64.

// the lane's end: the next lane's start, or `last` for lane 63
__device__ __forceinline__ uint32_t lane_end(uint32_t a, uint32_t last) {
    const uint32_t nx = uint32_t(__shfl_down(int(a), 1, 64));
    return (threadIdx.x & 63) == 63 ? last : nx;
}

// store (optional; kPre 2): the body returns its item's result and
// store(i, r) writes the pair's results after both calls, in item order, so
// the lane swap does not split each output line over two partial writes.
struct NoStore {
    template <class R>
    __device__ void operator()(int64_t, R) const {}
};

template <uint32_t kBytes, bool kPair, int kPre, bool kSwap = false, class Body, class Ch,
          class Store = NoStore>
__device__ __forceinline__ void chunk_loop(Ch& ch, int w, const uint8_t* blob,
                                           const uint32_t* off, int64_t n, uint32_t* stage,
                                           Body body, Store store = Store{}) {
    constexpr bool kOrdered = !std::is_same_v<Store, NoStore>;
    static_assert(!kOrdered || kPre == 2, "ordered stores need both spans up front");
    const int lane = int(threadIdx.x & 63);
    if constexpr (kPre == 3) {
        int64_t c = ch.first(w);
        PairOffs cur;
        if (c < ch.nchunks) cur = pair_offs(off, c * 64, n);
        while (c < ch.nchunks) {
            // a pair when chunk c + 1 is this wave's too and both fit the stage
            const bool two = kPair && blob && ch.paired(c) &&
                             cur.o2 - (cur.o0 & ~3u) <= kBytes;
            const int nsub = two ? 2 : 1;
            const int64_t cn = ch.next(c + nsub - 1);
            PairOffs nxt;
            if (cn < ch.nchunks) nxt = pair_offs(off, cn * 64, n);
            uint32_t a0 = 0;
            const bool staged = blob && stage_wave<kBytes>(blob, cur.o0, two ? cur.o2 : cur.o1,
                                                           stage, &a0);
            VC_PMARK(0);
            body(c * 64 + lane, staged, a0, cur.A0, lane_end(cur.A0, cur.o1));
            if (two) body(c * 64 + 64 + lane, staged, a0, cur.A1, lane_end(cur.A1, cur.o2));
            wave_done();
            VC_PMARK(5);
            c = cn;
            cur = nxt;
        }
        return;
    }
    for (int64_t c = ch.first(w); c < ch.nchunks;) {
        const int64_t base = c * 64;
        const bool pair = kPair && ch.paired(c);
        // this lane's [A0, E0) and [A1, E1) in chunks c and c + 1 (clamped
        // to n past the end), and the spans' ends o1 = off[base + 64],
        // o2 = off[base + 128]
        uint32_t A0 = 0, E0 = 0, A1 = 0, E1 = 0, o0 = 0, o1 = 0, o2 = 0;
        if (off) {
            const int64_t i0 = base + lane, i1 = i0 + 64;
            if (kPre >= 1) {
                A0 = off_ld(off + (i0 < n ? i0 : n));
                E0 = off_ld(off + (i0 + 1 < n ? i0 + 1 : n));
            }
            if (kPre >= 2) {
                A1 = off_ld(off + (i1 < n ? i1 : n));
                E1 = off_ld(off + (i1 + 1 < n ? i1 + 1 : n));
            }
            o0 = off_ld(off + base);
            o1 = off_ld(off + (base + 64 < n ? base + 64 : n));
            o2 = off_ld(off + (base + 128 < n ? base + 128 : n));
            VC_CHECK(o0 <= o1 && o1 <= o2 && o2 <= off[n], 301, base, o2);
        }
        uint32_t a0 = 0;
        int nsub = 1;
        bool staged = false;
        if (blob) {
            if (pair && stage_wave<kBytes>(blob, o0, o2, stage, &a0)) {
                staged = true;
                nsub = 2;
            }
            if (!staged) staged = stage_wave<kBytes>(blob, o0, o1, stage, &a0);
        }
        VC_PMARK(0);
        // the lane's shorter item first (see kSwap above); a lane mask, so
        // the items' indices stay a scalar base plus the lane
        const bool sw = kSwap && kPre == 2 && nsub == 2 && E1 - A1 < E0 - A0;
        if (sw) {
            const uint32_t ta = A0, te = E0;
            A0 = A1; E0 = E1; A1 = ta; E1 = te;
        }
        if constexpr (kOrdered) {
            const int64_t i = base + lane;
            VC_CHECK(!off || (A0 <= E0 && E0 <= off[n]), 303, base, E0);
            const auto r0 = body(sw ? i + 64 : i, staged, a0, A0, E0);
            if (nsub == 1) {
                if (i < n) store(i, r0);
            } else {
                VC_CHECK(!off || (A1 <= E1 && E1 <= off[n]), 303, base, E1);
                const auto r1 = body(sw ? i : i + 64, staged, a0, A1, E1);
                if (i < n) store(i, sw ? r1 : r0);
                if (i + 64 < n) store(i + 64, sw ? r0 : r1);
            }
        }
        for (int sub = 0; sub < (kOrdered ? 0 : nsub); ++sub) {
            if (off && (kPre == 0 || (kPre == 1 && sub == 1))) {
                const int64_t i = base + 64 * sub + lane;
                A0 = off[i < n ? i : n];
                E0 = off[i + 1 < n ? i + 1 : n];
            }
            VC_CHECK(!off || (A0 <= E0 && E0 <= off[n]), 303, base, E0);
            body(base + ((sub != 0) != sw ? 64 : 0) + lane, staged, a0, kPre == 2 && sub ? A1 : A0, kPre == 2 && sub ? E1 : E0);
        }
        wave_done();
        VC_PMARK(5);
        c = ch.next(c + nsub - 1);
    }
}

// kDefer: no call in the loop -- lanes that need an out-of-line step are
// written as kDeferred and counted in ticket[1] for hint_defer_kernel, which
// runs next on the stream.  With hint-uris in the batch and the image, a
// port-0 lane with a uri takes the host fast path too (host_only_fast's
// `uri`: the uri cannot change the answer unless the top host level has
// candidates it orders) and defers otherwise; a uri lane with a port or no
// host always defers.  !kDefer (an unstaged batch): every lane is finished
// here, uri lanes through the general path.
template <bool kStage, bool kDefer, bool kUri = false>
__global__ __launch_bounds__(kHintBlock, VC_HINT_MINW) void hint_kernel(
    HintImage img, const uint8_t* __restrict__ host_blob, const uint32_t* __restrict__ host_off,
    const uint8_t* __restrict__ host_null, const uint16_t* __restrict__ port,
    const uint8_t* __restrict__ uri_blob, const uint32_t* __restrict__ uri_off,
    const uint8_t* __restrict__ uri_null, int64_t n, int32_t* __restrict__ out,
    uint32_t* __restrict__ ticket) {
    __shared__ uint32_t stage[kWaves][kStageWords];
    const int lane = int(threadIdx.x & 63), w = int(threadIdx.x >> 6);
    ChunksT<kPerTicket, kTailChunks, kTailRounds, VC_HINT_STATIC> ch(ticket, (n + 63) / 64);
    // kUri: the deferring kernel's instance for batches with uris (the
    // host-only instance, the C5 pool pass's, carries no uri logic)
    const bool general = (kUri || !kDefer) && uri_blob && img.has_uri_keys;
    // Out-of-line slow paths take the image by address; give them their own
    // copy so the fast path keeps reading the kernel argument (whose table
    // pointers the compiler then knows to be global).
    HintImage slow_img = img;
    // kUri: deferred lanes are common (a few percent), so a wave counts them
    // over its chunks and adds once at its end -- one same-address atomic
    // per chunk (C4uri: 262K per launch) serialised at the memory side and
    // held the kernel at 2.9 ms
    uint32_t ndef = 0;
    VC_PBEGIN();
    chunk_loop<kStageBytes, true, VC_HINT_PRE, bool(VC_HINT_SWAP)>(ch, w, kStage ? host_blob : nullptr, host_off, n, stage[w],
                                  [&](int64_t i, bool staged, uint32_t a0, uint32_t a, uint32_t e) {
        int32_t r = -1;
        if (i < n) {
            const int p = port ? int(port[i]) : 0;
            const bool has_host = host_blob && !(host_null && host_null[i]);
            const bool has_uri = uri_blob && !(uri_null && uri_null[i]);
            const bool lane_uri = general && has_uri;
            if (kDefer && lane_uri && (p != 0 || !has_host)) {
                r = kDeferred;                    // the general search decides
            } else if (kDefer || !lane_uri) {
                // uri null (or no hint-uri anywhere): host-only levels; a
                // port-0 uri lane whose answer they already give (kDefer)
                if (has_host) {
                    if (staged)
                        r = host_only_fast<kDefer>(img, &slow_img,
                                                   LdsSrc{stage[w], int(kApron + (a - a0))},
                                                   int(e - a), p, lane_uri);
                    else if (kDefer)
                        r = kDeferred;
                    else
                        r = host_only_slow(slow_img, host_blob + a, int(e - a), p);
                    // (a uri_slot_code -- one SPLIT key holds the top host
                    // level -- is left to hint_defer_kernel's uri_in_slot:
                    // scoring the members here made every wave wait on the
                    // few lanes that need it and spilled the chunk loop)
                }
            } else if (!kDefer) {
                DStr h{nullptr, -1}, u{nullptr, -1};
                if (has_host) h = DStr{host_blob + a, int(e - a)};
                const uint32_t ua = uri_off[i], ue = uri_off[i + 1];
                u = DStr{uri_blob + ua, int(ue - ua)};
                r = hint_general(slow_img, format_host(h), p, format_uri(u));
            }
            out[i] = r;
        }
        if (kDefer && ticket) {
            const uint64_t dm = __ballot(i < n && (r == kDeferred || (kUri && is_uri_slot_code(r))));
            if constexpr (kUri)
                ndef += uint32_t(__popcll(dm));
            else if (dm && lane == 0)
                atomicAdd(ticket + 1, uint32_t(__popcll(dm)));
        }
    });
    if (kUri && ticket && ndef && lane == 0) atomicAdd(ticket + 1, ndef);
    VC_PEND();
}

// The lanes hint_kernel<*, true> deferred, through the reference-shaped
// host-only search (Hint.formatHost + every dot-suffix probed in turn), or
// for a lane with a uri (when the image has hint-uris) the general search
// (the whole Hint.matchLevel over the candidate lists); a lane left as a
// uri_slot_code takes uri_in_slot over that key's members first.
// ctl = the launch's ticket slot: [1] deferred lanes (0: nothing to do),
// [2] workgroups done; the last workgroup zeroes both for the slot's next
// launch.  Without a slot every workgroup scans.
// One deferred lane (out[i] < -1): its full search.
__device__ __forceinline__ void hint_defer_one(const HintImage& img, const uint8_t* host_blob,
                                               const uint32_t* host_off, const uint8_t* host_null,
                                               const uint16_t* port, const uint8_t* uri_blob,
                                               const uint32_t* uri_off, const uint8_t* uri_null,
                                               int64_t i, int32_t* out) {
    const int32_t o = out[i];
    if (is_uri_slot_code(o)) {          // one SPLIT key's members by uri level
        const uint32_t ua = uri_off[i], ue = uri_off[i + 1];
        const int32_t r = uri_in_slot(img, -2 - o, uri_blob + ua, int(ue - ua));
        if (r != kDeferred) {
            out[i] = r;
            return;
        }
    }
    const int p = port ? int(port[i]) : 0;
    const bool has_host = !(host_null && host_null[i]);
    const uint32_t a = host_off[i], e = host_off[i + 1];
    if (uri_blob && img.has_uri_keys && !(uri_null && uri_null[i])) {
        const uint32_t ua = uri_off[i], ue = uri_off[i + 1];
        const DStr h = has_host ? DStr{host_blob + a, int(e - a)} : DStr{nullptr, -1};
        out[i] = p == 0 ? hint_port0_uri(img, h, uri_blob + ua, int(ue - ua))
                        : hint_general(img, format_host(h), p,
                                       format_uri(DStr{uri_blob + ua, int(ue - ua)}));
    } else {
        out[i] = host_only_slow(img, host_blob + a, int(e - a), p);
    }
}

// The workgroup gathers the deferred lanes of its share into an LDS queue
// and runs them 256 at a time, every thread busy: a uri batch defers a few
// percent of its lanes (c4uri: 3 %), and run where they lie each wave
// carried its few deferred lanes through their dependent loads one after
// another (0.65 ms on c4uri).
constexpr int kDeferBlock = 256;
__global__ __launch_bounds__(kDeferBlock) void hint_defer_kernel(
    HintImage img, const uint8_t* __restrict__ host_blob, const uint32_t* __restrict__ host_off,
    const uint8_t* __restrict__ host_null, const uint16_t* __restrict__ port,
    const uint8_t* __restrict__ uri_blob, const uint32_t* __restrict__ uri_off,
    const uint8_t* __restrict__ uri_null, int64_t n, int32_t* __restrict__ out, uint32_t* ctl) {
    __shared__ uint32_t todo;
    __shared__ int qn;
    __shared__ int64_t q[2 * kDeferBlock];
    const int t = int(threadIdx.x);
    if (t == 0) {
        todo = ctl ? __hip_atomic_load(ctl + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) : 1u;
        qn = 0;
    }
    __syncthreads();
    if (todo) {
        const int64_t stride = int64_t(gridDim.x) * kDeferBlock;
        for (int64_t base = int64_t(blockIdx.x) * kDeferBlock; base < n; base += stride) {
            const int64_t i = base + t;
            if (i < n && out[i] < -1) q[atomicAdd(&qn, 1)] = i;      // LDS atomic
            __syncthreads();
            const int m = qn;
            if (m >= kDeferBlock) {                  // a full round: every thread one lane
                hint_defer_one(img, host_blob, host_off, host_null, port, uri_blob, uri_off,
                               uri_null, q[t], out);
                __syncthreads();
                if (t < m - kDeferBlock) q[t] = q[kDeferBlock + t];
                __syncthreads();
                if (t == 0) qn = m - kDeferBlock;
            }
            __syncthreads();
        }
        if (t < qn)
            hint_defer_one(img, host_blob, host_off, host_null, port, uri_blob, uri_off, uri_null,
                           q[t], out);
    }
    if (ctl && t == 0 && atomicAdd(ctl + 2, 1u) == gridDim.x - 1) {
        atomicExch(ctl + 1, 0u);
        atomicExch(ctl + 2, 0u);
    }
}

// one query's answer (chunk_loop's ordered stores)
struct DnsRes {
    int32_t value;
    uint8_t kind;
};

template <bool kStage, bool kDefer>
__global__ __launch_bounds__(kHintBlock, VC_DNS_MINW) void dns_kernel(
    HostsImage hosts, HintImage img, const uint8_t* __restrict__ qblob,
    const uint32_t* __restrict__ qoff, int64_t n, uint8_t* __restrict__ kind,
    int32_t* __restrict__ value, uint32_t* __restrict__ ticket) {
    __shared__ uint32_t stage[kWaves][kStageWords];
    const int lane = int(threadIdx.x & 63), w = int(threadIdx.x >> 6);
    ChunksT<kPerTicket, kTailChunks, kTailRounds, VC_DNS_STATIC> ch(ticket, (n + 63) / 64);
    HintImage slow_img = img;
    VC_PBEGIN();
#if VC_DNS_PAIR
    // two chunks per stage, as hint_kernel, once the loop had no call in it
    // (0.807 -> 0.78 ms)
    chunk_loop<kStageBytes, true, VC_DNS_PRE, bool(VC_DNS_SWAP) && VC_DNS_PRE == 2>(ch, w, kStage ? qblob : nullptr, qoff, n, stage[w],
                                  [&](int64_t i, bool staged, uint32_t a0, uint32_t a, uint32_t e) {
        uint8_t kd = 0;
        int32_t val = 0;
        if (i < n) {
            if (staged) {
                dns_one<kDefer>(hosts, img, &slow_img, LdsSrc{stage[w], int(kApron + (a - a0))},
                                int(e - a), &kd, &val);
            } else if (kDefer) {
                kd = kDnsDeferred;
            } else {
                dns_one(hosts, img, &slow_img, PtrSrc{qblob + a}, int(e - a), &kd, &val);
            }
#if !VC_DNS_ORDERED
            kind[i] = kd;
            value[i] = val;
#endif
        }
        if (kDefer && ticket) {
            const uint64_t dm = __ballot(i < n && kd == kDnsDeferred);
            if (dm && lane == 0) atomicAdd(ticket + 1, uint32_t(__popcll(dm)));
        }
        return DnsRes{val, kd};
    }
#if VC_DNS_ORDERED
    , [&](int64_t i, DnsRes r) {
        kind[i] = r.kind;
        value[i] = r.value;
    }
#endif
    );
#else
    // one chunk per stage: staging two (chunk_loop) adds live registers
    // that spill in this kernel's hot path (DNS 1.08 -> 1.21 ms)
    for (int64_t c = ch.first(w); c < ch.nchunks; c = ch.next(c)) {
        const int64_t base = c * 64;
        const int64_t i = base + lane;
        const int64_t last = base + 64 < n ? base + 64 : n;
        uint32_t a0 = 0;
        const bool staged = kStage && stage_wave<kStageBytes>(qblob, qoff[base], qoff[last], stage[w], &a0);
        VC_PMARK(0);
        uint8_t kd = 0;
        if (i < n) {
            const uint32_t a = qoff[i], e = qoff[i + 1];
            VC_CHECK(a <= e && e <= qoff[n], 302, i, e);
            int32_t val = 0;
            if (staged) {
                dns_one<kDefer>(hosts, img, &slow_img, LdsSrc{stage[w], int(kApron + (a - a0))},
                                int(e - a), &kd, &val);
            } else if (kDefer) {
                kd = kDnsDeferred;
            } else {
                dns_one(hosts, img, &slow_img, PtrSrc{qblob + a}, int(e - a), &kd, &val);
            }
            kind[i] = kd;
            value[i] = val;
        }
        if (kDefer && ticket) {
            const uint64_t dm = __ballot(i < n && kd == kDnsDeferred);
            if (dm && lane == 0) atomicAdd(ticket + 1, uint32_t(__popcll(dm)));
        }
        if (kStage) wave_done();
        VC_PMARK(5);
    }
#endif
    VC_PEND();
}

// The queries dns_kernel<*, true> deferred, through the complete flow
// (out-of-line IP-literal parse, high-byte transcoding, the reference-shaped
// host search).  ctl as hint_defer_kernel's.
__global__ __launch_bounds__(256) void dns_defer_kernel(
    HostsImage hosts, HintImage img, const uint8_t* __restrict__ qblob,
    const uint32_t* __restrict__ qoff, int64_t n, uint8_t* __restrict__ kind,
    int32_t* __restrict__ value, uint32_t* ctl) {
    __shared__ uint32_t todo;
    if (threadIdx.x == 0) todo = ctl ? __hip_atomic_load(ctl + 1, __ATOMIC_RELAXED,
                                                          __HIP_MEMORY_SCOPE_AGENT)
                                     : 1u;
    __syncthreads();
    if (todo) {
        for (int64_t i = int64_t(blockIdx.x) * blockDim.x + threadIdx.x; i < n;
             i += int64_t(gridDim.x) * blockDim.x) {
            if (kind[i] != kDnsDeferred) continue;
            const uint32_t a = qoff[i], e = qoff[i + 1];
            uint8_t kd;
            int32_t val;
            dns_one(hosts, img, &img, PtrSrc{qblob + a}, int(e - a), &kd, &val);
            kind[i] = kd;
            value[i] = val;
        }
    }
    if (ctl && threadIdx.x == 0 && atomicAdd(ctl + 2, 1u) == gridDim.x - 1) {
        atomicExch(ctl + 1, 0u);
        atomicExch(ctl + 2, 0u);
    }
}

template <bool kStage>
__global__ __launch_bounds__(kHintBlock) void cert_kernel(
    CertImage certs, const uint8_t* __restrict__ blob, const uint32_t* __restrict__ off,
    const uint8_t* __restrict__ null, int64_t n, int32_t* __restrict__ out,
    uint32_t* __restrict__ ticket) {
    __shared__ uint32_t stage[kWaves][kStageWords];
    const int w = int(threadIdx.x >> 6);
    ChunksT<kPerTicket, kTailChunks, kTailRounds, 25> ch(ticket, (n + 63) / 64);
    VC_PBEGIN();
    chunk_loop<kStageBytes, true, 2, bool(VC_CERT_SWAP)>(ch, w, kStage ? blob : nullptr, off, n, stage[w],
                                  [&](int64_t i, bool staged, uint32_t a0, uint32_t a, uint32_t e) {
        int32_t r = -1;
        if (i < n) {
            const bool is_null = null && null[i];
            r = staged ? cert_one(certs, LdsSrc{stage[w], int(kApron + (a - a0))}, int(e - a),
                                  is_null)
                       : cert_one(certs, PtrSrc{blob + a}, int(e - a), is_null);
#if !VC_CERT_ORDERED
            out[i] = r;
#endif
        }
        return r;
    }
#if VC_CERT_ORDERED
    , [&](int64_t i, int32_t r) { out[i] = r; }
#endif
    );
    VC_PEND();
}


// ---------------------------------------------------------------------------
// DNSServer's drain loop, one datagram per lane (DNSServer.java:457-500):
// securityGroup.allow(UDP, remote address, remote port) -> `read == 0`
// -> Formatter.parsePackets (Formatter.java:162-372: header, questions,
// answer / authority / additional resources with the A, AAAA, CNAME, PTR,
// TXT and SRV rdata checks) -> isResponse / opcode / handleRequest's
// per-question classification (DNSServer.java:116-166, dns_one).  The
// datagram is validated completely before any question is classified (a
// malformed packet anywhere makes parsePackets throw).  Shapes outside the
// kernel's contract come back VC_DNSD_HOST for the Java path: more than one
// packet in the datagram, more than VC_DNSD_MAXQ questions, a decoded qname
// over kNameCap bytes, a compression-pointer chain over kMaxPtr (Java
// recurses once per pointer; a pointer loop overflows its stack).
// ---------------------------------------------------------------------------
constexpr int kDnsdBlock = 128;
constexpr int kDnsdWaves = kDnsdBlock / 64;
// LDS per 128-thread workgroup: two 4 KiB stages (64 queries of up to 64 B
// on average per wave; longer spans are read from global memory).  The
// deferring kernel classifies each qname in place in the stage (dnsd_one);
// the others decode it into a per-lane buffer (kNameWords).
constexpr uint32_t kDnsdStage = 4096;
constexpr uint32_t kDnsdStageWords = (kDnsdStage + 2 * kApron) / 4;
constexpr int kNameCap = 128;                 // decoded qname chars classified (contract)
// Readable bytes around a qname: LdsSrc reads the aligned word pair that
// holds [pos, pos + 4) for pos in [-3, len + 3].
constexpr int kNameApron = 4;
// an odd stride in words: lane l's word k sits in bank (35 l + k) mod 64, so
// the lanes' buffers do not collide when they read the same word index
// (an even stride of 40 words put them on 8 banks)
constexpr int name_words(int cap) { return (cap + 2 * kNameApron) / 4 + 1; }
constexpr int kNameWords = name_words(kNameCap);
static_assert((kNameApron + kNameCap + 3) / 4 + 1 < kNameWords, "qname buffer too short");
static_assert(kNameWords & 1, "odd stride");
constexpr int kMaxPtr = 16;

enum : int { kNameOk = 0, kNameBad = 1, kNameHost = 2 };

// parse_name's output for a validation-only pass
struct NoOut {
    __device__ void operator()(int) const {}
};

// Formatter.parseDomainName over the datagram p[0, n): the name at index 0
// of the view [vs, vs + vlen) (vlen may be <= 0: SubByteArray takes a
// negative length and its first get throws).  Reads past the view are the
// ByteArray bounds exceptions parsePackets turns into a malformed packet; a
// pointer restarts in the view [o, n) of the whole datagram (rawPacket).
// *used = bytes of the view the name takes (offsetHolder[0]); out(b) gets
// the qname's chars ((char) b per label byte, '.' after each label).
template <class Out>
__device__ __forceinline__ int parse_name(const uint8_t* p, int n, int vs, int vlen, int* used,
                                          Out out) {
    int i = 0, len = 0, depth = 0;
    bool top = true;
    for (;;) {
        if (i >= vlen) return kNameBad;
        const int b = p[vs + i];
        if (len == 0) {
            if (b == 0) break;
            if ((b & 0xC0) == 0xC0) {                 // pointer: the rest of the name is there
                if (i + 1 >= vlen) return kNameBad;
                const int o = ((b & 0x3F) << 8) | p[vs + i + 1];
                if (top) *used = i + 2;
                top = false;
                if (++depth > kMaxPtr) return kNameHost;
                vs = o;
                vlen = n - o;
                i = 0;
                continue;
            }
            if constexpr (std::is_same_v<Out, NoOut>) {
                // validation only: a label's bytes matter only through the
                // bounds check each read makes, and the next length byte's
                // check fails whenever one of them would: jump over it
                i += b + 1;
                continue;
            }
            len = b;                                  // any other byte is a label length
        } else {
            out(b);
            if (--len == 0) out('.');
        }
        ++i;
    }
    if (top) *used = i + 1;
    return kNameOk;
}


__device__ __forceinline__ int be16(const uint8_t* p, int i) { return (p[i] << 8) | p[i + 1]; }

// DNSClass lookup (Formatter.parseClass): IN 1, CH 3, HS 4 anywhere; NONE
// 254 and ANY 255 in questions only; anything else throws.
__device__ __forceinline__ bool dns_class_ok(int c, bool question) {
    return c == 1 || c == 3 || c == 4 || (question && (c == 254 || c == 255));
}

// One resource record at `at` (Formatter.parseResource); the packet ends at
// n.  Returns the record's length, or -1 (malformed) / -2 (host).
__device__ __forceinline__ int dns_resource(const uint8_t* p, int n, int at) {
    int used = 0;
    const int r = parse_name(p, n, at, n - at, &used, NoOut{});
    if (r != kNameOk) return r == kNameBad ? -1 : -2;
    const int o = at + used;
    if (o + 10 > n) return -1;                        // type, class, ttl, rdlen
    const int type = be16(p, o), clazz = be16(p, o + 2), rdlen = be16(p, o + 8);
    if (type >= 252 && type <= 255) return -1;        // question-only types (DNSType)
    if (type != 41 && !dns_class_ok(clazz, false)) return -1;   // OPT: no class
    const int rd = o + 10;
    if (n - rd < rdlen) return -1;                    // data.sub(offset, rdlen)
    switch (type) {
    case 1:                                           // A
        if (rdlen != 4) return -1;
        break;
    case 28:                                          // AAAA
        if (rdlen != 16) return -1;
        break;
    case 5:                                           // CNAME
    case 12: {                                        // PTR
        int u = 0;
        const int q = parse_name(p, n, rd, rdlen, &u, NoOut{});
        if (q != kNameOk) return q == kNameBad ? -1 : -2;
        if (u != rdlen) return -1;
        break;
    }
    case 16: {                                        // TXT: length-prefixed strings, exactly
        int k = 0;
        while (k < rdlen) {
            const int l = p[rd + k];
            ++k;
            if (rdlen - k < l) return -1;
            k += l;
        }
        break;
    }
    case 33: {                                        // SRV: the target is parsed from
        int u = 0;                                    // rdata[6:] but its length compared
        const int q = parse_name(p, n, rd + 6, rdlen - 6, &u, NoOut{});   // with the whole
        if (q == kNameHost) return -2;                // rdata (SRV.java:27-36): never equal
        return -1;
    }
    default:
        break;
    }
    return rd + rdlen - at;
}

struct DnsdIn {
    const uint8_t* rfam;            // remote family per datagram (4/6), null = all IPv4
    const uint32_t* r4;
    const uint8_t* r6;              // 16 bytes per datagram, 16-byte aligned
    const uint16_t* rport;
};

// Per datagram: status; UDP rule; questions evaluated; per question (up to
// VC_DNSD_MAXQ) its qtype, VC_DNS_* kind and value.
struct DnsdOut {
    uint8_t* status;
    int32_t* acl;
    uint8_t* nq;
    uint16_t* qtype;
    uint8_t* kind;
    int32_t* value;
};

// status of a datagram the deferring dnsd kernel leaves to its second pass
constexpr uint8_t kDnsdDeferred = 0xFF;

// kDefer: a question dns_one<true> defers makes the whole datagram
// kDnsdDeferred (status only); dnsd_defer_kernel redoes it.  Returns the
// status written.
//
// kDefer also classifies in place: the datagram is this lane's own bytes in
// the wave's LDS stage (`name` = the stage, p at byte p_off of it).
// Formatter.parseDomainName's qname is the name's wire bytes after its first
// length byte with every later length byte and the terminating 0 read as
// '.' (a '.' after each label), so for a query of one question whose name
// holds no compression pointer -- a resolver's query -- those bytes are
// patched to '.' in the stage and the qname is searched where it lies: no
// byte-by-byte decode into a per-lane buffer, and no such buffer in the
// kernel's LDS.  Other shapes (several questions, a pointer) are deferred.
template <bool kDefer, int kCap = kNameCap>
__device__ __forceinline__ uint8_t dnsd_one(const HostsImage& hosts, const HintImage& img,
                                            const HintImage* slow_img, const AclImage& acl,
                                            const DnsdIn& in, const DnsdOut& out, int64_t i,
                                            const uint8_t* p, int n, uint32_t* name,
                                            int p_off = 0) {
    // securityGroup.allow(Protocol.UDP, remote.getAddress(), remote.getPort())
    const bool six = in.rfam && in.rfam[i] == 6;
    const uint32_t port = in.rport[i];
    uint32_t v;
#if defined(VC_ABL_NOACL)          // timing ablation only: no ACL search (default verdict)
    if (port != 0x7FFFFFFF) {
        v = VC_NONE;
    } else
#endif
    if (six) {
        uint64_t hi, lo;
        v6_key(reinterpret_cast<const uint4*>(in.r6)[i], &hi, &lo);
        v = acl6_global(acl.fam[1][1], acl.fam[1][0], hi, lo, port);
    } else {
        const AclFamilyImage& f = acl.fam[1][0];
        v = acl_value(f.rec, f.pieces, acl4_interval(f, in.r4[i]), port);
    }
    const bool allow = v == VC_NONE ? acl.default_allow != 0
                                    : glb_ld(acl.allow + acl.n_tcp + v) != 0;
    if (out.acl) out.acl[i] = out_index(v);
    int nq = 0;
    uint8_t st;
    auto put = [&](int q, int qtype, uint8_t kd, int32_t val) {
        const int64_t k = i * VC_DNSD_MAXQ + q;
        if (out.qtype) out.qtype[k] = uint16_t(qtype);
        out.kind[k] = kd;
        out.value[k] = val;
    };
    if (!allow) {
        st = VC_DNSD_REJECTED;
    } else if (n == 0) {
        st = VC_DNSD_EMPTY;
    } else if (n < 12) {
        st = VC_DNSD_MALFORMED;
    } else {
        // Formatter.parseHeader
        const int b2 = p[2], b3 = p[3];
        const int opcode = (b2 >> 3) & 15, rcode = b3 & 15;
        const int qd = be16(p, 4);
        const int nres = be16(p, 6) + be16(p, 8) + be16(p, 10);
        st = VC_DNSD_ANSWER;
        if (!(opcode <= 2 || (opcode >= 4 && opcode <= 6)) || rcode > 11) st = VC_DNSD_MALFORMED;
        // questions (Formatter.parseQuestion), then every resource
        int at = 12;
        for (int q = 0; q < qd && st == VC_DNSD_ANSWER; ++q) {
            int used = 0;
            const int r = parse_name(p, n, at, n - at, &used, NoOut{});
            if (r != kNameOk) {
                st = r == kNameBad ? VC_DNSD_MALFORMED : VC_DNSD_HOST;
                break;
            }
            at += used;
            if (at + 4 > n || !dns_class_ok(be16(p, at + 2), true)) st = VC_DNSD_MALFORMED;
            at += 4;
        }
        for (int k = 0; k < nres && st == VC_DNSD_ANSWER; ++k) {
            const int r = dns_resource(p, n, at);
            if (r < 0) st = r == -1 ? VC_DNSD_MALFORMED : VC_DNSD_HOST;
            else at += r;
        }
        if (st == VC_DNSD_ANSWER) {
            if (at != n) {
                st = VC_DNSD_HOST;                    // another packet follows (parsePackets loops)
            } else if (b2 & 0x80) {
                st = VC_DNSD_RESPONSE;                // p.isResponse: skipped
            } else if (opcode != 0) {
                st = VC_DNSD_RECURSIVE;               // runRecursive(p, remote)
            } else if (qd > VC_DNSD_MAXQ) {
                st = VC_DNSD_HOST;
            } else if (kDefer) {
                // one question, its name in place (see above)
                int j = 12;
                bool ptr = qd != 1;
                while (!ptr) {
                    const int b = p[j];
                    if ((b & 0xC0) == 0xC0) {
                        ptr = true;
                        break;
                    }
                    if (j > 12) const_cast<uint8_t*>(p)[j] = '.';
                    if (b == 0) break;
                    j += b + 1;
                }
                if (ptr) {
                    st = kDnsdDeferred;
                } else {
                    const int len = j - 12;           // the qname's chars, its last '.' included
                    const int qtype = be16(p, j + 1);
                    nq = 1;
                    if (qtype != 1 && qtype != 28 && qtype != 33) {   // not A / AAAA / SRV
                        put(0, qtype, VC_DNS_RECURSIVE, 0);
                        st = VC_DNSD_RECURSIVE;
                    } else if (len > kNameCap) {      // the Java path decides
                        st = VC_DNSD_HOST;
                        nq = 0;
                    } else {
                        uint8_t kd;
                        int32_t val;
                        dns_one<kDefer>(hosts, img, slow_img, LdsSrc{name, p_off + 13}, len, &kd,
                                        &val);
                        if (kd == kDnsDeferred) {
                            st = kDnsdDeferred;
                        } else {
                            put(0, qtype, kd, val);
                            if (kd == VC_DNS_RECURSIVE) st = VC_DNSD_RECURSIVE;
                        }
                    }
                }
            } else {
                // handleRequest: questions in order until one goes recursive
                at = 12;
                uint8_t* nb = reinterpret_cast<uint8_t*>(name) + kNameApron;
                for (int q = 0; q < qd; ++q) {
                    int used = 0, len = 0;
                    parse_name(p, n, at, n - at, &used, [&](int b) {
                        if (len < kCap) nb[len] = uint8_t(b);
                        ++len;
                    });
                    at += used;
                    const int qtype = be16(p, at);
                    at += 4;
                    nq = q + 1;
                    if (qtype != 1 && qtype != 28 && qtype != 33) {   // not A / AAAA / SRV
                        put(q, qtype, VC_DNS_RECURSIVE, 0);
                        st = VC_DNSD_RECURSIVE;
                        break;
                    }
                    if (len > kNameCap) {               // the Java path decides
                        st = VC_DNSD_HOST;
                        nq = 0;
                        break;
                    }
                    uint8_t kd;
                    int32_t val;
                    dns_one<kDefer>(hosts, img, slow_img, LdsSrc{name, kNameApron}, len, &kd, &val);
                    if (kDefer && kd == kDnsDeferred) {
                        st = kDnsdDeferred;
                        break;
                    }
                    put(q, qtype, kd, val);
                    if (kd == VC_DNS_RECURSIVE) {
                        st = VC_DNSD_RECURSIVE;
                        break;
                    }
                }
            }
        }
    }
    out.status[i] = st;
    if (kDefer && st == kDnsdDeferred) return st;
    if (out.nq) out.nq[i] = uint8_t(nq);
    for (int q = nq; q < VC_DNSD_MAXQ; ++q) out.kind[i * VC_DNSD_MAXQ + q] = 0;   // not evaluated
    return st;
}

// Minimum waves per SIMD of dnsd_kernel (the register budget it compiles
// to).  5 (96 VGPRs, no spills) since the qname is classified in place and
// the workgroup's LDS is 8 KiB: 1.55 -> 1.43 ms for the bench's 16.7M
// datagrams against 3 (98 VGPRs), interleaved on one box
// (profiles/r06_ab_dnsd_minw.jsonl).
#ifndef VC_DNSD_MINW
#define VC_DNSD_MINW 5
#endif
template <bool kStage, bool kDefer>
__global__ __launch_bounds__(kDnsdBlock, VC_DNSD_MINW) void dnsd_kernel(
    HostsImage hosts, HintImage img, AclImage acl, const uint8_t* __restrict__ blob,
    const uint32_t* __restrict__ off, int64_t n, DnsdIn in, DnsdOut out,
    uint32_t* __restrict__ ticket) {
    __shared__ uint32_t stage[kStage ? kDnsdWaves : 1][kStage ? kDnsdStageWords : 1];
    // kDefer classifies the qname in place in the stage: no per-lane buffer
    __shared__ uint32_t names[kDefer ? 1 : kDnsdBlock][kDefer ? 1 : kNameWords];
    const int lane = int(threadIdx.x & 63), w = int(threadIdx.x >> 6);
    HintImage slow_img = img;
    // 64-datagram chunks from the work tickets, or the static grid-stride
    // sequence without them.  16-chunk big tickets and two rounds of 4-chunk
    // tail tickets: the drain loop's chunks cost more than the other string
    // kernels', and their 24 / 8 / 1 layout ran it 3.99 against 3.94 ms
    // (profiles/r04_ab_ticket_confirm.txt); 60 % of the chunks static
    // (chunks.h ChunksT)
    ChunksT<16, 4, 2, 60> ch(ticket, (n + 63) / 64);
    int64_t c = ch.first(w);
    LaneSpan cur = c < ch.nchunks ? lane_span(off, c * 64, n) : LaneSpan{0, 0};
    while (c < ch.nchunks) {
        const int64_t base = c * 64;
        const int64_t i = base + lane;
        uint32_t o0, o1, a0 = 0;
        span_of(cur, base, n, &o0, &o1);
        const uint32_t a = cur.a, e = cur.e;
        const int64_t nx = ch.next(c);
        if (nx < ch.nchunks) cur = lane_span(off, nx * 64, n);             // next chunk's
        const bool staged = kStage && stage_wave<kDnsdStage>(blob, o0, o1, stage[w], &a0);
        uint8_t st = 0;
        if (i < n) {
            if (staged) {
                const int po = int(kApron + (a - a0));
                st = dnsd_one<kDefer>(hosts, img, &slow_img, acl, in, out, i,
                                      reinterpret_cast<const uint8_t*>(stage[w]) + po, int(e - a),
                                      kDefer ? stage[w] : names[threadIdx.x], po);
            } else if (kDefer) {
                st = kDnsdDeferred;
                out.status[i] = st;
            } else {
                st = dnsd_one<false>(hosts, img, &slow_img, acl, in, out, i, blob + a, int(e - a),
                                     names[threadIdx.x]);
            }
        }
        if (kDefer && ticket) {
            const uint64_t dm = __ballot(i < n && st == kDnsdDeferred);
            if (dm && lane == 0) atomicAdd(ticket + 1, uint32_t(__popcll(dm)));
        }
        if (kStage) wave_done();
        c = nx;
    }
}

// The datagrams dnsd_kernel<*, true> deferred, redone whole from global
// memory with the complete classification.  ctl as hint_defer_kernel's.
constexpr int kDnsdDeferBlock = 128;
__global__ __launch_bounds__(kDnsdDeferBlock) void dnsd_defer_kernel(
    HostsImage hosts, HintImage img, AclImage acl, const uint8_t* __restrict__ blob,
    const uint32_t* __restrict__ off, int64_t n, DnsdIn in, DnsdOut out, uint32_t* ctl) {
    __shared__ uint32_t names[kDnsdDeferBlock][kNameWords];
    __shared__ uint32_t todo;
    if (threadIdx.x == 0) todo = ctl ? __hip_atomic_load(ctl + 1, __ATOMIC_RELAXED,
                                                          __HIP_MEMORY_SCOPE_AGENT)
                                     : 1u;
    __syncthreads();
    if (todo) {
        for (int64_t i = int64_t(blockIdx.x) * blockDim.x + threadIdx.x; i < n;
             i += int64_t(gridDim.x) * blockDim.x) {
            if (out.status[i] != kDnsdDeferred) continue;
            const uint32_t a = off[i], e = off[i + 1];
            dnsd_one<false>(hosts, img, &img, acl, in, out, i, blob + a, int(e - a),
                            names[threadIdx.x]);
        }
    }
    if (ctl && threadIdx.x == 0 && atomicAdd(ctl + 2, 1u) == gridDim.x - 1) {
        atomicExch(ctl + 1, 0u);
        atomicExch(ctl + 2, 0u);
    }
}

}  // namespace vcd

namespace vc {

hipError_t launch_certs(const LaunchCfg& c, const CertImage& certs, const uint8_t* blob,
                        const uint32_t* off, const uint8_t* null, int64_t n, int32_t* out) {
    if (n <= 0) return hipSuccess;
    const int64_t want = (n + vcd::kHintBlock - 1) / vcd::kHintBlock;
    if ((reinterpret_cast<uintptr_t>(blob) & 3) == 0)
        hipLaunchKernelGGL(vcd::cert_kernel<true>,
                           dim3(resident_grid(c, reinterpret_cast<const void*>(vcd::cert_kernel<true>), vcd::kHintBlock, 0, want)),
                           dim3(vcd::kHintBlock), vcd::kProfLds, c.stream,
                           certs, blob, off, null, n, out, c.tickets ? c.tickets->next(c.stream) : nullptr);
    else
        hipLaunchKernelGGL(vcd::cert_kernel<false>,
                           dim3(resident_grid(c, reinterpret_cast<const void*>(vcd::cert_kernel<false>), vcd::kHintBlock, 0, want)),
                           dim3(vcd::kHintBlock), vcd::kProfLds, c.stream,
                           certs, blob, off, null, n, out, c.tickets ? c.tickets->next(c.stream) : nullptr);
    return hipGetLastError();
}

hipError_t launch_hint(const LaunchCfg& c, const HintImage& img, const uint8_t* host_blob,
                       const uint32_t* host_off, const uint8_t* host_null, const uint16_t* port,
                       const uint8_t* uri_blob, const uint32_t* uri_off, const uint8_t* uri_null,
                       int64_t n, int32_t* out, unsigned long long* counters) {
    if (n <= 0) return hipSuccess;
    const int64_t want = (n + vcd::kHintBlock - 1) / vcd::kHintBlock;
    const bool stage = host_blob && (reinterpret_cast<uintptr_t>(host_blob) & 3) == 0;
    // the deferring kernel whenever the names can be staged: uri lanes the
    // host levels do not decide go to the follow-up's general search
    const bool defer = VC_HINT_DEFER && stage;
    uint32_t* ticket = VC_HINT_TICKETS && c.tickets ? c.tickets->next(c.stream) : nullptr;
    auto go = [&](auto kernel) {
        hipLaunchKernelGGL(kernel,
                           dim3(resident_grid(c, reinterpret_cast<const void*>(kernel), vcd::kHintBlock, 0, want)),
                           dim3(vcd::kHintBlock), vcd::kProfLds, c.stream,
                           img, host_blob, host_off, host_null, port, uri_blob, uri_off, uri_null,
                           n, out, ticket);
    };
    const bool uri = uri_blob && img.has_uri_keys;
    if (defer && uri) go(vcd::hint_kernel<true, true, true>);
    else if (defer) go(vcd::hint_kernel<true, true>);
    else if (stage) go(vcd::hint_kernel<true, false>);
    else go(vcd::hint_kernel<false, false>);
    hipError_t e = hipGetLastError();
    if (e == hipSuccess && defer) {
        const int64_t dwant = (n + 255) / 256;
        // uri batches defer a few percent of their lanes to the general
        // search, a chain of dependent loads per lane: a resident grid
        // (C4uri: 24.8 ms on 128 workgroups)
        const int64_t dgrid =
            uri ? resident_grid(c, reinterpret_cast<const void*>(vcd::hint_defer_kernel), 256, 0,
                                dwant)
                : (dwant < VC_DEFER_GRID ? dwant : VC_DEFER_GRID);
        hipLaunchKernelGGL(vcd::hint_defer_kernel, dim3(unsigned(dgrid)), dim3(256), 0, c.stream,
                           img, host_blob, host_off, host_null, port, uri_blob, uri_off, uri_null,
                           n, out, ticket);
        e = hipGetLastError();
    }
    if (e != hipSuccess || !counters) return e;
    return launch_hist(c, VC_HIST_PLAIN, out, nullptr, n, img.n_groups, 0, img.n_groups, 0,
                       counters);
}

hipError_t launch_dns(const LaunchCfg& c, const HostsImage& hosts, const HintImage& hints,
                      const uint8_t* qblob, const uint32_t* qoff, int64_t n, uint8_t* kind,
                      int32_t* value, unsigned long long* group_counters) {
    if (n <= 0) return hipSuccess;
    const int64_t want = (n + vcd::kHintBlock - 1) / vcd::kHintBlock;
    const bool stage = (reinterpret_cast<uintptr_t>(qblob) & 3) == 0;
    const bool defer = VC_DNS_DEFER && stage;
    uint32_t* ticket = c.tickets ? c.tickets->next(c.stream) : nullptr;
    auto go = [&](auto kernel) {
        hipLaunchKernelGGL(kernel,
                           dim3(resident_grid(c, reinterpret_cast<const void*>(kernel), vcd::kHintBlock, 0, want)),
                           dim3(vcd::kHintBlock), vcd::kProfLds, c.stream,
                           hosts, hints, qblob, qoff, n, kind, value, ticket);
    };
    if (defer) go(vcd::dns_kernel<true, true>);
    else if (stage) go(vcd::dns_kernel<true, false>);
    else go(vcd::dns_kernel<false, false>);
    hipError_t e = hipGetLastError();
    if (e == hipSuccess && defer) {
        const int64_t dwant = (n + 255) / 256;
        const int64_t dgrid = dwant < VC_DEFER_GRID ? dwant : VC_DEFER_GRID;
        hipLaunchKernelGGL(vcd::dns_defer_kernel, dim3(unsigned(dgrid)), dim3(256), 0, c.stream,
                           hosts, hints, qblob, qoff, n, kind, value, ticket);
        e = hipGetLastError();
    }
    if (e != hipSuccess || !group_counters) return e;
    return launch_hist(c, VC_HIST_DNS, value, kind, n, hints.n_groups, 0, hints.n_groups, 0,
                       group_counters);
}

hipError_t launch_dns_datagrams(const LaunchCfg& c, const HostsImage& hosts,
                                const HintImage& hints, const AclImage& acl, const uint8_t* blob,
                                const uint32_t* off, int64_t n, const uint8_t* rfam,
                                const uint32_t* r4, const uint8_t* r6, const uint16_t* rport,
                                uint8_t* status, int32_t* out_acl, uint8_t* nq, uint16_t* qtype,
                                uint8_t* kind, int32_t* value) {
    if (n <= 0) return hipSuccess;
    const int64_t want = (n + vcd::kDnsdBlock - 1) / vcd::kDnsdBlock;
    const bool stage = (reinterpret_cast<uintptr_t>(blob) & 3) == 0;
    const bool defer = VC_DNS_DEFER && stage;
    const vcd::DnsdIn in{rfam, r4, r6, rport};
    const vcd::DnsdOut o{status, out_acl, nq, qtype, kind, value};
    uint32_t* tk = VC_DNSD_TICKETS && c.tickets ? c.tickets->next(c.stream) : nullptr;
    auto go = [&](auto kernel) {
        const int grid = resident_grid(c, reinterpret_cast<const void*>(kernel), vcd::kDnsdBlock,
                                       0, want);
        hipLaunchKernelGGL(kernel, dim3(grid), dim3(vcd::kDnsdBlock), 0, c.stream,
                           hosts, hints, acl, blob, off, n, in, o, tk);
    };
    if (defer) go(vcd::dnsd_kernel<true, true>);
    else if (stage) go(vcd::dnsd_kernel<true, false>);
    else go(vcd::dnsd_kernel<false, false>);
    hipError_t e = hipGetLastError();
    if (e == hipSuccess && defer) {
        const int64_t dwant = (n + vcd::kDnsdDeferBlock - 1) / vcd::kDnsdDeferBlock;
        const int64_t dgrid = dwant < VC_DEFER_GRID ? dwant : VC_DEFER_GRID;
        hipLaunchKernelGGL(vcd::dnsd_defer_kernel, dim3(unsigned(dgrid)), dim3(vcd::kDnsdDeferBlock),
                           0, c.stream, hosts, hints, acl, blob, off, n, in, o, tk);
        e = hipGetLastError();
    }
    return e;
}

}  // namespace vc

#if defined(VC_HINT_PROF)
// Profiling build only: read and clear the phase sums (not in vclassify.h).
extern "C" int vc_debug_hint_prof(unsigned long long* out) {
    unsigned long long z[vcd::kProfPhases + 1] = {};
    if (hipMemcpyFromSymbol(out, HIP_SYMBOL(vcd::vc_hint_prof), sizeof(z)) != hipSuccess) return -1;
    return hipMemcpyToSymbol(HIP_SYMBOL(vcd::vc_hint_prof), z, sizeof(z)) == hipSuccess ? 0 : -1;
}
#endif

VC_DEVCHECK_READER(hint)

#include "http_dev.h"

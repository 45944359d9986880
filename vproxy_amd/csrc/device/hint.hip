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
#include "hint_dev.h"
#include "launch.h"

namespace vcd {

constexpr int kHintBlock = 256;
constexpr int kWaves = kHintBlock / 64;
constexpr uint32_t kStageBytes = 4096;   // per wave: 64 names of up to 64 B on average

// A wave's 64 names are contiguous in the blob: copy them into LDS with
// coalesced dword loads once, so the per-lane character scans (reversed
// suffix hashing, key compares) read LDS instead of issuing scattered byte
// loads to HBM.  Returns the LDS base for this wave's names (names then sit
// at stage + (off[i] - a0)), or nullptr when the span does not fit.
__device__ __forceinline__ const uint8_t* stage_wave(const uint8_t* blob, uint32_t o0, uint32_t o1,
                                                     uint8_t* stage, uint32_t* a0_out) {
    const uint32_t a0 = o0 & ~3u;                  // blob is dword aligned (launcher checks)
    *a0_out = a0;
    if (o1 - a0 > kStageBytes) return nullptr;
    const int lane = int(threadIdx.x & 63);
    const uint32_t full = (o1 & ~3u) - a0;         // whole dwords inside [a0, o1)
    const uint32_t* gw = reinterpret_cast<const uint32_t*>(blob + a0);
    uint32_t* lw = reinterpret_cast<uint32_t*>(stage);
    for (uint32_t k = uint32_t(lane); k < full / 4; k += 64) lw[k] = gw[k];
    const uint32_t tail = o1 - (o1 & ~3u);
    if (uint32_t(lane) < tail) stage[full + lane] = blob[(o1 & ~3u) + lane];
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    return stage;
}

__device__ __forceinline__ void wave_done() {
    // every lane has finished reading the staged names before the next copy
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

template <bool kStage>
__global__ __launch_bounds__(kHintBlock) void hint_kernel(
    HintImage img, const uint8_t* __restrict__ host_blob, const uint32_t* __restrict__ host_off,
    const uint8_t* __restrict__ host_null, const uint16_t* __restrict__ port,
    const uint8_t* __restrict__ uri_blob, const uint32_t* __restrict__ uri_off,
    const uint8_t* __restrict__ uri_null, int64_t n, int32_t* __restrict__ out) {
    __shared__ __attribute__((aligned(16))) uint8_t stage[kWaves][kStageBytes];
    const int lane = int(threadIdx.x & 63), w = int(threadIdx.x >> 6);
    const int64_t wstride = int64_t(gridDim.x) * kWaves * 64;
    for (int64_t base = (int64_t(blockIdx.x) * kWaves + w) * 64; base < n; base += wstride) {
        const int64_t i = base + lane;
        const int64_t last = base + 64 < n ? base + 64 : n;
        const uint8_t* names = nullptr;
        uint32_t a0 = 0;
        if (kStage) names = stage_wave(host_blob, host_off[base], host_off[last], stage[w], &a0);
        if (i < n) {
            DStr h{nullptr, -1}, u{nullptr, -1};
            if (host_blob && !(host_null && host_null[i])) {
                const uint32_t a = host_off[i], e = host_off[i + 1];
                h = DStr{names ? names + (a - a0) : host_blob + a, int(e - a)};
            }
            if (uri_blob && !(uri_null && uri_null[i])) {
                const uint32_t a = uri_off[i], e = uri_off[i + 1];
                u = DStr{uri_blob + a, int(e - a)};
            }
            const int p = port ? int(port[i]) : 0;
            out[i] = search_for_group(img, format_host(h), p, format_uri(u));
        }
        if (kStage) wave_done();
    }
}

template <bool kStage>
__global__ __launch_bounds__(kHintBlock) void dns_kernel(
    HostsImage hosts, HintImage img, const uint8_t* __restrict__ qblob,
    const uint32_t* __restrict__ qoff, int64_t n, uint8_t* __restrict__ kind,
    int32_t* __restrict__ value) {
    __shared__ __attribute__((aligned(16))) uint8_t stage[kWaves][kStageBytes];
    const int lane = int(threadIdx.x & 63), w = int(threadIdx.x >> 6);
    const int64_t wstride = int64_t(gridDim.x) * kWaves * 64;
    for (int64_t base = (int64_t(blockIdx.x) * kWaves + w) * 64; base < n; base += wstride) {
        const int64_t i = base + lane;
        const int64_t last = base + 64 < n ? base + 64 : n;
        const uint8_t* names = nullptr;
        uint32_t a0 = 0;
        if (kStage) names = stage_wave(qblob, qoff[base], qoff[last], stage[w], &a0);
        if (i < n) {
            const uint32_t a = qoff[i], e = qoff[i + 1];
            const uint8_t* q = names ? names + (a - a0) : qblob + a;
            const int qn = int(e - a);
            // (1) hosts.get(qname) on the raw qname (trailing dot kept), :127
            uint32_t h = kFnvBasis;
            for (int j = 0; j < qn; ++j) h = fnv_step(h, q[j]);
            KeySlot k;
            int32_t g = -1;
            uint8_t kd;
            int32_t val = 0;
            if (hosts.n > 0 &&
                probe(hosts.tags, hosts.slots, hosts.mask, hosts.blob, h, q, qn, &k) >= 0) {
                kd = VC_DNS_HOSTS;
                val = k.a;
            } else {
                // (2) strip one trailing dot, :133-135
                const int dn = (qn > 0 && q[qn - 1] == '.') ? qn - 1 : qn;
                // (3) rrsets.searchForGroup(Hint.ofHost(domain)), :136
                g = hint_host_only(img, format_host(DStr{q, dn}), 0);
                if (g >= 0) {
                    kd = VC_DNS_GROUP;
                    val = g;
                } else if (d_is_ip_literal(q, dn)) {             // (4) IP literal, :140-149
                    kd = VC_DNS_IP_LITERAL;
                    val = d_count(q, dn, ':') ? 6 : 4;
                } else {                                          // (5) *.vproxy.local, :150-157
                    const char* sfx = ".vproxy.local";
                    bool internal = dn >= 13;
                    for (int j = 0; internal && j < 13; ++j)
                        internal = q[dn - 13 + j] == uint8_t(sfx[j]);
                    kd = internal ? VC_DNS_INTERNAL : VC_DNS_RECURSIVE;   // (6) :164
                }
            }
            kind[i] = kd;
            value[i] = val;
        }
        if (kStage) wave_done();
    }
}

}  // namespace vcd

namespace vc {

hipError_t launch_hint(const LaunchCfg& c, const HintImage& img, const uint8_t* host_blob,
                       const uint32_t* host_off, const uint8_t* host_null, const uint16_t* port,
                       const uint8_t* uri_blob, const uint32_t* uri_off, const uint8_t* uri_null,
                       int64_t n, int32_t* out, unsigned long long* counters) {
    if (n <= 0) return hipSuccess;
    int64_t want = (n + vcd::kHintBlock - 1) / vcd::kHintBlock;
    int64_t cap = int64_t(c.num_cus) * 8;
    int grid = int(want < cap ? want : cap);
    if (host_blob && (reinterpret_cast<uintptr_t>(host_blob) & 3) == 0)
        hipLaunchKernelGGL(vcd::hint_kernel<true>, dim3(grid), dim3(vcd::kHintBlock), 0, c.stream,
                           img, host_blob, host_off, host_null, port, uri_blob, uri_off, uri_null,
                           n, out);
    else
        hipLaunchKernelGGL(vcd::hint_kernel<false>, dim3(grid), dim3(vcd::kHintBlock), 0, c.stream,
                           img, host_blob, host_off, host_null, port, uri_blob, uri_off, uri_null,
                           n, out);
    hipError_t e = hipGetLastError();
    if (e != hipSuccess || !counters) return e;
    return launch_hist(c, VC_HIST_PLAIN, out, nullptr, n, img.n_groups, 0, img.n_groups, 0,
                       counters);
}

hipError_t launch_dns(const LaunchCfg& c, const HostsImage& hosts, const HintImage& hints,
                      const uint8_t* qblob, const uint32_t* qoff, int64_t n, uint8_t* kind,
                      int32_t* value, unsigned long long* group_counters) {
    if (n <= 0) return hipSuccess;
    int64_t want = (n + vcd::kHintBlock - 1) / vcd::kHintBlock;
    int64_t cap = int64_t(c.num_cus) * 8;
    int grid = int(want < cap ? want : cap);
    if ((reinterpret_cast<uintptr_t>(qblob) & 3) == 0)
        hipLaunchKernelGGL(vcd::dns_kernel<true>, dim3(grid), dim3(vcd::kHintBlock), 0, c.stream,
                           hosts, hints, qblob, qoff, n, kind, value);
    else
        hipLaunchKernelGGL(vcd::dns_kernel<false>, dim3(grid), dim3(vcd::kHintBlock), 0, c.stream,
                           hosts, hints, qblob, qoff, n, kind, value);
    hipError_t e = hipGetLastError();
    if (e != hipSuccess || !group_counters) return e;
    return launch_hist(c, VC_HIST_DNS, value, kind, n, hints.n_groups, 0, hints.n_groups, 0,
                       group_counters);
}

}  // namespace vc

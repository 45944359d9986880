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

__global__ __launch_bounds__(kHintBlock) void hint_kernel(
    HintImage img, const uint8_t* __restrict__ host_blob, const uint32_t* __restrict__ host_off,
    const uint8_t* __restrict__ host_null, const uint16_t* __restrict__ port,
    const uint8_t* __restrict__ uri_blob, const uint32_t* __restrict__ uri_off,
    const uint8_t* __restrict__ uri_null, int64_t n, int32_t* __restrict__ out) {
    const int64_t stride = int64_t(gridDim.x) * blockDim.x;
    for (int64_t i = int64_t(blockIdx.x) * blockDim.x + threadIdx.x; i < n; i += stride) {
        DStr h{nullptr, -1}, u{nullptr, -1};
        if (host_blob && !(host_null && host_null[i])) {
            const uint32_t a = host_off[i], e = host_off[i + 1];
            h = DStr{host_blob + a, int(e - a)};
        }
        if (uri_blob && !(uri_null && uri_null[i])) {
            const uint32_t a = uri_off[i], e = uri_off[i + 1];
            u = DStr{uri_blob + a, int(e - a)};
        }
        const int p = port ? int(port[i]) : 0;
        const int32_t g = search_for_group(img, format_host(h), p, format_uri(u));
        out[i] = g;
    }
}

__global__ __launch_bounds__(kHintBlock) void dns_kernel(
    HostsImage hosts, HintImage img, const uint8_t* __restrict__ qblob,
    const uint32_t* __restrict__ qoff, int64_t n, uint8_t* __restrict__ kind,
    int32_t* __restrict__ value) {
    const int64_t stride = int64_t(gridDim.x) * blockDim.x;
    for (int64_t i = int64_t(blockIdx.x) * blockDim.x + threadIdx.x; i < n; i += stride) {
        const uint32_t a = qoff[i], e = qoff[i + 1];
        const uint8_t* q = qblob + a;
        const int qn = int(e - a);
        // (1) hosts.get(qname) on the raw qname (trailing dot kept), :127
        uint64_t h = kFnvBasis;
        for (int j = 0; j < qn; ++j) h = fnv_step(h, q[j]);
        KeySlot k;
        if (hosts.n > 0 && probe(hosts.slots, hosts.mask, hosts.blob, h, q, qn, &k) >= 0) {
            kind[i] = VC_DNS_HOSTS;
            value[i] = k.a;
            continue;
        }
        // (2) strip one trailing dot, :133-135
        const int dn = (qn > 0 && q[qn - 1] == '.') ? qn - 1 : qn;
        // (3) rrsets.searchForGroup(Hint.ofHost(domain)), :136
        const int32_t g = hint_host_only(img, format_host(DStr{q, dn}), 0);
        if (g >= 0) {
            kind[i] = VC_DNS_GROUP;
            value[i] = g;
            continue;
        }
        // (4) IP literal, :140-149
        if (d_is_ip_literal(q, dn)) {
            kind[i] = VC_DNS_IP_LITERAL;
            value[i] = d_count(q, dn, ':') ? 6 : 4;
            continue;
        }
        // (5) *.vproxy.local, :150-157
        const char* sfx = ".vproxy.local";
        bool internal = dn >= 13;
        for (int j = 0; internal && j < 13; ++j) internal = q[dn - 13 + j] == uint8_t(sfx[j]);
        kind[i] = internal ? VC_DNS_INTERNAL : VC_DNS_RECURSIVE;   // (6) recursive, :164
        value[i] = 0;
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
    int64_t cap = int64_t(c.num_cus) * 16;
    int grid = int(want < cap ? want : cap);
    hipLaunchKernelGGL(vcd::hint_kernel, dim3(grid), dim3(vcd::kHintBlock), 0, c.stream, img,
                       host_blob, host_off, host_null, port, uri_blob, uri_off, uri_null, n, out);
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
    int64_t cap = int64_t(c.num_cus) * 16;
    int grid = int(want < cap ? want : cap);
    hipLaunchKernelGGL(vcd::dns_kernel, dim3(grid), dim3(vcd::kHintBlock), 0, c.stream, hosts,
                       hints, qblob, qoff, n, kind, value);
    hipError_t e = hipGetLastError();
    if (e != hipSuccess || !group_counters) return e;
    return launch_hist(c, VC_HIST_DNS, value, kind, n, hints.n_groups, 0, hints.n_groups, 0,
                       group_counters);
}

}  // namespace vc

// packet.hip -- batched header extraction (packet_dev.h): one lane per frame.
#include "acl_dev.h"
#include "launch.h"
#include "packet_dev.h"
#include "route_dev.h"
#include "chunks.h"
#include "stage.h"

namespace vcd {

constexpr int kPktBlock = 256;
constexpr int kPktWaves = kPktBlock / 64;
#ifndef VC_PKT_STAGE
#define VC_PKT_STAGE 7168
#endif
// per wave: 64 frames of up to 112 B on average.  LDS bounds the residency of
// these latency-bound kernels: 7 KiB gives 5 blocks per CU where 8 KiB gave
// 4 (switch 1.70 -> 1.47 ms); 6 KiB overflows on the benchmark's 100-B frames.
constexpr uint32_t kPktStage = VC_PKT_STAGE;
constexpr uint32_t kPktStageWords = (kPktStage + 2 * kApron) / 4;

__device__ __forceinline__ void store_pkt(const vc_pkt_out& out, int64_t i, const PktOut& o) {
    if (out.status) out.status[i] = o.status;
    if (out.l3) out.l3[i] = o.l3;
    if (out.l4) out.l4[i] = o.l4;
    if (out.proto) out.proto[i] = o.proto;
    if (out.vni) out.vni[i] = o.vni;
    if (out.ether_type) out.ether_type[i] = o.ether_type;
    if (out.sport) out.sport[i] = o.sport;
    if (out.dport) out.dport[i] = o.dport;
    const bool v4 = o.l3 == VC_L3_IPV4;
    if (out.src4) out.src4[i] = v4 ? bswap32(o.src[0]) : 0u;
    if (out.dst4) out.dst4[i] = v4 ? bswap32(o.dst[0]) : 0u;
    const bool v6 = o.l3 == VC_L3_IPV6;
    if (out.src6) {
        uint4 w = make_uint4(0, 0, 0, 0);
        if (v6) w = *reinterpret_cast<const uint4*>(o.src);
        reinterpret_cast<uint4*>(out.src6)[i] = w;
    }
    if (out.dst6) {
        uint4 w = make_uint4(0, 0, 0, 0);
        if (v6) w = *reinterpret_cast<const uint4*>(o.dst);
        reinterpret_cast<uint4*>(out.dst6)[i] = w;
    }
}

// kStage: the wave's 64 frames are copied into LDS with coalesced dword
// loads (stage.h) and parsed from there; a per-lane parse from global
// memory issues one scattered byte load per header byte.  Waves whose
// frames do not fit the stage parse from global memory.
template <bool kStage>
__global__ __launch_bounds__(kPktBlock) void packet_kernel(
    const uint8_t* __restrict__ blob, const uint32_t* __restrict__ off, int64_t n, int layer,
    vc_pkt_out out, uint32_t* __restrict__ ticket) {
    __shared__ uint32_t stage[kStage ? kPktWaves : 1][kStage ? kPktStageWords : 1];
    const int lane = int(threadIdx.x & 63), w = int(threadIdx.x >> 6);
    Chunks ch(ticket, (n + 63) / 64);              // chunks.h: work tickets or static
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
        const bool staged = kStage && stage_wave<kPktStage>(blob, o0, o1, stage[w], &a0);
        if (i < n) {
            PktOut o;
            if (staged) {
                const uint8_t* lp = reinterpret_cast<const uint8_t*>(stage[w]) + kApron + (a - a0);
                parse_packet(lp, int(e - a), layer, &o);
            } else {
                parse_packet(blob + a, int(e - a), layer, &o);
            }
            store_pkt(out, i, o);
        }
        if (kStage) wave_done();
        c = nx;
    }
}

// ---------------------------------------------------------------------------
// Switch.PacketHandler.readable's per-datagram chain in one pass
// (core/src/main/java/vswitch/Switch.java:679-700, 744-776, L3.java:423-444):
// bareVXLanAccess.allow(UDP, remote, vxlanBindingAddress.port) on the outer
// sender, VXLanPacket.from on the payload, and RouteTable.lookup(dst) of the
// inner IPv4/IPv6 packet -- the parse results stay in registers, no SoA
// round trip through HBM between the three.
// ---------------------------------------------------------------------------
struct SwitchIn {
    const uint8_t* rfam;            // remote family per datagram (4/6), null = all IPv4
    const uint32_t* r4;
    const uint8_t* r6;              // 16 bytes per datagram, 16-byte aligned
    uint32_t bind_port;
};

struct SwitchOut {
    int32_t* acl;
    uint8_t* allow;
    int32_t* route;
};

// The route image of `vni` (Switch.java:562 tables.get(vni)): a binary
// search over the compiled VNIs (a few dozen words, L2-resident), or null.
__device__ __forceinline__ const RouteImage* vni_table(const VniImage& vt, uint32_t vni) {
    int lo = 0, len = vt.n;
    while (len > 1) {
        const int half = len >> 1;
        lo = glb_ld(vt.vni + lo + half) <= vni ? lo + half : lo;
        len -= half;
    }
    return glb_ld(vt.vni + lo) == vni ? vt.tables + lo : nullptr;
}

#ifndef VC_SWITCH_PRELOAD
#define VC_SWITCH_PRELOAD 1
#endif
// pb / pv / pnb: the UDP list's IPv4 image at the bind port, staged in LDS
// (images.h AclPortImage), or pnb == 0 for the general image.
__device__ __forceinline__ void switch_one(const AclImage& acl, const RouteImage& rt,
                                           const VniImage& vt, const SwitchIn& in, int64_t i,
                                           const PktOut& o, const SwitchOut& so,
                                           const uint32_t* pb, const uint32_t* pv, int pnb) {
    // one table (no VNI map) and an IPv4 inner packet: its route's root
    // entry is loaded first, so that gather (into a table of up to 64 MB)
    // is in flight during the ACL's dependent loads instead of after them
    const bool pre = VC_SWITCH_PRELOAD && vt.n == 0 && o.status == VC_PKT_OK && o.l3 == VC_L3_IPV4;
    const uint32_t k4 = bswap32(o.dst[0]);
    uint32_t e0 = 0;
    if (pre) e0 = glb_ld(rt.fam[0].nodes + (k4 >> (32 - rt.fam[0].root_bits)));
    // SecurityGroup.allow(Protocol.UDP, remote, port): the UDP list
    const bool six = in.rfam && in.rfam[i] == 6;
    uint32_t v;
    if (six) {
        uint64_t hi, lo;
        v6_key(reinterpret_cast<const uint4*>(in.r6)[i], &hi, &lo);
        v = acl6_global(acl.fam[1][1], acl.fam[1][0], hi, lo, in.bind_port);
    } else if (pnb) {
        v = lds_ld(pv + bsearch_u32<true>(pb, pnb, in.r4[i]));
    } else {
        const AclFamilyImage& f = acl.fam[1][0];
        v = acl_value(f.rec, f.pieces, acl4_interval(f, in.r4[i]), in.bind_port);
    }
    const bool allow = v == VC_NONE ? acl.default_allow != 0 : acl.allow[acl.n_tcp + v] != 0;
    if (so.acl) so.acl[i] = out_index(v);
    if (so.allow) so.allow[i] = allow ? 1 : 0;
    // the inner packet's route in the table of its VNI, for allowed
    // datagrams that parsed
    int32_t r = -1;
    if (allow && o.status == VC_PKT_OK) {
        TrieImage t4 = rt.fam[0], t6 = rt.fam[1];
        bool have = true;
        if (vt.n > 0) {
            const RouteImage* tb = vni_table(vt, o.vni);
            have = tb != nullptr;
            if (have) {
                t4.nodes = glb_ld(&tb->fam[0].nodes);
                t4.root_bits = glb_ld(&tb->fam[0].root_bits);
                t6.nodes = glb_ld(&tb->fam[1].nodes);
                t6.root_bits = glb_ld(&tb->fam[1].root_bits);
            }
        }
        if (!have) {
            r = VC_SWITCH_NO_TABLE;                   // inputVXLan: vni not defined, drop
        } else if (pre) {
            r = out_index(trie_v4_from(t4.nodes, t4.root_bits, k4, e0));
        } else if (o.l3 == VC_L3_IPV4) {
            r = out_index(trie_v4(t4.nodes, t4.root_bits, k4));
        } else if (o.l3 == VC_L3_IPV6) {
            uint64_t hi, lo;
            v6_key(*reinterpret_cast<const uint4*>(o.dst), &hi, &lo);
            r = out_index(trie_v6(t6.nodes, t6.root_bits, hi, lo));
        }
    }
    so.route[i] = r;
}

// kPort: the bind port's AclPortImage (at most kSwitchPortMax intervals)
// copied into LDS first; the sender's UDP rule is then one LDS search.
constexpr int kSwitchPortMax = 256;
template <bool kStage, bool kPort>
__global__ __launch_bounds__(kPktBlock) void switch_kernel(
    const uint8_t* __restrict__ blob, const uint32_t* __restrict__ off, int64_t n, int layer,
    vc_pkt_out out, AclImage acl, RouteImage rt, VniImage vt, SwitchIn in, SwitchOut so,
    AclPortImage ap, uint32_t* __restrict__ ticket) {
    __shared__ uint32_t stage[kStage ? kPktWaves : 1][kStage ? kPktStageWords : 1];
    __shared__ uint32_t pb[kPort ? kSwitchPortMax : 1], pv[kPort ? kSwitchPortMax : 1];
    const int lane = int(threadIdx.x & 63), w = int(threadIdx.x >> 6);
    if (kPort) {
        for (int t = int(threadIdx.x); t < ap.nb; t += kPktBlock) {
            pb[t] = glb_ld(ap.bounds + t);
            pv[t] = glb_ld(ap.value + t);
        }
        __syncthreads();
    }
    Chunks ch(ticket, (n + 63) / 64);              // chunks.h: work tickets or static
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
        const bool staged = kStage && stage_wave<kPktStage>(blob, o0, o1, stage[w], &a0);
        if (i < n) {
            PktOut o;
            if (staged) {
                const uint8_t* lp = reinterpret_cast<const uint8_t*>(stage[w]) + kApron + (a - a0);
                parse_packet(lp, int(e - a), layer, &o);
            } else {
                parse_packet(blob + a, int(e - a), layer, &o);
            }
            store_pkt(out, i, o);
            switch_one(acl, rt, vt, in, i, o, so, pb, pv, kPort ? ap.nb : 0);
        }
        if (kStage) wave_done();
        c = nx;
    }
}

}  // namespace vcd

namespace vc {

// The parse and switch kernels keep the static grid-stride split (a null
// ticket): their per-frame cost is even, and work tickets made them 3-5 %
// slower, while the mirror kernel, whose cost varies with the filters a frame
// reaches, gained 16 % from them (profiles/r03_ab_frame_tickets.txt).
hipError_t launch_switch(const LaunchCfg& c, const AclImage& acl, const RouteImage& rt,
                         const VniImage& vt, const uint8_t* blob, const uint32_t* off, int64_t n, int layer,
                         const vc_pkt_out& out, const uint8_t* rfam, const uint32_t* r4,
                         const uint8_t* r6, int bind_port, const AclPortImage& ap,
                         int32_t* out_acl, uint8_t* out_allow, int32_t* out_route) {
    if (n <= 0) return hipSuccess;
    const int64_t want = (n + vcd::kPktBlock - 1) / vcd::kPktBlock;
    const bool stage = (reinterpret_cast<uintptr_t>(blob) & 3) == 0;
    const bool port = stage && ap.nb > 0 && ap.nb <= vcd::kSwitchPortMax &&
                      ap.port == bind_port;
    const vcd::SwitchIn in{rfam, r4, r6, uint32_t(bind_port)};
    const vcd::SwitchOut so{out_acl, out_allow, out_route};
    auto go = [&](auto kernel) {
        const int grid = resident_grid(c, reinterpret_cast<const void*>(kernel), vcd::kPktBlock,
                                       0, want);
        hipLaunchKernelGGL(kernel, dim3(grid), dim3(vcd::kPktBlock), 0, c.stream, blob, off, n,
                           layer, out, acl, rt, vt, in, so, ap, nullptr);
    };
    if (port) go(vcd::switch_kernel<true, true>);
    else if (stage) go(vcd::switch_kernel<true, false>);
    else go(vcd::switch_kernel<false, false>);
    return hipGetLastError();
}

hipError_t launch_packets(const LaunchCfg& c, const uint8_t* blob, const uint32_t* off, int64_t n,
                          int layer, const vc_pkt_out& out) {
    if (n <= 0) return hipSuccess;
    const int64_t want = (n + vcd::kPktBlock - 1) / vcd::kPktBlock;
    const bool stage = (reinterpret_cast<uintptr_t>(blob) & 3) == 0;
    const void* k = stage ? reinterpret_cast<const void*>(vcd::packet_kernel<true>)
                          : reinterpret_cast<const void*>(vcd::packet_kernel<false>);
    const int grid = resident_grid(c, k, vcd::kPktBlock, 0, want);
    if (stage)
        hipLaunchKernelGGL(vcd::packet_kernel<true>, dim3(grid), dim3(vcd::kPktBlock), 0, c.stream,
                           blob, off, n, layer, out, nullptr);
    else
        hipLaunchKernelGGL(vcd::packet_kernel<false>, dim3(grid), dim3(vcd::kPktBlock), 0,
                           c.stream, blob, off, n, layer, out, nullptr);
    return hipGetLastError();
}

}  // namespace vc

VC_DEVCHECK_READER(packet)

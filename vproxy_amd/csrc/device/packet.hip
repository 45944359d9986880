// packet.hip -- batched header extraction (packet_dev.h): one lane per frame.
#include "launch.h"
#include "packet_dev.h"
#include "stage.h"

namespace vcd {

constexpr int kPktBlock = 256;
constexpr int kPktWaves = kPktBlock / 64;
constexpr uint32_t kPktStage = 8192;     // per wave: 64 frames of up to 128 B on average
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
    if (out.src4) out.src4[i] = v4 ? (uint32_t(o.src[0]) << 24 | uint32_t(o.src[1]) << 16 |
                                      uint32_t(o.src[2]) << 8 | o.src[3]) : 0u;
    if (out.dst4) out.dst4[i] = v4 ? (uint32_t(o.dst[0]) << 24 | uint32_t(o.dst[1]) << 16 |
                                      uint32_t(o.dst[2]) << 8 | o.dst[3]) : 0u;
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
    vc_pkt_out out) {
    __shared__ uint32_t stage[kStage ? kPktWaves : 1][kStage ? kPktStageWords : 1];
    const int lane = int(threadIdx.x & 63), w = int(threadIdx.x >> 6);
    const int64_t wstride = int64_t(gridDim.x) * kPktWaves * 64;
    for (int64_t base = (int64_t(blockIdx.x) * kPktWaves + w) * 64; base < n; base += wstride) {
        const int64_t i = base + lane;
        const int64_t last = base + 64 < n ? base + 64 : n;
        uint32_t a0 = 0;
        const bool staged =
            kStage && stage_wave<kPktStage>(blob, off[base], off[last], stage[w], &a0);
        if (i < n) {
            const uint32_t a = off[i], e = off[i + 1];
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
    }
}

}  // namespace vcd

namespace vc {

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
                           blob, off, n, layer, out);
    else
        hipLaunchKernelGGL(vcd::packet_kernel<false>, dim3(grid), dim3(vcd::kPktBlock), 0,
                           c.stream, blob, off, n, layer, out);
    return hipGetLastError();
}

}  // namespace vc

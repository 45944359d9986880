// packet.hip -- batched header extraction (packet_dev.h): one lane per frame.
#include "launch.h"
#include "packet_dev.h"

namespace vcd {

constexpr int kPktBlock = 256;

__global__ __launch_bounds__(kPktBlock) void packet_kernel(
    const uint8_t* __restrict__ blob, const uint32_t* __restrict__ off, int64_t n, int layer,
    vc_pkt_out out) {
    const int64_t stride = int64_t(gridDim.x) * blockDim.x;
    for (int64_t i = int64_t(blockIdx.x) * blockDim.x + threadIdx.x; i < n; i += stride) {
        const uint32_t a = off[i], e = off[i + 1];
        PktOut o;
        parse_packet(blob + a, int(e - a), layer, &o);
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
}

}  // namespace vcd

namespace vc {

hipError_t launch_packets(const LaunchCfg& c, const uint8_t* blob, const uint32_t* off, int64_t n,
                          int layer, const vc_pkt_out& out) {
    if (n <= 0) return hipSuccess;
    const int64_t want = (n + vcd::kPktBlock - 1) / vcd::kPktBlock;
    const int64_t cap = int64_t(c.num_cus) * 8;
    hipLaunchKernelGGL(vcd::packet_kernel, dim3(int(want < cap ? want : cap)), dim3(vcd::kPktBlock),
                       0, c.stream, blob, off, n, layer, out);
    return hipGetLastError();
}

}  // namespace vc

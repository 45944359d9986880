// select.hip -- ServerGroup.next(source) for method == source, batched.
//
//   SOURCE.hash       base/.../component/svrgroup/ServerGroup.java:387-397
//   sourceHashGet     ServerGroup.java:464-490
//   sourceReset       ServerGroup.java:620-664 (host side: compile.cpp)
//
// Per item: the sdbm hash of the client address bytes (Java int arithmetic
// on sign-extended bytes), then one read of the list's pick table at
// hash % size -- the first healthy server from there on, which is where the
// Java recursion's forward probe ends (images.h ServerImage.pick).  IPv4:
// four items per lane.
#include "dev_common.h"
#include "launch.h"

namespace vcd {

constexpr int kSelBlock = 256;
#ifndef VC_SOURCE_VEC
#define VC_SOURCE_VEC 1
#endif

// sdbm over the address bytes, Math.abs, MIN_VALUE -> 0
__device__ __forceinline__ int32_t sdbm_step(uint32_t h, uint32_t byte) {
    const uint32_t b = uint32_t(int32_t(int8_t(uint8_t(byte))));
    return int32_t(b + (h << 6) + (h << 16) - h);
}

__device__ __forceinline__ int32_t java_abs_hash(int32_t h) {
    if (h == INT32_MIN) return 0;
    return h < 0 ? -h : h;
}

// sourceHashGet (ServerGroup.java:479-490) through the per-position table:
// idx = hash % size, then the first healthy server from idx on, cyclically
// (ServerImage.pick).  hash >= 0 (Math.abs), so the modulo is unsigned.
__device__ __forceinline__ int32_t source_pick(const ServerImage& img, int32_t g, int view,
                                               int32_t hash) {
    if (g < 0 || g >= img.n_groups) return -1;
    const uint2 vo = reinterpret_cast<const uint2*>(img.view_off)[g * 3 + view];
    if (vo.y == 0) return -1;                                // :480 empty list
    return img.pick[vo.x + uint32_t(hash) % vo.y];
}

__device__ __forceinline__ int32_t sdbm_v4(uint32_t a) {     // IP.ipv4Bytes2Int order
    uint32_t h = 0;
    h = uint32_t(sdbm_step(h, a >> 24));
    h = uint32_t(sdbm_step(h, (a >> 16) & 255u));
    h = uint32_t(sdbm_step(h, (a >> 8) & 255u));
    h = uint32_t(sdbm_step(h, a & 255u));
    return java_abs_hash(int32_t(h));
}

// kVec: four items per lane per step (16-byte group / address / result
// accesses), so a lane has four table probes in flight; the n % 4 tail is
// done by block 0.  Otherwise one item per lane (unaligned arrays).
template <bool kVec>
__global__ __launch_bounds__(kSelBlock) void source_v4_kernel(
    ServerImage img, const int32_t* __restrict__ group, const uint32_t* __restrict__ src4,
    int64_t n, int view, int32_t* __restrict__ out) {
    const int64_t stride = int64_t(gridDim.x) * blockDim.x;
    const int64_t first = int64_t(blockIdx.x) * blockDim.x + threadIdx.x;
    if (kVec) {
        const int64_t n4 = n >> 2;
        for (int64_t i = first; i < n4; i += stride) {
            const int4 g = reinterpret_cast<const int4*>(group)[i];
            const uint4 a = reinterpret_cast<const uint4*>(src4)[i];
            int4 o;
            o.x = source_pick(img, g.x, view, sdbm_v4(a.x));
            o.y = source_pick(img, g.y, view, sdbm_v4(a.y));
            o.z = source_pick(img, g.z, view, sdbm_v4(a.z));
            o.w = source_pick(img, g.w, view, sdbm_v4(a.w));
            reinterpret_cast<int4*>(out)[i] = o;
        }
        if (blockIdx.x == 0 && threadIdx.x < (n & 3)) {
            const int64_t i = (n4 << 2) + threadIdx.x;
            out[i] = source_pick(img, group[i], view, sdbm_v4(src4[i]));
        }
        return;
    }
    for (int64_t i = first; i < n; i += stride)
        out[i] = source_pick(img, group[i], view, sdbm_v4(src4[i]));
}

__global__ __launch_bounds__(kSelBlock) void source_v6_kernel(
    ServerImage img, const int32_t* __restrict__ group, const uint8_t* __restrict__ src6,
    int64_t n, int view, int32_t* __restrict__ out) {
    const int64_t stride = int64_t(gridDim.x) * blockDim.x;
    for (int64_t i = int64_t(blockIdx.x) * blockDim.x + threadIdx.x; i < n; i += stride) {
        const uint4 w = reinterpret_cast<const uint4*>(src6)[i];
        const uint32_t words[4] = {w.x, w.y, w.z, w.w};
        uint32_t h = 0;
#pragma unroll
        for (int k = 0; k < 4; ++k)
#pragma unroll
            for (int b = 0; b < 4; ++b) h = uint32_t(sdbm_step(h, (words[k] >> (8 * b)) & 255u));
        out[i] = source_pick(img, group[i], view, java_abs_hash(int32_t(h)));
    }
}

}  // namespace vcd

namespace vc {

hipError_t launch_source(const LaunchCfg& c, const ServerImage& img, const int32_t* group,
                         const void* src, int family, int64_t n, int view, int32_t* out) {
    if (n <= 0) return hipSuccess;
    const int vi = view == VC_SOURCE_IPV4 ? 1 : (view == VC_SOURCE_IPV6 ? 2 : 0);
    const bool vec = family == 4 && VC_SOURCE_VEC && ((reinterpret_cast<uintptr_t>(group) |
                                                       reinterpret_cast<uintptr_t>(src) |
                                                       reinterpret_cast<uintptr_t>(out)) & 15) == 0;
    const int64_t items = vec ? (n + 3) / 4 : n;
    const int64_t want = (items + vcd::kSelBlock - 1) / vcd::kSelBlock;
    const void* kern = family == 4 ? (vec ? reinterpret_cast<const void*>(vcd::source_v4_kernel<true>)
                                          : reinterpret_cast<const void*>(vcd::source_v4_kernel<false>))
                                   : reinterpret_cast<const void*>(vcd::source_v6_kernel);
    const int grid = resident_grid(c, kern, vcd::kSelBlock, 0, want);
    if (family == 4 && vec)
        hipLaunchKernelGGL(vcd::source_v4_kernel<true>, dim3(grid), dim3(vcd::kSelBlock), 0, c.stream,
                           img, group, static_cast<const uint32_t*>(src), n, vi, out);
    else if (family == 4)
        hipLaunchKernelGGL(vcd::source_v4_kernel<false>, dim3(grid), dim3(vcd::kSelBlock), 0,
                           c.stream, img, group, static_cast<const uint32_t*>(src), n, vi, out);
    else
        hipLaunchKernelGGL(vcd::source_v6_kernel, dim3(grid), dim3(vcd::kSelBlock), 0, c.stream, img,
                           group, static_cast<const uint8_t*>(src), n, vi, out);
    return hipGetLastError();
}

}  // namespace vc

VC_DEVCHECK_READER(select)

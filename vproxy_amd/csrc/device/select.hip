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

#ifndef VC_SEL_BLOCK
#define VC_SEL_BLOCK 256
#endif
constexpr int kSelBlock = VC_SEL_BLOCK;
constexpr size_t kSelLdsMax = 40 * 1024;   // the LDS copy of a view's lists, at most
#ifndef VC_SOURCE_VEC
#define VC_SOURCE_VEC 1
#endif
#ifndef VC_SOURCE_LDS
#define VC_SOURCE_LDS 1
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
__device__ __forceinline__ int32_t pick_at(const ServerImage& img, uint32_t off, uint32_t cnt,
                                           int32_t hash) {
    if (cnt == 0) return -1;                                 // :480 empty list
    return img.pick[off + uint32_t(hash) % cnt];
}

// kLds: the launch's view of ServerImage.view_pk is copied into LDS once per
// workgroup, so an item's list (offset, count) is an LDS read and its pick
// the one L2 gather left (from the global view_off: two dependent gathers)
template <bool kLds>
struct Lists {
    const ServerImage& img;
    const uint32_t* pk;                                      // LDS, kLds
    int view;
    __device__ __forceinline__ int32_t operator()(int32_t g, int32_t hash) const {
        if (g < 0 || g >= img.n_groups) return -1;
        if constexpr (kLds) {
            const uint32_t w = pk[g];
            return pick_at(img, w >> 8, w & 255u, hash);
        } else {
            const uint2 vo = reinterpret_cast<const uint2*>(img.view_off)[g * 3 + view];
            return pick_at(img, vo.x, vo.y, hash);
        }
    }
};

template <bool kLds>
__device__ __forceinline__ Lists<kLds> lists_of(const ServerImage& img, int view, uint32_t* lds) {
    if constexpr (kLds) {
        const uint32_t* src = img.view_pk + int64_t(view) * img.n_groups;
        for (int k = threadIdx.x; k < img.n_groups; k += blockDim.x) lds[k] = src[k];
        __syncthreads();
    }
    return Lists<kLds>{img, lds, view};
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
template <bool kVec, bool kLds>
__global__ __launch_bounds__(kSelBlock) void source_v4_kernel(
    ServerImage img, const int32_t* __restrict__ group, const uint32_t* __restrict__ src4,
    int64_t n, int view, int32_t* __restrict__ out) {
    extern __shared__ uint32_t vpk[];
    const auto pick = lists_of<kLds>(img, view, vpk);
    const int64_t stride = int64_t(gridDim.x) * blockDim.x;
    const int64_t first = int64_t(blockIdx.x) * blockDim.x + threadIdx.x;
    if (kVec) {
        const int64_t n4 = n >> 2;
        for (int64_t i = first; i < n4; i += stride) {
            const int4 g = reinterpret_cast<const int4*>(group)[i];
            const uint4 a = reinterpret_cast<const uint4*>(src4)[i];
            int4 o;
            o.x = pick(g.x, sdbm_v4(a.x));
            o.y = pick(g.y, sdbm_v4(a.y));
            o.z = pick(g.z, sdbm_v4(a.z));
            o.w = pick(g.w, sdbm_v4(a.w));
            reinterpret_cast<int4*>(out)[i] = o;
        }
        if (blockIdx.x == 0 && threadIdx.x < (n & 3)) {
            const int64_t i = (n4 << 2) + threadIdx.x;
            out[i] = pick(group[i], sdbm_v4(src4[i]));
        }
        return;
    }
    for (int64_t i = first; i < n; i += stride)
        out[i] = pick(group[i], sdbm_v4(src4[i]));
}

template <bool kLds>
__global__ __launch_bounds__(kSelBlock) void source_v6_kernel(
    ServerImage img, const int32_t* __restrict__ group, const uint8_t* __restrict__ src6,
    int64_t n, int view, int32_t* __restrict__ out) {
    extern __shared__ uint32_t vpk[];
    const auto pick = lists_of<kLds>(img, view, vpk);
    const int64_t stride = int64_t(gridDim.x) * blockDim.x;
    for (int64_t i = int64_t(blockIdx.x) * blockDim.x + threadIdx.x; i < n; i += stride) {
        const uint4 w = reinterpret_cast<const uint4*>(src6)[i];
        const uint32_t words[4] = {w.x, w.y, w.z, w.w};
        uint32_t h = 0;
#pragma unroll
        for (int k = 0; k < 4; ++k)
#pragma unroll
            for (int b = 0; b < 4; ++b) h = uint32_t(sdbm_step(h, (words[k] >> (8 * b)) & 255u));
        out[i] = pick(group[i], java_abs_hash(int32_t(h)));
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
    // the view's lists in LDS when they fit a quarter of it (VC_SOURCE_LDS=0: the global table)
    const size_t lds = size_t(img.n_groups) * 4;
    const bool use_lds = VC_SOURCE_LDS && img.pk_ok && img.view_pk && img.n_groups > 0 &&
                         lds <= vcd::kSelLdsMax;
    const int64_t items = vec ? (n + 3) / 4 : n;
    const int64_t want = (items + vcd::kSelBlock - 1) / vcd::kSelBlock;
    const void* kern;
    if (family == 4)
        kern = vec ? (use_lds ? reinterpret_cast<const void*>(vcd::source_v4_kernel<true, true>)
                              : reinterpret_cast<const void*>(vcd::source_v4_kernel<true, false>))
                   : (use_lds ? reinterpret_cast<const void*>(vcd::source_v4_kernel<false, true>)
                              : reinterpret_cast<const void*>(vcd::source_v4_kernel<false, false>));
    else
        kern = use_lds ? reinterpret_cast<const void*>(vcd::source_v6_kernel<true>)
                       : reinterpret_cast<const void*>(vcd::source_v6_kernel<false>);
    const size_t shmem = use_lds ? lds : 0;
    const int grid = resident_grid(c, kern, vcd::kSelBlock, shmem, want);
    const auto* s4 = static_cast<const uint32_t*>(src);
    const auto* s6 = static_cast<const uint8_t*>(src);
    const dim3 g(grid), b(vcd::kSelBlock);
    if (family == 4 && vec && use_lds)
        hipLaunchKernelGGL((vcd::source_v4_kernel<true, true>), g, b, shmem, c.stream, img, group, s4, n, vi, out);
    else if (family == 4 && vec)
        hipLaunchKernelGGL((vcd::source_v4_kernel<true, false>), g, b, shmem, c.stream, img, group, s4, n, vi, out);
    else if (family == 4 && use_lds)
        hipLaunchKernelGGL((vcd::source_v4_kernel<false, true>), g, b, shmem, c.stream, img, group, s4, n, vi, out);
    else if (family == 4)
        hipLaunchKernelGGL((vcd::source_v4_kernel<false, false>), g, b, shmem, c.stream, img, group, s4, n, vi, out);
    else if (use_lds)
        hipLaunchKernelGGL(vcd::source_v6_kernel<true>, g, b, shmem, c.stream, img, group, s6, n, vi, out);
    else
        hipLaunchKernelGGL(vcd::source_v6_kernel<false>, g, b, shmem, c.stream, img, group, s6, n, vi, out);
    return hipGetLastError();
}

}  // namespace vc

VC_DEVCHECK_READER(select)

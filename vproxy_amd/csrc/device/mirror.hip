// mirror.hip -- traffic-mirror filter kernels (see mirror_dev.h).
//
// One lane per item.  The filter list is small and read by every lane of a
// wave at the same address (uniform loop), so it stays in the scalar cache;
// the kernels are bound by their item streams.
#include "launch.h"
#include "mirror_dev.h"

namespace vcd {

constexpr int kMirrorBlock = 256;
constexpr int kLdsFilters = 128;          // 16 KiB of records staged per workgroup

// The filter records are read by every lane at the same address: staged in
// LDS once per workgroup they are broadcast reads; a longer list stays in
// global memory (L2).
__device__ __forceinline__ MirrorImage stage_filters(const MirrorImage& img, MirrorRec* lds) {
    if (img.n > kLdsFilters) return img;
    const uint4* g = reinterpret_cast<const uint4*>(img.f);
    uint4* l = reinterpret_cast<uint4*>(lds);
    const int words = img.n * int(sizeof(MirrorRec) / 16);
    for (int k = threadIdx.x; k < words; k += blockDim.x) l[k] = g[k];
    __syncthreads();
    return MirrorImage{lds, img.n};
}

__global__ __launch_bounds__(kMirrorBlock) void mirror_match_kernel(
    MirrorImage img, int32_t origin, vc_mirror_items in, int64_t n, uint64_t* __restrict__ out) {
    __shared__ MirrorRec lds[kLdsFilters];
    const MirrorImage fi = stage_filters(img, lds);
    const int64_t stride = int64_t(gridDim.x) * blockDim.x;
    for (int64_t i = int64_t(blockIdx.x) * blockDim.x + threadIdx.x; i < n; i += stride) {
        const MirrorItem it = mirror_item(in, i);
        out[i] = mirror_eval(fi, origin, it, mirror_level(it));
    }
}

__global__ __launch_bounds__(kMirrorBlock) void mirror_switch_kernel(
    MirrorImage img, int32_t origin, const uint8_t* __restrict__ blob,
    const uint32_t* __restrict__ off, int64_t n, int layer, uint64_t* __restrict__ out) {
    __shared__ MirrorRec lds[kLdsFilters];
    const MirrorImage fi = stage_filters(img, lds);
    const int64_t stride = int64_t(gridDim.x) * blockDim.x;
    for (int64_t i = int64_t(blockIdx.x) * blockDim.x + threadIdx.x; i < n; i += stride) {
        const uint32_t a = off[i], e = off[i + 1];
        out[i] = mirror_switch_one(fi, origin, blob + a, int(e - a), layer);
    }
}

}  // namespace vcd

namespace vc {

namespace {
int mirror_grid(const LaunchCfg& c, int64_t n) {
    int64_t want = (n + vcd::kMirrorBlock - 1) / vcd::kMirrorBlock;
    const int64_t cap = int64_t(c.num_cus) * 8;
    return int(want < cap ? want : cap);
}
}  // namespace

hipError_t launch_mirror_match(const LaunchCfg& c, const MirrorImage& img, int32_t origin,
                               const vc_mirror_items& in, int64_t n, uint64_t* out) {
    if (n <= 0) return hipSuccess;
    hipLaunchKernelGGL(vcd::mirror_match_kernel, dim3(mirror_grid(c, n)),
                       dim3(vcd::kMirrorBlock), 0, c.stream, img, origin, in, n, out);
    return hipGetLastError();
}

hipError_t launch_mirror_switch(const LaunchCfg& c, const MirrorImage& img, int32_t origin,
                                const uint8_t* blob, const uint32_t* off, int64_t n, int layer,
                                uint64_t* out) {
    if (n <= 0) return hipSuccess;
    hipLaunchKernelGGL(vcd::mirror_switch_kernel, dim3(mirror_grid(c, n)),
                       dim3(vcd::kMirrorBlock), 0, c.stream, img, origin, blob, off, n, layer, out);
    return hipGetLastError();
}

}  // namespace vc

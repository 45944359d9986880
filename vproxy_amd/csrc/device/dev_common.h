// dev_common.h -- small device helpers shared by the classifier kernels.
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

#include "../common/images.h"
#include "vclassify.h"

// Lookup helpers are __host__ __device__ so tests/native can run the exact
// same probe code on the host against a compiled image (test harness only).
#define VC_HD __host__ __device__ __forceinline__

namespace vcd {

constexpr uint32_t kFnvBasis = 2166136261u;   // 32-bit FNV-1a
constexpr uint32_t kFnvPrime = 16777619u;

VC_HD uint32_t fnv_step(uint32_t h, uint32_t c) {
    return (h ^ c) * kFnvPrime;
}

VC_HD uint32_t bswap32(uint32_t x) { return __builtin_bswap32(x); }

// 16 raw address bytes (one uint4 load) -> big-endian (hi, lo) key
VC_HD void v6_key(uint4 w, uint64_t* hi, uint64_t* lo) {
    *hi = (uint64_t(bswap32(w.x)) << 32) | bswap32(w.y);
    *lo = (uint64_t(bswap32(w.z)) << 32) | bswap32(w.w);
}

VC_HD int32_t out_index(uint32_t v) {
    return v == VC_NONE ? -1 : int32_t(v);
}

// Device-side checks (debug builds, -DVC_DEVCHECK: vproxy_amd/libvclassify_chk.so).
// VC_CHECK(cond, site, a, b) records the first failing site of the kernel
// file in a device word with two detail values, counts every failure, and
// lets the access go ahead; the library's VC_SYNC_CHECK mode reads the
// words after every launch (launch.h devcheck_take) and names the entry
// point.  Sites: 1xx stage.h, 2xx acl_dev.h, 3xx hint.hip, 4xx classify.hip,
// 5xx packet.hip.  Normal builds compile the checks away.
#if defined(VC_DEVCHECK)
static __device__ uint32_t vc_devcheck_flags[4];
#endif
#if defined(VC_DEVCHECK) && defined(__HIP_DEVICE_COMPILE__)
__device__ __noinline__ inline void devcheck_fail(uint32_t site, uint32_t a, uint32_t b) {
    if (atomicCAS(&vc_devcheck_flags[0], 0u, site) == 0u) {
        vc_devcheck_flags[2] = a;
        vc_devcheck_flags[3] = b;
    }
    atomicAdd(&vc_devcheck_flags[1], 1u);
}
#define VC_CHECK(cond, site, a, b) \
    do { if (!(cond)) ::vcd::devcheck_fail((site), uint32_t(a), uint32_t(b)); } while (0)
#else
#define VC_CHECK(cond, site, a, b) ((void)0)
#endif

}  // namespace vcd

// One reader per kernel file (each code object has its own flag words).
#if defined(VC_DEVCHECK)
#define VC_DEVCHECK_READER(name)                                                            \
    namespace vc {                                                                          \
    hipError_t devcheck_take_##name(uint32_t out[4]) {                                      \
        const uint32_t z[4] = {};                                                           \
        hipError_t e = hipMemcpyFromSymbol(out, HIP_SYMBOL(vcd::vc_devcheck_flags), 16);    \
        if (e == hipSuccess) e = hipMemcpyToSymbol(HIP_SYMBOL(vcd::vc_devcheck_flags), z, 16); \
        return e;                                                                           \
    }                                                                                       \
    }
#else
#define VC_DEVCHECK_READER(name)
#endif

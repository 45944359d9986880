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

}  // namespace vcd

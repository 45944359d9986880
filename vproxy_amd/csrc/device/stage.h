// stage.h -- per-wave LDS staging of variable-length items (names, frames)
// that sit contiguously in a blob: one coalesced dword copy per wave.
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

namespace vcd {

constexpr uint32_t kApron = 16;          // readable bytes before and after the items

// A wave's 64 items are contiguous in the blob: copy [o0, o1) into the
// wave's stage with coalesced dword loads once.  Item bytes then sit at
// byte kApron + (off - a0) of the stage.  Returns false when the span does
// not fit kBytes (the caller reads global memory instead).
template <uint32_t kBytes>
__device__ __forceinline__ bool stage_wave(const uint8_t* blob, uint32_t o0, uint32_t o1,
                                           uint32_t* stage, uint32_t* a0_out) {
    const uint32_t a0 = o0 & ~3u;                  // blob is dword aligned (launcher checks)
    *a0_out = a0;
    if (o1 - a0 > kBytes) return false;
    const int lane = int(threadIdx.x & 63);
    const uint32_t full = (o1 & ~3u) - a0;         // whole dwords inside [a0, o1)
    const uint32_t* gw = reinterpret_cast<const uint32_t*>(blob + a0);
    uint32_t* lw = stage + kApron / 4;
    for (uint32_t k = uint32_t(lane); k < full / 4; k += 64) lw[k] = gw[k];
    const uint32_t tail = o1 - (o1 & ~3u);
    if (lane == 0 && tail) {                       // last partial dword, byte loads
        uint32_t v = 0;
        for (uint32_t b = 0; b < tail; ++b) v |= uint32_t(blob[(o1 & ~3u) + b]) << (8 * b);
        lw[full / 4] = v;
    }
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    return true;
}

__device__ __forceinline__ void wave_done() {
    // every lane has finished reading the staged items before the next copy
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

}  // namespace vcd

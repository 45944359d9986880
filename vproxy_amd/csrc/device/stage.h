// stage.h -- per-wave LDS staging of variable-length items (names, frames)
// that sit contiguously in a blob: one coalesced dword copy per wave.
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

#include "dev_common.h"

namespace vcd {

constexpr uint32_t kApron = 16;          // readable bytes before and after the items

#ifndef VC_STAGE_Q
#define VC_STAGE_Q 1
#endif
// VC_STAGE_NT: the staged copy's loads carry the nontemporal hint, so the
// streamed blob does not displace the probed tables from L2: C4 0.613 ->
// 0.602 ms, DNS 0.757 -> 0.746, SNI 0.531 -> 0.519, the C5 pool pass in the
// schedule 0.770 -> 0.761 (profiles/r05_ab_stage_nt.jsonl); the DNS drain
// loop 3.935 -> 3.849 ms, parse / mirror / switch unchanged
// (r05_ab_stage_nt_frames.jsonl)
#ifndef VC_STAGE_NT
#define VC_STAGE_NT 1
#endif

// A wave's 64 items are contiguous in the blob: copy [o0, o1) into the
// wave's stage with coalesced dword loads once.  Item bytes then sit at
// byte kApron + (off - a0) of the stage.  Returns false when the span does
// not fit kBytes (the caller reads global memory instead).
template <uint32_t kBytes>
__device__ __forceinline__ bool stage_wave(const uint8_t* blob, uint32_t o0, uint32_t o1,
                                           uint32_t* stage, uint32_t* a0_out) {
    VC_CHECK(o0 <= o1, 102, o0, o1);
    const uint32_t a0 = o0 & ~3u;                  // blob is dword aligned (launcher checks)
    *a0_out = a0;
    if (o1 - a0 > kBytes) return false;
    const int lane = int(threadIdx.x & 63);
    const uint32_t full = (o1 & ~3u) - a0;         // whole dwords inside [a0, o1)
#if defined(VC_ABL_NOSTAGE)                        // timing ablation only: no copy
    if (full != 0xFFFFFFFFu) return true;
#endif
#if VC_STAGE_Q
    // 16-byte pieces, every load of a round (4 KiB) in flight before any LDS
    // write: one global round trip per round.  (A dword loop compiled to
    // batches of four loads per lane, each waited for before the next: three
    // round trips for a pair of hint chunks.)  Piece indices are clamped to
    // the last piece instead of predicated -- the duplicate loads and LDS
    // writes of lanes past the end carry the same bytes to the same place --
    // so a round is straight-line code.  The blob is only dword aligned; an
    // unaligned dwordx4 global load is legal on gfx950.
    typedef uint4 __attribute__((aligned(4))) q4;
    typedef uint32_t __attribute__((ext_vector_type(4), aligned(4))) v4a;
    const uint32_t nq = full >> 4;                 // whole 16-byte pieces
    const q4* gq = reinterpret_cast<const q4*>(blob + a0);
    uint32_t* lw = stage + kApron / 4;
    // the bytes past the pieces: up to three whole dwords (lanes 0-2) and
    // the partial last dword (byte loads), loaded before the first round
    const uint32_t rw = (full >> 2) & 3u, tail = o1 & 3u;
    const uint32_t* gw = reinterpret_cast<const uint32_t*>(blob + a0 + 16 * nq);
    uint32_t t = 0;
    if (uint32_t(lane) < rw) {
        t = gw[lane];
    } else if (uint32_t(lane) == rw && tail) {
        for (uint32_t b = 0; b < tail; ++b) t |= uint32_t(blob[(o1 & ~3u) + b]) << (8 * b);
    }
    constexpr uint32_t kRound = 4;                 // pieces per lane per round
    for (uint32_t r0 = 0; r0 < nq; r0 += 64 * kRound) {
        const uint32_t last = nq - 1;
        uint4 v[kRound];
#pragma unroll
        for (uint32_t j = 0; j < kRound; ++j) {
            const uint32_t k = r0 + 64 * j + uint32_t(lane);
#if VC_STAGE_NT
            const v4a t4 = __builtin_nontemporal_load(
                reinterpret_cast<const v4a*>(gq + (k < last ? k : last)));
            v[j] = make_uint4(t4.x, t4.y, t4.z, t4.w);
#else
            v[j] = gq[k < last ? k : last];
#endif
        }
#if VC_STAGE_Q == 2
        __builtin_amdgcn_sched_barrier(0);         // every load issued before a write
#endif
#pragma unroll
        for (uint32_t j = 0; j < kRound; ++j) {
            const uint32_t k0 = r0 + 64 * j + uint32_t(lane), k = k0 < last ? k0 : last;
            uint32_t* d = lw + 4 * k;
            d[0] = v[j].x;
            d[1] = v[j].y;
            d[2] = v[j].z;
            d[3] = v[j].w;
        }
        if (kBytes <= 64 * 16 * kRound) break;     // one round covers the stage
    }
    if (uint32_t(lane) < rw + (tail ? 1u : 0u)) lw[4 * nq + uint32_t(lane)] = t;
#else
    const uint32_t* gw = reinterpret_cast<const uint32_t*>(blob + a0);
    uint32_t* lw = stage + kApron / 4;
    for (uint32_t k = uint32_t(lane); k < full / 4; k += 64) lw[k] = gw[k];
    const uint32_t tail = o1 - (o1 & ~3u);
    if (lane == 0 && tail) {                       // last partial dword, byte loads
        uint32_t v = 0;
        for (uint32_t b = 0; b < tail; ++b) v |= uint32_t(blob[(o1 & ~3u) + b]) << (8 * b);
        lw[full / 4] = v;
    }
#endif
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    return true;
}

// A lane's item [a, e) of the chunk starting at `base` (clamped to n past
// the end).  The streaming kernels load the next chunk's offsets before
// parsing the current one, and take the chunk's span from lanes 0 and
// last (span_of), so a chunk costs one blob round trip instead of three
// dependent ones (offsets of the span, the blob, the lane's offsets).
struct LaneSpan {
    uint32_t a, e;
};

__device__ __forceinline__ LaneSpan lane_span(const uint32_t* off, int64_t base, int64_t n) {
    const int64_t i = base + int(threadIdx.x & 63);
    const LaneSpan s{off[i < n ? i : n], off[i + 1 < n ? i + 1 : n]};
#if defined(VC_DEVCHECK)
    // offsets ascend and stay inside the blob [0, off[n])
    VC_CHECK(s.a <= s.e && s.e <= off[n], 101, i, s.e);
#endif
    return s;
}

// [o0, o1) of the chunk's items, from the lanes' spans (wave-uniform)
__device__ __forceinline__ void span_of(const LaneSpan& s, int64_t base, int64_t n, uint32_t* o0,
                                        uint32_t* o1) {
    const int lastl = int((base + 64 < n ? base + 64 : n) - base - 1);
    *o0 = uint32_t(__builtin_amdgcn_readfirstlane(int(s.a)));
    *o1 = uint32_t(__builtin_amdgcn_readlane(int(s.e), lastl));
}

__device__ __forceinline__ void wave_done() {
    // every lane has finished reading the staged items before the next copy
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

}  // namespace vcd

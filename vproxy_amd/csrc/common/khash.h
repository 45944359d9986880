// khash.h -- the key hash of the host-name tables (hint-host keys, DNS hosts
// map), shared by the table compiler (host) and the kernels (device).
//
// The hash walks a string right to left in 4-byte chunks aligned to the END
// of the string: chunk k holds bytes [L-4k-4, L-4k) as a little-endian word,
// and the leftmost chunk, when L is not a multiple of 4, holds the first
// L mod 4 bytes in its HIGH bytes with the low bytes zero.  Because every
// dot-suffix of a name ends where the name ends, one right-to-left pass over
// a query host yields, at each '.', the state after the suffix's whole
// chunks; the suffix's hash is that state mixed with the current chunk
// masked below the dot, finalised with the suffix length.  So a host and
// all of its "." + H candidates (Hint.java:136 host.endsWith("." + H)) are
// hashed in one pass, a word at a time, with one multiply per 4 bytes.
//
// The hash only picks the probe position and the 32-bit tag; every tag hit
// is confirmed by a full key compare, so collisions cost time, not results.
#pragma once

#include <stdint.h>

#if defined(__HIPCC__) || defined(__HIP__)
#include <hip/hip_runtime.h>
#define VC_KH __host__ __device__ __forceinline__
#else
#define VC_KH inline
#endif

namespace vck {

constexpr uint32_t kSeed = 0x9E3779B9u;

VC_KH uint32_t mix(uint32_t h, uint32_t w) {
    h = (h ^ w) * 0x85EBCA77u;
    return h ^ (h >> 15);
}

// murmur3 fmix32 of the state with the length folded in
VC_KH uint32_t fin(uint32_t h, uint32_t len) {
    h ^= len * 0xC2B2AE3Du;
    h ^= h >> 16;
    h *= 0x85EBCA6Bu;
    h ^= h >> 13;
    h *= 0xC2B2AE35u;
    h ^= h >> 16;
    return h;
}

// Reference form over plain bytes (table compiler, slow device paths).
VC_KH uint32_t khash(const uint8_t* p, int len) {
    uint32_t h = kSeed;
    int e = len;
    while (e >= 4) {
        const uint32_t w = uint32_t(p[e - 4]) | (uint32_t(p[e - 3]) << 8) |
                           (uint32_t(p[e - 2]) << 16) | (uint32_t(p[e - 1]) << 24);
        h = mix(h, w);
        e -= 4;
    }
    if (e > 0) {                      // first e bytes into the high bytes
        uint32_t w = 0;
        for (int i = 0; i < e; ++i) w |= uint32_t(p[i]) << (8 * (4 - e + i));
        h = mix(h, w);
    }
    return fin(h, uint32_t(len));
}

// Per-byte 0x80 flags of the bytes of w equal to c (exact, no borrow
// between bytes).
VC_KH uint32_t byte_eq_flags(uint32_t w, uint32_t c4) {
    const uint32_t x = w ^ c4;
    return ~((((x & 0x7F7F7F7Fu) + 0x7F7F7F7Fu) | x) | 0x7F7F7F7Fu);
}

}  // namespace vck

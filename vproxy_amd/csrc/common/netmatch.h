// netmatch.h -- Network.maskMatch (base/src/main/java/vproxybase/util/Network.java:183-278)
// on 16-byte address words, shared by the host control plane (host/net.cpp)
// and the kernels (device/mirror_dev.h).
//
// An address or mask of 4 or 16 bytes is held as four little-endian words of
// its left-aligned bytes (a 4-byte value in word 0).  Java compares
// `(inputB & maskB) != ruleB` on sign-extended bytes, which is the same as
// comparing the raw bytes, so whole words compare at once.
#pragma once

#include <stdint.h>

#if defined(__HIPCC__) || defined(__HIP__)
#include <hip/hip_runtime.h>
#define VC_NM __host__ __device__ inline
#else
#define VC_NM inline
#endif

namespace vcn {

struct Addr {
    uint32_t w[4];
    int len;                      // 4 or 16
};

// Utils.lowBitsV6V4(ip, 11, 10) (Utils.java:122-133): bytes 0..9 zero and
// bytes 10..11 both 0x00 or both 0xFF.
VC_NM bool low_bits_v6v4(const Addr& a) {
    return a.w[0] == 0 && a.w[1] == 0 && (a.w[2] == 0 || a.w[2] == 0xFFFF0000u);
}

// last word of a 4- or 16-byte value
VC_NM uint32_t last_word(const Addr& a) { return a.len == 16 ? a.w[3] : a.w[0]; }

VC_NM bool mask_match(const Addr& in, const Addr& rule, const Addr& mask) {
    if (in.len == rule.len && rule.len > mask.len)       // (1) v6 in, v6 rule, 4-byte mask
        return (in.w[0] & mask.w[0]) == rule.w[0];
    if (in.len < rule.len && rule.len > mask.len)        // (2) v4 in, v6 rule, 4-byte mask
        return false;
    if (in.len < rule.len && rule.len == mask.len)       // (3) v4 in, v6 rule, 16-byte mask
        return (in.w[0] & mask.w[3]) == rule.w[3] && low_bits_v6v4(rule);
    // (4) and (5): compare the last min(lengths) bytes, aligned at the ends
    if (in.len == 16 && rule.len == 16 && mask.len == 16) {
        for (int k = 0; k < 4; ++k)
            if ((in.w[k] & mask.w[k]) != rule.w[k]) return false;
        return true;
    }
    if ((last_word(in) & last_word(mask)) != last_word(rule)) return false;
    return in.len > rule.len ? low_bits_v6v4(in) : true;
}

VC_NM Addr addr_of(const uint8_t* p, int len) {
    Addr a{{0, 0, 0, 0}, len};
    for (int k = 0; k < len && k < 16; ++k) a.w[k >> 2] |= uint32_t(p[k]) << (8 * (k & 3));
    return a;
}

}  // namespace vcn

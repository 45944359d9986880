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

// Network.contains(IP) compiled per input family (common to the mirror
// filters): maskMatch's case analysis depends only on the three lengths, so
// for a fixed rule and mask every case reduces to
//   (in & m) == r  (word-wise)  [&& lowBitsV6V4(in) when `low`]
// -- "never" is m = 0, r != 0.
struct NetMatch {
    uint32_t m6[4], r6[4];        // 16-byte inputs
    uint32_t low6;                // 16-byte inputs also need lowBitsV6V4(input)
    uint32_t m4, r4;              // 4-byte inputs
    uint32_t pad;
};

VC_NM NetMatch net_matcher(const Addr& rule, const Addr& mask) {
    NetMatch n{{0, 0, 0, 0}, {0, 0, 0, 0}, 0, 0, 0, 0};
    // 4-byte input
    if (rule.len == 4) {                                  // (5): tails, the last mask word
        n.m4 = last_word(mask);
        n.r4 = rule.w[0];
    } else if (mask.len == 16 && low_bits_v6v4(rule)) {   // (3)
        n.m4 = mask.w[3];
        n.r4 = rule.w[3];
    } else {                                              // (2), or (3) failing lowBits
        n.m4 = 0;
        n.r4 = 1;
    }
    // 16-byte input
    if (rule.len == 16 && mask.len == 4) {                // (1): first 4 bytes
        n.m6[0] = mask.w[0];
        n.r6[0] = rule.w[0];
    } else if (rule.len == 16) {                          // (5): all 16 bytes
        for (int k = 0; k < 4; ++k) {
            n.m6[k] = mask.w[k];
            n.r6[k] = rule.w[k];
        }
    } else {                                              // (4): last 4 bytes + lowBits(input)
        n.m6[3] = last_word(mask);
        n.r6[3] = rule.w[0];
        n.low6 = 1;
    }
    return n;
}

// in.len 4 or 16; in_low = low_bits_v6v4(in) for 16-byte inputs
VC_NM bool net_match(const NetMatch& n, const Addr& in, bool in_low) {
    if (in.len == 4) return (in.w[0] & n.m4) == n.r4;
    const uint32_t d = ((in.w[0] & n.m6[0]) ^ n.r6[0]) | ((in.w[1] & n.m6[1]) ^ n.r6[1]) |
                       ((in.w[2] & n.m6[2]) ^ n.r6[2]) | ((in.w[3] & n.m6[3]) ^ n.r6[3]);
    return d == 0 && (!n.low6 || in_low);
}

VC_NM Addr addr_of(const uint8_t* p, int len) {
    Addr a{{0, 0, 0, 0}, len};
    for (int k = 0; k < len && k < 16; ++k) a.w[k >> 2] |= uint32_t(p[k]) << (8 * (k & 3));
    return a;
}

}  // namespace vcn

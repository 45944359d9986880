// acl_dev.h -- device side of SecurityGroup.allow (SecurityGroup.java:30-45).
//
// The ACL image (common/images.h) turns the first-match scan over the
// protocol's rule list into: interval search on the source address, then a
// port -> first-rule function for that interval.
#pragma once

#include "dev_common.h"

namespace vcd {

// Typed reads.  A table pointer taken from a struct or chosen per item (the
// protocol's list) is generic to the compiler, and a generic read compiles
// to flat_load, which also waits on vmcnt: LDS-staged boundaries are read
// through an LDS pointer (ds_read), the image's tables through a global one.
#if defined(__HIP_DEVICE_COMPILE__)
#define VC_AS_LDS __attribute__((address_space(3)))
#define VC_AS_GLB __attribute__((address_space(1)))
#else
#define VC_AS_LDS
#define VC_AS_GLB
#endif
template <class T>
VC_HD T lds_ld(const T* p) {
#if defined(VC_GENERIC_LDS)       // A/B builds only: the generic (flat) read
    return *p;
#else
    return *(const VC_AS_LDS T*)(p);
#endif
}
template <class T>
VC_HD T glb_ld(const T* p) { return *(const VC_AS_GLB T*)(p); }
template <bool kL, class T>
VC_HD T tbl_ld(const T* p) { return kL ? lds_ld(p) : glb_ld(p); }

// Last j with b[j] <= key (b[0] == 0, so j >= 0).  Fixed trip count per nb.
// kL: b is staged in LDS.
template <bool kL = false>
VC_HD int bsearch_u32(const uint32_t* b, int nb, uint32_t key) {
    int lo = 0, len = nb;
    while (len > 1) {
        int half = len >> 1;
        lo = (tbl_ld<kL>(b + lo + half) <= key) ? lo + half : lo;
        len -= half;
    }
    return lo;
}

VC_HD bool le128(uint64_t ah, uint64_t al, uint64_t bh, uint64_t bl) {
    return ah < bh || (ah == bh && al <= bl);
}

// bounds6 = (hi, lo) pairs; last j with bounds[j] <= key
template <bool kL = false>
VC_HD int bsearch_u128(const uint64_t* b, int nb, uint64_t kh, uint64_t kl) {
    int lo = 0, len = nb;
    while (len > 1) {
        int half = len >> 1;
        const ulonglong2 v = tbl_ld<kL>(reinterpret_cast<const ulonglong2*>(b + 2 * (lo + half)));
        lo = le128(v.x, v.y, kh, kl) ? lo + half : lo;
        len -= half;
    }
    return lo;
}

// The v4 interval of `key` from the global boundaries: through the bucket
// directory when the image has one (images.h), else a whole binary search.
VC_HD int acl4_interval(const AclFamilyImage& f, uint32_t key) {
    if (f.dir4) {
        const uint32_t e = glb_ld(f.dir4 + (key >> (32 - f.dir_bits)));
        const int s = int(e & 0xFFFFu);
        VC_CHECK(s + int(e >> 16) < f.nb, 201, key, e);
        return s + bsearch_u32(f.bounds4 + s, int(e >> 16) + 1, key);
    }
    return bsearch_u32(f.bounds4, f.nb, key);
}

// desc (x, y) -> rule index (or VC_NONE) for `port`
VC_HD uint32_t port_lookup(const uint32_t* pieces, uint2 d, uint32_t port) {
    if (d.y == 0) return d.x;
    const uint2* p = reinterpret_cast<const uint2*>(pieces) + d.x;
    int n = int(d.y);
    if (n <= 8) {
        uint32_t v = glb_ld(p).y;
        for (int k = 1; k < n; ++k) {
            uint2 q = glb_ld(p + k);
            if (q.x > port) break;
            v = q.y;
        }
        return v;
    }
    int lo = 0, len = n;
    while (len > 1) {
        int half = len >> 1;
        lo = (glb_ld(p + lo + half).x <= port) ? lo + half : lo;
        len -= half;
    }
    return glb_ld(p + lo).y;
}

// Rule index (or VC_NONE) of interval j for `port`: one 16-byte record
// load (images.h AclFamilyImage.rec); the pieces array only for intervals
// with more than four port pieces.
VC_HD uint32_t acl_rec_value(uint4 r, const uint32_t* pieces, uint32_t port) {
    const uint32_t k = (r.x >> 16) & 0xFFu;
    if (k == 0xFFu) return port_lookup(pieces, make_uint2(r.y, r.z), port);
    uint32_t v = r.x & 0xFFFFu;
    if (k > 1 && port >= (r.y >> 16)) v = r.y & 0xFFFFu;
    if (k > 2 && port >= (r.z >> 16)) v = r.z & 0xFFFFu;
    if (k > 3 && port >= (r.w >> 16)) v = r.w & 0xFFFFu;
    return v == 0xFFFFu ? VC_NONE : v;
}

VC_HD uint32_t acl_value(const uint32_t* rec, const uint32_t* pieces, int j, uint32_t port) {
    return acl_rec_value(glb_ld(reinterpret_cast<const uint4*>(rec) + j), pieces, port);
}

// An IPv6 key (hi, lo = bytes 0-7, 8-15) in the forms an IPv4 rule can
// match (Network.maskMatch cases 4/5, Network.java:246-277, with
// Utils.lowBitsV6V4(ip, 11, 10), Utils.java:122-133): ::a.b.c.d or
// ::ffff:a.b.c.d.  Such a key matches an IPv4 rule iff its low 32 bits do.
VC_HD bool v6_v4_form(uint64_t hi, uint64_t lo) {
    const uint32_t w = uint32_t(lo >> 32);
    return hi == 0 && (w == 0u || w == 0xFFFFu);
}

// Rule index (or VC_NONE) of an IPv6 key on one list, from global memory:
// f6 / f4 are the list's v6 and v4 images.  A list of plain IPv4 rules
// (f6.v4_only) classifies the key's low 32 bits through the v4 image (its
// bucket directory) when the key has an IPv4 form, and as no rule
// otherwise; any other list runs the 128-bit interval search.
VC_HD uint32_t acl6_global(const AclFamilyImage& f6, const AclFamilyImage& f4, uint64_t hi,
                           uint64_t lo, uint32_t port) {
    if (f6.v4_only)
        return v6_v4_form(hi, lo) ? acl_value(f4.rec, f4.pieces, acl4_interval(f4, uint32_t(lo)), port)
                                  : VC_NONE;
    return acl_value(f6.rec, f6.pieces, bsearch_u128(f6.bounds6, f6.nb, hi, lo), port);
}

}  // namespace vcd

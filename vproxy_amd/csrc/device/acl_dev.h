// acl_dev.h -- device side of SecurityGroup.allow (SecurityGroup.java:30-45).
//
// The ACL image (common/images.h) turns the first-match scan over the
// protocol's rule list into: interval search on the source address, then a
// port -> first-rule function for that interval.
#pragma once

#include "dev_common.h"

namespace vcd {

// Last j with b[j] <= key (b[0] == 0, so j >= 0).  Fixed trip count per nb.
VC_HD int bsearch_u32(const uint32_t* b, int nb, uint32_t key) {
    int lo = 0, len = nb;
    while (len > 1) {
        int half = len >> 1;
        lo = (b[lo + half] <= key) ? lo + half : lo;
        len -= half;
    }
    return lo;
}

VC_HD bool le128(uint64_t ah, uint64_t al, uint64_t bh, uint64_t bl) {
    return ah < bh || (ah == bh && al <= bl);
}

// bounds6 = (hi, lo) pairs; last j with bounds[j] <= key
VC_HD int bsearch_u128(const uint64_t* b, int nb, uint64_t kh, uint64_t kl) {
    int lo = 0, len = nb;
    while (len > 1) {
        int half = len >> 1;
        const ulonglong2 v = *reinterpret_cast<const ulonglong2*>(b + 2 * (lo + half));
        lo = le128(v.x, v.y, kh, kl) ? lo + half : lo;
        len -= half;
    }
    return lo;
}

// desc (x, y) -> rule index (or VC_NONE) for `port`
VC_HD uint32_t port_lookup(const uint32_t* pieces, uint2 d, uint32_t port) {
    if (d.y == 0) return d.x;
    const uint2* p = reinterpret_cast<const uint2*>(pieces) + d.x;
    int n = int(d.y);
    if (n <= 8) {
        uint32_t v = p[0].y;
        for (int k = 1; k < n; ++k) {
            uint2 q = p[k];
            if (q.x > port) break;
            v = q.y;
        }
        return v;
    }
    int lo = 0, len = n;
    while (len > 1) {
        int half = len >> 1;
        lo = (p[lo + half].x <= port) ? lo + half : lo;
        len -= half;
    }
    return p[lo].y;
}

VC_HD uint2 load_desc(const uint32_t* desc, int j) {
    return reinterpret_cast<const uint2*>(desc)[j];
}

}  // namespace vcd

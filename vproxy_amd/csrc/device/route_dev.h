// route_dev.h -- device side of RouteTable.lookup (RouteTable.java:44-59).
//
// Walks the leaf-pushed stride trie: root entry, then at most one node per
// remaining byte of the prefix (the first one up to the byte boundary), or one 16-byte one-prefix record where
// the subtree holds a single prefix (images.h VC_ONE).  Every entry holds the
// min list index of the prefixes covering it, so the last entry reached is
// the answer.
#pragma once

#include "dev_common.h"

namespace vcd {

// One-prefix record: the key's top bits (hi = key bits 0-63, left-aligned)
// against the record's prefix.
VC_HD uint32_t one_match(uint4 r, uint64_t hi) {
    const uint32_t len = r.w >> 24;                        // rb < len <= 64
    const uint64_t key = (uint64_t(r.x) << 32) | r.y;
    const uint32_t miss = r.w & 0xFFFFFFu;
    if (((hi ^ key) >> (64 - len)) == 0) return r.z;
    return miss == 0xFFFFFFu ? VC_NONE : miss;
}

// Bits a node at depth `bits` consumes: up to the next byte boundary.
VC_HD int trie_stride(int bits) { return 8 - (bits & 7); }

// Next entry below pointer entry e: the child node's entry `sub`, or the
// record's answer (never a pointer, so the walk ends).
VC_HD uint32_t trie_next(const uint32_t* nodes, uint32_t root, uint32_t e, uint32_t sub,
                         uint64_t hi) {
    if (e & VC_ONE) return one_match(reinterpret_cast<const uint4*>(nodes)[e & ~(VC_PTR | VC_ONE)], hi);
    return nodes[root + (e & ~VC_PTR) * 16u + sub];
}

// The `s` key bits after the first `bits` (s = trie_stride(bits), so they
// never straddle a byte boundary).
VC_HD uint32_t v4_sub(uint32_t key, int bits, int s) {
    return (key >> (32 - bits - s)) & ((1u << s) - 1u);
}

// The walk from the root entry e = nodes[key >> (32 - rb)], which a caller
// may load ahead of time (its latency then overlaps other work).
VC_HD uint32_t trie_v4_from(const uint32_t* nodes, int rb, uint32_t key, uint32_t e) {
    int bits = rb;
    const uint32_t root = 1u << rb;
    while (e & VC_PTR) {
        const int s = trie_stride(bits);
        e = trie_next(nodes, root, e, v4_sub(key, bits, s), uint64_t(key) << 32);
        bits += s;
    }
    return e;
}

VC_HD uint32_t trie_v4(const uint32_t* nodes, int rb, uint32_t key) {
    return trie_v4_from(nodes, rb, key, nodes[key >> (32 - rb)]);
}

VC_HD uint32_t v6_sub(uint64_t hi, uint64_t lo, int bits, int s) {
    const uint64_t m = (uint64_t(1) << s) - 1u;
    return bits < 64 ? uint32_t((hi >> (64 - bits - s)) & m) : uint32_t((lo >> (128 - bits - s)) & m);
}

// Wide-root entry of root slot s (images.h TrieImage.wide): the one-prefix
// record inline, or {root entry, 0, 0, 0}.
VC_HD void wide_entry(const uint32_t* nodes, uint32_t s, uint32_t out[4]) {
    const uint32_t e = nodes[s];
    if ((e & VC_PTR) && (e & VC_ONE)) {
        const uint32_t* r = nodes + 4u * (e & ~(VC_PTR | VC_ONE));
        out[0] = r[0]; out[1] = r[1]; out[2] = r[2]; out[3] = r[3];
    } else {
        out[0] = e; out[1] = 0u; out[2] = 0u; out[3] = 0u;
    }
}

// First step of an IPv6 walk from a wide-root entry: the answer of a
// one-prefix slot, else the root entry (a value or a node pointer).
VC_HD uint32_t wide_first(uint4 w, uint64_t hi) {
    return (w.w >> 24) ? one_match(w, hi) : w.x;
}

VC_HD uint32_t trie_v6(const uint32_t* nodes, int rb, uint64_t hi, uint64_t lo);

// trie_v6 through the wide root when the image has one (one load for a
// one-prefix slot instead of two dependent ones).
VC_HD uint32_t trie_v6w(const uint32_t* nodes, const uint32_t* wide, int rb, uint64_t hi,
                        uint64_t lo) {
    if (!wide) return trie_v6(nodes, rb, hi, lo);
    uint32_t e = wide_first(reinterpret_cast<const uint4*>(wide)[hi >> (64 - rb)], hi);
    int bits = rb;
    const uint32_t root = 1u << rb;
    while (e & VC_PTR) {
        const int s = trie_stride(bits);
        e = trie_next(nodes, root, e, v6_sub(hi, lo, bits, s), hi);
        bits += s;
    }
    return e;
}

VC_HD uint32_t trie_v6(const uint32_t* nodes, int rb, uint64_t hi, uint64_t lo) {
    uint32_t e = nodes[hi >> (64 - rb)];
    int bits = rb;
    const uint32_t root = 1u << rb;
    while (e & VC_PTR) {
        const int s = trie_stride(bits);
        e = trie_next(nodes, root, e, v6_sub(hi, lo, bits, s), hi);
        bits += s;
    }
    return e;
}

}  // namespace vcd

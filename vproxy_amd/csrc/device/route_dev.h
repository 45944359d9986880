// route_dev.h -- device side of RouteTable.lookup (RouteTable.java:44-59).
//
// Walks the leaf-pushed stride trie: root entry, then at most one 8-bit node
// per remaining byte of the prefix.  Every entry holds the min list index of
// the prefixes covering it, so the last entry reached is the answer.
#pragma once

#include "dev_common.h"

namespace vcd {

VC_HD uint32_t trie_v4(const uint32_t* nodes, int rb, uint32_t key) {
    uint32_t e = nodes[key >> (32 - rb)];
    int shift = 32 - rb;
    const uint32_t root = 1u << rb;
    while (e & VC_PTR) {
        shift -= 8;
        e = nodes[root + (e & ~VC_PTR) * 256u + ((key >> shift) & 255u)];
    }
    return e;
}

VC_HD uint32_t trie_v6(const uint32_t* nodes, int rb, uint64_t hi, uint64_t lo) {
    uint32_t e = nodes[hi >> (64 - rb)];
    int bits = rb;
    const uint32_t root = 1u << rb;
    while (e & VC_PTR) {
        uint32_t sub = bits < 64 ? uint32_t(hi >> (56 - bits)) & 255u
                                 : uint32_t(lo >> (120 - bits)) & 255u;
        e = nodes[root + (e & ~VC_PTR) * 256u + sub];
        bits += 8;
    }
    return e;
}

}  // namespace vcd

// images.h -- the device-resident table images the HIP kernels read.
//
// Built on the host by csrc/compile/*.cpp, copied to HBM once per compile
// (snapshot), read-only afterwards.  Layouts are flat arrays of 4/8/16-byte
// words so every probe is one aligned load.
#pragma once

#include <stdint.h>

#define VC_NONE 0x7FFFFFFFu       // "no rule" in a value slot (-> -1 on output)
#define VC_PTR  0x80000000u       // trie entry: child node pointer flag
#define VC_ONE  0x40000000u       // with VC_PTR: one-prefix record (RouteImage)
#define VC_ONE_MAX 0x40000000u    // record ids (16-byte units from the node base)

// ---------------------------------------------------------------------------
// ACL (SecurityGroup): one image per (protocol list, input family).
//
// The input key space (32-bit for IPv4 inputs, 128-bit for IPv6 inputs) is
// cut into elementary intervals at every rule-projection edge.  Interval j
// = [bounds[j], bounds[j+1]).  desc[j] describes the port -> first-rule
// function on that interval:
//   desc.y == 0 : constant, desc.x = rule index or VC_NONE
//   desc.y  > 0 : desc.y pieces at pieces[desc.x ...], each (port_start,
//                 value), port_start ascending, first port_start == 0.
// Identical port functions share one piece run.
// ---------------------------------------------------------------------------
struct AclFamilyImage {
    const uint32_t* bounds4;      // v4: nb boundaries (bounds4[0] == 0)
    const uint64_t* bounds6;      // v6: nb boundaries as (hi, lo) pairs, 2*nb words
    // 4*nb words: one 16-byte record per interval, read with one load:
    // word 0 = value of piece 0 (port 0 up; 16 bits, 0xFFFF = VC_NONE) |
    // piece count k << 16, words 1..k-1 = port_start << 16 | value of the
    // next pieces; k == 0xFF: words 1, 2 = (x, y) into `pieces` (more than
    // four pieces or a rule index >= 0xFFFF; y == 0: the value is x)
    const uint32_t* rec;
    const uint32_t* pieces;       // 2*np words: (port_start, value)
    // v4, 16 < nb < 65536: a bucket directory over the key's top dir_bits
    // bits, entry t = s(t) | (s(t + 1) - s(t)) << 16, s(t) = the interval of
    // key t << (32 - dir_bits): a key of bucket t is in [s(t), s(t + 1)].
    // Kernels that search the boundaries in global memory start there
    // (acl4_interval) -- about two dependent loads instead of log2(nb).
    const uint32_t* dir4;         // null: none
    int32_t nb;
    int32_t np;
    int32_t dir_bits;
    // v6 image of a list whose rules are all plain IPv4 networks: an IPv6
    // key can then only match in its ::a.b.c.d / ::ffff:a.b.c.d forms, on
    // its low 32 bits, exactly as the list's v4 image classifies them
    // (acl_dev.h acl6_global); bounds6 / rec stay built for that case too
    int32_t v4_only;
};

// SecurityGroup.allow(UDP, IPv4 key, port) for one fixed port (the Switch's
// VXLAN bind port, Switch.java:679): the UDP v4 image's intervals with the
// port function evaluated at that port, equal neighbours merged, so a
// lookup is one search of a table small enough for LDS.  nb == 0: none.
struct AclPortImage {
    const uint32_t* bounds;       // nb ascending interval starts, bounds[0] == 0
    const uint32_t* value;        // per interval: the UDP rule index or VC_NONE
    int32_t nb;
    int32_t port;
};

struct AclImage {
    AclFamilyImage fam[2][2];     // [0 = tcp list, 1 = udp list][0 = v4 input, 1 = v6 input]
    const uint8_t* allow;         // rule allow bits: tcp rules then udp rules
    int32_t n_tcp, n_udp;
    int32_t default_allow;
};

// ---------------------------------------------------------------------------
// RouteTable: one multibit stride trie per family (DIR-24-8 for IPv4).
// Root = 2^root_bits entries (16, 20 or 24).  Below it the walk strides to
// the next byte boundary, then 8 bits at a time: a node at depth `bits`
// has 2^(8 - bits % 8) entries (16 under a 20-bit root, else 256).
// Entry: VC_PTR | node_id  -> child at nodes[(1<<root_bits) + node_id*16]
//                             (nodes are allocated in 16-entry units, so
//                             every node starts on a 64-byte line)
//        VC_PTR | VC_ONE | id -> one-prefix record at ((uint4*)nodes)[id]:
//                             {key bits 0-31, key bits 32-63, match value,
//                              miss value (24 bits, 0xFFFFFF = none) | len << 24}
//                             -- the entry's subtree holds one prefix of
//                             length len <= 64; the answer is the match
//                             value when the key's top len bits equal it
//        otherwise value   -> min list index of the prefixes covering this
//                             entry's address range (VC_NONE if none).
// "min list index" is RouteTable.lookup's first-match (list order), not LPM.
// ---------------------------------------------------------------------------
//
// IPv6 wide root (`wide`, built on the device from the root at compile time,
// route_dev.h wide_entry): 4 words per root slot, so the first access of a
// walk answers a one-prefix slot by itself --
//   a one-prefix record's subtree: the record, inline (its word 3 has
//                             len << 24 with len > root_bits: nonzero)
//   any other slot:           {root entry, 0, 0, 0}
// IPv6 prefixes are /32-/64 on top of a 2^24 root, so without it a lookup
// inside a prefix read the root entry and then the record: two dependent
// misses.  The array is 16x the root's bytes, but only the slots under the
// address ranges in use are ever read (2000::/3 is 1/8 of them).
struct TrieImage {
    const uint32_t* nodes;
    const uint32_t* wide;         // IPv6 only: 4 words per root slot, or null
    int32_t root_bits;
    int32_t key_bits;             // 32 (v4) or 128 (v6)
    int32_t n_rules;
    int32_t pad_;
};

struct RouteImage {
    TrieImage fam[2];             // 0 = rulesV4, 1 = rulesV6
};

// Switch.tables: the RouteTable of each VNI (Switch.java:560-566), for the
// switch kernel.  vni[] ascending; tables[t] is the route image of vni[t].
struct VniImage {
    const uint32_t* vni;
    const RouteImage* tables;
    int32_t n;                    // 0: one network, the context's RouteImage
    int32_t pad_;
};

// ---------------------------------------------------------------------------
// Upstream hint matching + DNS hosts.
//
// Host-name keys (merged hint-host H, and the DNS hosts map) live in
// open-addressing tables keyed by the end-aligned chunk hash of
// common/khash.h, so one right-to-left pass over a query host hashes the
// host and every dot-suffix.  Power-of-two capacity, linear probing from the
// hash's 4-slot group.  Probes walk a compact tag array (4 B per slot,
// hash | 1, 0 = empty; L2-resident for 100k keys) and read the slot's
// 64-byte record -- one cache line holding the key inline and the answer --
// only on a tag hit; every tag hit is confirmed by a full key compare.
//
// URI keys (merged hint-uri U) are matched by prefix, so they hash
// left-to-right with 32-bit FNV-1a: one scan of a URI yields the hash of
// every prefix.  They use the older 32-byte KeySlot (general path only).
// ---------------------------------------------------------------------------
#define VC_REC_INLINE 48           // key bytes held inline in a HostRec
#define VC_REC_HAS_PM 0x80000000u  // HostRec.len_pm: key has hint-port minima
// Hint table only (Hint.matchLevel with a uri): some member of the key has a
// hint-uri; SPLIT: and the key has two or more members, so the uri level can
// decide among them.  A key without SPLIT answers a port-0 hint with a uri
// exactly as without one when it is the only key at the hint's top host
// level (hint_dev.h host_only_fast).
#define VC_REC_ANYURI 0x40000000u
#define VC_REC_SPLIT  0x20000000u
#define VC_REC_LEN    0x1FFFFFFFu  // key length bits of len_pm

struct HostRec {                   // 64 bytes, 64-byte aligned
    uint32_t len_pm;               // key length | VC_REC_HAS_PM
    int32_t a;                     // hint table: min handle index (any port); hosts: value
    int32_t b;                     // hint table: min handle index with no hint-port
    uint32_t key_off;              // whole key in the blob (16-byte aligned, zero padded)
    uint8_t key[VC_REC_INLINE];    // first 48 key bytes, zero padded
};

struct HostExt {                   // 16 bytes per host slot (slow paths only)
    uint32_t list_off;             // member list (handle indices ascending) in lists[]
    uint32_t list_cnt;
    uint32_t pm_off;               // distinct nonzero hint-ports in port_mins[]
    uint32_t pm_cnt;
};

struct KeySlot {                   // 32 bytes (URI table)
    uint64_t hash;                 // 32-bit FNV-1a in the low word
    int32_t key_len;               // -1 = empty slot
    uint32_t key_off;              // into HintImage.blob
    int32_t a;
    int32_t b;
    uint32_t list_off;             // member list (handle indices ascending) in lists[]
    uint32_t list_cnt;
};

struct PortMin {                   // per host key: min index per distinct hint-port
    int32_t port;
    int32_t idx;
};

struct GroupRec {                  // merged annotations of one ServerGroupHandle
    int32_t host_len;              // -1 = null
    uint32_t host_off;
    int32_t uri_len;               // -1 = null (bytes)
    uint32_t uri_off;
    int32_t port;                  // 0 = absent
    int32_t any;                   // 0 when H, P and U are all absent (level is always 0)
    int32_t uri_units;             // U.length(): UTF-16 code units of the UTF-8 bytes
    int32_t pad;
};

struct HintImage {
    const uint8_t* blob;           // key / annotation bytes
    const HostRec* host_recs;      // keyed by H (chunk hash)
    const HostExt* host_ext;
    const uint32_t* host_tags;     // hash | 1 per host slot, 0 = empty
    const KeySlot* uri_slots;      // keyed by U (forward FNV-1a)
    const uint32_t* uri_tags;
    const uint32_t* lists;         // member lists
    const PortMin* port_mins;
    const GroupRec* groups;
    uint32_t host_mask;            // capacity - 1
    uint32_t uri_mask;
    int32_t n_groups;
    int32_t wildcard_slot;         // host slot of "*" or -1
    int32_t uri_star_slot;         // uri slot of "*" or -1
    int32_t has_uri_keys;          // any group with a hint-uri
    // the "*" record's meta (len_pm, a, b; HostRec) in the kernel argument,
    // so a miss picks the wildcard without a dependent load
    uint32_t wild_len_pm;
    int32_t wild_a, wild_b;
    // hint-uri key lengths present: bit l (l < 63) for length l, bit 63 for
    // any length >= 63 (the general search probes only those prefixes)
    uint32_t uri_len_lo, uri_len_hi;
};

struct HostsImage {
    const uint8_t* blob;
    const HostRec* recs;           // keyed by the exact qname (chunk hash); value in .a
    const uint32_t* tags;
    uint32_t mask;
    int32_t n;
};

// ---------------------------------------------------------------------------
// SSLContextHolder.choose (SNI -> certificate holder): one host-key table
// over every certificate name.  A plain name N is the key N with .a = the
// first holder listing it; a wildcard "*.S" is the key ".S" with .b = the
// first holder listing it.  A query matches plain names by the whole SNI
// and wildcards by the SNI's suffix from its first dot (the prefix before a
// wildcard suffix holds no dot), so two exact probes replace the linear
// scan over holders and names.
// ---------------------------------------------------------------------------
struct CertImage {
    HostsImage names;              // .a = plain-name holder, .b = wildcard holder (VC_NONE)
    int32_t n_holders;
};

// ---------------------------------------------------------------------------
// Mirror filters (vmirror/FilterConfig.java): one 160-byte record per
// FilterConfig in list order, read by all lanes of a wave at once through
// the scalar cache (the per-filter kernels; MirrorSwImage below for the
// bit-set ones).
// Each network is compiled to its per-input-family masked compare
// (common/netmatch.h NetMatch); MACs as the low 48 bits of a u64.
// ---------------------------------------------------------------------------
#define VC_MF_MAC_X  1u
#define VC_MF_MAC_Y  2u
#define VC_MF_NET_X  4u
#define VC_MF_NET_Y  8u
#define VC_MF_PORT_X 16u
#define VC_MF_PORT_Y 32u

struct MirrorNet {                 // common/netmatch.h NetMatch, 48 bytes
    uint32_t m6[4], r6[4];
    uint32_t low6, m4, r4, pad;
};

struct MirrorRec {                 // 160 bytes
    MirrorNet net_x, net_y;        // Network.contains per input family
    uint64_t mac_x, mac_y;
    int32_t origin, mirror, flags, transport, app;
    int32_t port_x0, port_x1, port_y0, port_y1;
    uint32_t pad[3];
};
static_assert(sizeof(MirrorRec) == 160, "MirrorRec layout");

struct MirrorImage {
    const MirrorRec* f;
    int32_t n;
};

// Mirror.switchPacket's filter step for one origin as bit sets (built at
// compile time for every origin with 1..64 filters whose networks compile
// to prefix ranges).  switchPacket reaches only matchEthernet and matchIp
// (Mirror.java:73-87), and every Network.contains projection onto one input
// family is a union of at most two key ranges (common/netmatch.h cases 1-5;
// case 4's lowBitsV6V4 gives ::a.b.c.d and ::ffff:a.b.c.d).  So the
// elementary intervals of all ranges of the origin's filters carry, per
// interval, the filters whose netX / netY contain it: one interval search
// per address, then the match of every filter at once in 64-bit masks.
// Keys: IPv4 as the big-endian u32; IPv6 as (hi, lo) big-endian u64 halves.
struct MirrorSwMac {               // a filter with a MAC (matchEthernet)
    uint64_t bit;                  // 1 << filter's position in the origin
    uint64_t mac_x, mac_y;
    uint32_t has_y, pad;
};

struct MirrorSwMir {               // filters whose FilterConfig.mirror is `bit`
    uint64_t filters;
    uint32_t bit, pad;
};

struct MirrorSwId {                // filters whose transport / app id is `id`
    uint64_t filters;
    int32_t id, pad;
};

struct MirrorSwImage {
    uint64_t all;                  // the origin's filters
    uint64_t has_x, has_y;         // NET_X / NET_Y
    uint64_t mac;                  // filters with a MAC_X
    int32_t n_mac, n_mir, nb4, nb6;
    int32_t lds, pad;              // the kernel copies the tables into LDS (both nb <= 48)
    const MirrorSwMac* macs;
    const MirrorSwMir* mirs;
    const uint32_t* b4;            // nb4 ascending interval starts, b4[0] = 0
    const uint64_t* p4;            // per interval: (xmask, ymask)
    const uint64_t* b6;            // nb6 ascending interval starts as (hi, lo), b6[0] = (0, 0)
    const uint64_t* p6;            // per interval: (xmask, ymask)
    // Mirror.mirror's transport and application levels (MirrorData items,
    // FilterConfig.java:57-94): protocol ids as sets, port ranges as
    // intervals over the key uint32(port) ^ 0x80000000 (Java's int order)
    uint64_t has_px, has_py;       // PORT_X / PORT_Y
    uint64_t any_t, any_a;         // transport / app -1: any
    int32_t n_t, n_a, nbp, pad2;
    const MirrorSwId* tids;
    const MirrorSwId* aids;
    const uint32_t* bp;            // nbp ascending port interval starts, bp[0] = 0
    const uint64_t* pp;            // per port interval: (xmask, ymask)
    // matchEthernet as sets (the items kernel): the distinct MACs of the
    // origin's filters, ascending, each with the filters whose macX / macY
    // it is
    uint64_t mac_both, mac_xonly;  // MAC_X with MAC_Y / MAC_X alone
    int32_t nbm, pad3;
    const uint64_t* bm;            // nbm ascending MACs (low 48 bits)
    const uint64_t* pm;            // per MAC: (xmask, ymask)
};

// ---------------------------------------------------------------------------
// ServerGroup source hashing (method == source): per group, three lists of
// server indices (all / IPv4 / IPv6 servers with weight > 0, in
// sourceReset's sort order).  view_off holds (offset, count) into order[]
// for [group][view 0..2]; order[] holds global server indices; healthy[]
// is per global server (a new snapshot per vc_servers_set_health);
// group_base[g] is the global index of group g's first server.  pick[]
// holds, per order[] entry, sourceHashGet's answer when hash % size lands
// there: the first healthy server from that position on, cyclically within
// the list, as an index within its group (-1: none healthy) -- rebuilt on
// the host with every health update (compile.cpp source_pick_table).
// view_pk is view_off packed for the kernels' LDS copy: [view][group] =
// offset << 8 | count, present (pk_ok) when every offset < 2^24 and every
// count < 256.
// ---------------------------------------------------------------------------
struct ServerImage {
    const uint32_t* view_off;      // 6 words per group
    const int32_t* order;
    const uint8_t* healthy;
    const int32_t* group_base;
    const int32_t* pick;
    const uint32_t* view_pk;       // 3 * n_groups words, or null
    int32_t n_groups;
    int32_t n_servers;
    int32_t pk_ok;
};

// compile.hpp -- host-side table compilers: reference rule lists -> the flat
// images of common/images.h (still in host memory; capi.cpp uploads them).
#pragma once

#include <cstdint>
#include <string>
#include <vector>

#include "vclassify.h"
#include "../common/images.h"
#include "../common/khash.h"

namespace vc {

struct AclFamilyBuilt {
    std::vector<uint32_t> bounds4;
    std::vector<uint64_t> bounds6;   // (hi, lo) pairs
    std::vector<uint32_t> desc;      // (x, y) pairs
    std::vector<uint32_t> rec;       // 4 words per interval (images.h AclFamilyImage.rec)
    std::vector<uint32_t> pieces;    // (port_start, value) pairs
    std::vector<uint32_t> dir4;      // v4: bucket directory (images.h AclFamilyImage)
    int32_t nb = 0;
    int32_t dir_bits = 0;
    int32_t v4_only = 0;             // v6 image: every rule a plain IPv4 network
};

struct AclBuilt {
    AclFamilyBuilt fam[2][2];        // [tcp/udp][v4/v6]
    std::vector<uint8_t> allow;
    int32_t n_tcp = 0, n_udp = 0, default_allow = 0;
};

// SecurityGroup lists -> ACL image.  Returns VC_OK or VC_EINVAL (bad rule).
int build_acl(const vc_acl_rule* tcp, int n_tcp, const vc_acl_rule* udp, int n_udp,
              int default_allow, AclBuilt* out);

// One list's IPv4 image at a fixed port (images.h AclPortImage): interval
// starts and the rule index (or VC_NONE) of each, equal neighbours merged.
void build_acl_port(const AclFamilyBuilt& f, uint32_t port, std::vector<uint32_t>* bounds,
                    std::vector<uint32_t>* value);

struct TrieBuilt {
    std::vector<uint32_t> nodes;     // root, 256-entry nodes, then one-prefix records
    int32_t root_bits = 16;
    int32_t key_bits = 32;
    int32_t n_rules = 0;
    int32_t n_nodes = 0;             // 16-entry units of nodes below the root
    int32_t n_records = 0;           // one-prefix records (images.h VC_ONE)
};

// One RouteTable family list (list order = priority) -> stride trie.
// root_bits: 16, 20 or 24; 0 picks default_root_bits(n, family).
int default_root_bits(int n, int family);
int build_trie(const vc_net* rules, int n, int family, TrieBuilt* out, int root_bits = 0);

struct KeySlotH {                    // host mirror of KeySlot (URI table)
    uint64_t hash;
    int32_t key_len;
    uint32_t key_off;
    int32_t a, b;
    uint32_t list_off, list_cnt;
};

// Host-name key table (hint-host keys, hosts map): tags + 64-byte records
// (common/images.h HostRec) + per-slot extension, keyed by vck::khash.
struct HostTableBuilt {
    std::vector<uint32_t> tags;
    std::vector<HostRec> recs;
    std::vector<HostExt> ext;
    int32_t n = 0;
    void init(size_t n_keys);
    // insert a key (not present yet); returns its slot
    uint32_t insert(const std::string& key, int32_t a, int32_t b, std::vector<uint8_t>* blob);
};

struct HintBuilt {
    std::vector<uint8_t> blob;
    HostTableBuilt host;
    std::vector<KeySlotH> uri_slots;
    std::vector<uint32_t> uri_tags;
    std::vector<uint32_t> lists;
    std::vector<int32_t> port_mins;      // (port, idx) pairs
    std::vector<int32_t> groups;         // 8 words per GroupRec
    int32_t n_groups = 0;
    int32_t wildcard_slot = -1, uri_star_slot = -1, has_uri_keys = 0;
    uint64_t uri_len_mask = 0;           // HintImage.uri_len_lo / _hi
};

int build_hints(const vc_group_annos* groups, int n, HintBuilt* out);

struct HostsBuilt {
    std::vector<uint8_t> blob;
    HostTableBuilt table;
    int32_t n = 0;
};

int build_hosts(const char* const* keys, const int32_t* key_lens, const int32_t* values, int n,
                HostsBuilt* out);

// SSLContextHolder certificate names -> CertImage table (see images.h).
// holder[i] in [0, n_holders) is the holder (add() order) listing names[i].
int build_certs(const char* const* names, const int32_t* name_lens, const int32_t* holder, int n,
                int n_holders, HostsBuilt* out);

// Mirror FilterConfig list -> MirrorRec records (images.h).
int build_mirror(const vc_mirror_filter* f, int n, std::vector<MirrorRec>* out);

// One origin's filters as MirrorSwImage bit sets (images.h); the image's
// pointers are left for the upload.  Returns false (nothing built) when the
// origin has no filter or more than 64, or when a network's projection is
// not a union of prefix ranges (a non-contiguous mask): switchPacket then
// takes the per-filter path.
struct MirrorSwBuilt {
    MirrorSwImage img{};
    std::vector<MirrorSwMac> macs;
    std::vector<MirrorSwMir> mirs;
    std::vector<uint32_t> b4, bp;
    std::vector<uint64_t> p4, b6, p6, pp, bm, pm;
    std::vector<MirrorSwId> tids, aids;
};
bool build_mirror_switch(const std::vector<MirrorRec>& recs, int32_t origin, MirrorSwBuilt* out);

// ServerGroup source-hash lists (ServerGroup.java:620-664), see ServerImage.
struct ServersBuilt {
    std::vector<uint32_t> view_off;      // 6 words per group
    std::vector<int32_t> order;
    std::vector<uint8_t> healthy;
    std::vector<int32_t> group_base;
    std::vector<int32_t> pick;           // per order[] entry (images.h ServerImage)
    std::vector<uint32_t> view_pk;       // [view][group] offset << 8 | count (when pk_ok)
    bool pk_ok = false;
    int32_t n_groups = 0;
    int32_t n_servers = 0;
};

int build_servers(const vc_server* servers, const int32_t* group_off, int n_groups,
                  ServersBuilt* out);

// ServerImage.pick for the lists of `b` under `healthy` (one byte per server)
void source_pick_table(const ServersBuilt& b, const uint8_t* healthy, std::vector<int32_t>* pick);

// Digest of a host-built image: 64-bit FNV-1a over its 8-byte words (each
// array prefixed by its length, scalars included), so ranks that replicate
// the tables can check they compiled the same image (vc_table_digest).
uint64_t digest(const AclBuilt& b);
uint64_t digest(const TrieBuilt& t4, const TrieBuilt& t6);
uint64_t digest(const HintBuilt& b);

// 32-bit FNV-1a over bytes, forwards and right-to-left (must match device code).
inline uint32_t fnv_fwd(const uint8_t* p, size_t n) {
    uint32_t h = 2166136261u;
    for (size_t i = 0; i < n; ++i) { h ^= p[i]; h *= 16777619u; }
    return h;
}
inline uint32_t fnv_rev(const uint8_t* p, size_t n) {
    uint32_t h = 2166136261u;
    for (size_t i = n; i-- > 0;) { h ^= p[i]; h *= 16777619u; }
    return h;
}

}  // namespace vc

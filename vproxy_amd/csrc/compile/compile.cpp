// compile.cpp -- rule lists -> device table images (see common/images.h).
#include "compile.hpp"

#include <algorithm>
#include <cstring>
#include <map>
#include <set>
#include <string>
#include <thread>
#include <unordered_map>

#include "../common/images.h"
#include "../common/netmatch.h"
#include "../host/net.hpp"

#ifndef VC_ACL_DIR_MAX
#define VC_ACL_DIR_MAX 16
#endif
#ifndef VC_ACL_DIR_EXTRA
#define VC_ACL_DIR_EXTRA 2
#endif

namespace vc {

using u128 = unsigned __int128;

namespace {

u128 key128(const uint8_t* b, int len) {   // big-endian bytes -> integer
    u128 k = 0;
    for (int i = 0; i < len; ++i) k = (k << 8) | b[i];
    return k;
}

// A network must be what Network(String)/NetworkHandle produce: a standard
// mask (parseMask(m) bytes) and validNetwork(ip, mask).
bool standard_net(const vc_net& n) {
    if (n.ip_len != 4 && n.ip_len != 16) return false;
    if (n.mask_len != 4 && n.mask_len != 16) return false;
    int m = mask_int(n.mask, n.mask_len);
    uint8_t ref[16];
    int ml = parse_mask(m, ref);
    if (ml != n.mask_len || std::memcmp(ref, n.mask, ml) != 0) return false;
    return valid_network(n.ip, n.ip_len, n.mask, n.mask_len);
}

u128 low_ones(int bits) {   // 2^bits - 1 (bits in 0..128)
    if (bits <= 0) return 0;
    if (bits >= 128) return ~(u128)0;
    return (((u128)1) << bits) - 1;
}

struct Iv {
    u128 lo, hi;   // inclusive
    int rule;
};

// Projection of one SecurityGroupRule network onto an input family, exactly
// as Network.maskMatch (Network.java:183-278) decides membership
// (SURVEY.md Appendix A.1).  Appends 0, 1 or 2 intervals.
void project(const vc_net& n, int family, int rule, std::vector<Iv>* out) {
    int m = mask_int(n.mask, n.mask_len);
    if (family == 0) {                       // IPv4 input (4 bytes)
        if (n.ip_len == 4) {                 // case 5: plain v4 prefix
            u128 lo = key128(n.ip, 4);
            out->push_back({lo, lo | low_ones(32 - m), rule});
        } else if (n.mask_len == 16) {       // case 3: low 32 bits + lowBitsV6V4(rule)
            const uint8_t* r = n.ip;
            for (int i = 0; i < 10; ++i)
                if (r[i] != 0) return;
            if (!((r[10] == 0 && r[11] == 0) || (r[10] == 0xFF && r[11] == 0xFF))) return;
            int m4 = m > 96 ? m - 96 : 0;
            u128 lo = key128(r + 12, 4);
            out->push_back({lo, lo | low_ones(32 - m4), rule});
        }
        // v6 rule with a 4-byte mask: case 2, never matches IPv4 input
    } else {                                 // IPv6 input (16 bytes)
        if (n.ip_len == 4) {                 // case 4: tail compare + lowBitsV6V4(input)
            u128 lo = key128(n.ip, 4);
            u128 span = low_ones(32 - m);
            out->push_back({lo, lo | span, rule});                      // ::a.b.c.d
            u128 mapped = ((u128)0xFFFF) << 32;
            out->push_back({mapped | lo, mapped | lo | span, rule});     // ::ffff:a.b.c.d
        } else {                             // cases 1 and 5: plain v6 prefix
            u128 lo = key128(n.ip, 16);
            out->push_back({lo, lo | low_ones(128 - m), rule});
        }
    }
}

struct PortRule {
    int rule, plo, phi;
};

// port -> min rule index over `act` (ascending rule order, truncated at the
// first full-range rule).  Emits (port_start, value) pairs.
void port_function(const std::vector<PortRule>& act, std::vector<uint32_t>* fn) {
    fn->clear();
    if (act.empty()) return;
    std::vector<std::pair<int, int>> ev;   // (port, +rule+1 / -(rule+1))
    ev.reserve(act.size() * 2);
    for (auto& p : act) {
        ev.push_back({p.plo, p.rule + 1});
        if (p.phi < 65535) ev.push_back({p.phi + 1, -(p.rule + 1)});
    }
    std::sort(ev.begin(), ev.end());
    std::set<int> live;
    uint32_t cur = 0xFFFFFFFFu;
    size_t k = 0;
    if (ev[0].first != 0) {
        fn->push_back(0);
        fn->push_back(VC_NONE);
        cur = VC_NONE;
    }
    while (k < ev.size()) {
        int port = ev[k].first;
        for (; k < ev.size() && ev[k].first == port; ++k) {
            if (ev[k].second > 0) live.insert(ev[k].second - 1);
            else live.erase(-ev[k].second - 1);
        }
        uint32_t v = live.empty() ? VC_NONE : static_cast<uint32_t>(*live.begin());
        if (v != cur) {
            fn->push_back(static_cast<uint32_t>(port));
            fn->push_back(v);
            cur = v;
        }
    }
}

void build_acl_family(const vc_acl_rule* rules, int n, int family, AclFamilyBuilt* out) {
    std::vector<Iv> ivs;
    std::vector<PortRule> pr(n);
    for (int i = 0; i < n; ++i) {
        int plo = std::max(rules[i].min_port, 0);
        int phi = std::min(rules[i].max_port, 65535);
        pr[i] = {i, plo, phi};
        if (plo > phi) continue;             // the port test can never pass
        project(rules[i].net, family, i, &ivs);
    }
    const u128 kmax = family == 0 ? low_ones(32) : ~(u128)0;
    std::vector<u128> pts;
    pts.reserve(ivs.size() * 2 + 1);
    pts.push_back(0);
    for (auto& iv : ivs) {
        pts.push_back(iv.lo);
        if (iv.hi != kmax) pts.push_back(iv.hi + 1);
    }
    std::sort(pts.begin(), pts.end());
    pts.erase(std::unique(pts.begin(), pts.end()), pts.end());
    const size_t K = pts.size();
    // events per elementary interval index
    std::vector<std::pair<uint32_t, int>> ev;   // (index, +rule+1 / -(rule+1))
    ev.reserve(ivs.size() * 2);
    for (auto& iv : ivs) {
        uint32_t s = static_cast<uint32_t>(std::lower_bound(pts.begin(), pts.end(), iv.lo) - pts.begin());
        ev.push_back({s, iv.rule + 1});
        if (iv.hi != kmax) {
            uint32_t e = static_cast<uint32_t>(
                std::lower_bound(pts.begin(), pts.end(), iv.hi + 1) - pts.begin());
            ev.push_back({e, -(iv.rule + 1)});
        }
    }
    std::sort(ev.begin(), ev.end());
    std::set<int> active;
    std::map<std::vector<uint32_t>, uint32_t> memo;
    std::vector<PortRule> act;
    std::vector<uint32_t> fn;
    size_t k = 0;
    uint32_t px = 0xFFFFFFFFu, py = 0xFFFFFFFFu;
    for (size_t j = 0; j < K; ++j) {
        for (; k < ev.size() && ev[k].first == j; ++k) {
            if (ev[k].second > 0) active.insert(ev[k].second - 1);
            else active.erase(-ev[k].second - 1);
        }
        act.clear();
        for (int r : active) {
            act.push_back(pr[r]);
            if (pr[r].plo == 0 && pr[r].phi == 65535) break;
        }
        uint32_t x, y;
        if (act.empty()) {
            x = VC_NONE;
            y = 0;
        } else if (act[0].plo == 0 && act[0].phi == 65535) {
            x = static_cast<uint32_t>(act[0].rule);
            y = 0;
        } else {
            port_function(act, &fn);
            if (fn.size() == 2) {
                x = fn[1];
                y = 0;
            } else {
                auto it = memo.find(fn);
                if (it == memo.end()) {
                    uint32_t off = static_cast<uint32_t>(out->pieces.size() / 2);
                    out->pieces.insert(out->pieces.end(), fn.begin(), fn.end());
                    it = memo.emplace(fn, off).first;
                }
                x = it->second;
                y = static_cast<uint32_t>(fn.size() / 2);
            }
        }
        if (x == px && y == py) continue;    // merge with the previous interval
        px = x;
        py = y;
        if (family == 0) {
            out->bounds4.push_back(static_cast<uint32_t>(pts[j]));
        } else {
            out->bounds6.push_back(static_cast<uint64_t>(pts[j] >> 64));
            out->bounds6.push_back(static_cast<uint64_t>(pts[j]));
        }
        out->desc.push_back(x);
        out->desc.push_back(y);
    }
    out->nb = static_cast<int32_t>(out->desc.size() / 2);
    // one 16-byte record per interval: up to four port pieces inline, else
    // (x, y) of desc for the pieces array (images.h AclFamilyImage.rec)
    out->rec.assign(size_t(out->nb) * 4, 0u);
    auto v16 = [](uint32_t v) { return v == VC_NONE ? 0xFFFFu : v; };
    for (int32_t j = 0; j < out->nb; ++j) {
        const uint32_t x = out->desc[2 * j], y = out->desc[2 * j + 1];
        uint32_t* r = &out->rec[size_t(j) * 4];
        bool inl = y <= 4;
        const uint32_t k = y == 0 ? 1 : y;
        for (uint32_t i = 0; inl && i < k; ++i) {
            const uint32_t v = y == 0 ? x : out->pieces[2 * (x + i) + 1];
            inl = v == VC_NONE || v < 0xFFFFu;
        }
        if (!inl) {
            r[0] = 0xFFu << 16;
            r[1] = x;
            r[2] = y;
            continue;
        }
        if (y == 0) {
            r[0] = v16(x) | (1u << 16);
            continue;
        }
        r[0] = v16(out->pieces[2 * x + 1]) | (k << 16);     // piece 0 starts at port 0
        for (uint32_t i = 1; i < k; ++i)
            r[i] = (out->pieces[2 * (x + i)] << 16) | v16(out->pieces[2 * (x + i) + 1]);
    }
    if (family == 0 && out->nb > 16 && out->nb < 65536) {
        // bucket directory over the key's top D bits: entry t = s(t) |
        // (s(t + 1) - s(t)) << 16, s(t) = last j with bounds4[j] <= t << (32 - D).
        // D: 2^D >= 4 nb (VC_ACL_DIR_EXTRA = 2), at most 16 bits (256 KB), so
        // most buckets hold no boundary and a lookup is the directory load and
        // the record load (12 bits, 1.2 boundaries per bucket at 5k intervals,
        // left one or two boundary loads between them)
        int d = 4;
        while ((1 << d) < out->nb && d < VC_ACL_DIR_MAX) ++d;
        d = std::min(d + VC_ACL_DIR_EXTRA, VC_ACL_DIR_MAX);
        const auto& b = out->bounds4;
        auto s = [&](uint64_t key) {
            return uint32_t(std::upper_bound(b.begin(), b.end(), key,
                                             [](uint64_t k, uint32_t x) { return k < x; }) -
                            b.begin()) - 1;
        };
        out->dir_bits = d;
        out->dir4.resize(size_t(1) << d);
        for (uint32_t t = 0; t < (1u << d); ++t) {
            const uint32_t s0 = s(uint64_t(t) << (32 - d));
            const uint32_t s1 = t + 1 < (1u << d) ? s(uint64_t(t + 1) << (32 - d))
                                                  : uint32_t(out->nb - 1);
            out->dir4[t] = s0 | ((s1 - s0) << 16);
        }
    }
}

}  // namespace

int build_acl(const vc_acl_rule* tcp, int n_tcp, const vc_acl_rule* udp, int n_udp,
              int default_allow, AclBuilt* out) {
    if (n_tcp < 0 || n_udp < 0) return VC_EINVAL;
    for (int i = 0; i < n_tcp; ++i)
        if (!standard_net(tcp[i].net)) return VC_EINVAL;
    for (int i = 0; i < n_udp; ++i)
        if (!standard_net(udp[i].net)) return VC_EINVAL;
    *out = AclBuilt{};
    out->n_tcp = n_tcp;
    out->n_udp = n_udp;
    out->default_allow = default_allow ? 1 : 0;
    for (int i = 0; i < n_tcp; ++i) out->allow.push_back(tcp[i].allow ? 1 : 0);
    for (int i = 0; i < n_udp; ++i) out->allow.push_back(udp[i].allow ? 1 : 0);
    if (out->allow.empty()) out->allow.push_back(0);
    // four independent images: build them concurrently
    std::thread th[4];
    for (int l = 0; l < 2; ++l)
        for (int f = 0; f < 2; ++f)
            th[l * 2 + f] = std::thread(build_acl_family, l == 0 ? tcp : udp, l == 0 ? n_tcp : n_udp,
                                        f, &out->fam[l][f]);
    for (auto& t : th) t.join();
    // Network.maskMatch (Network.java:246-277): an IPv6 input matches an
    // IPv4 rule only through its last four bytes, and only when
    // Utils.lowBitsV6V4 holds (bytes 0-9 zero, bytes 10-11 both 00 or both
    // FF).  With no other kind of rule in the list, its v6 image classifies
    // such a key like the v4 image classifies the low 32 bits, and every
    // other key as no rule: the kernels then skip the 128-bit search.
    for (int l = 0; l < 2; ++l) {
        const vc_acl_rule* r = l == 0 ? tcp : udp;
        const int n = l == 0 ? n_tcp : n_udp;
        int only4 = 1;
        for (int i = 0; i < n && only4; ++i) only4 = r[i].net.ip_len == 4 && r[i].net.mask_len == 4;
        out->fam[l][1].v4_only = only4;
    }
    return VC_OK;
}

// ---------------------------------------------------------------------------
// Route trie
// ---------------------------------------------------------------------------
// 24 bits above 4096 rules for both families: a 20-bit root measured 2.74
// L2 misses per C5 packet against 2.19 and a 15 % slower pipeline kernel
// (profiles/r03_ab_root.jsonl).
int default_root_bits(int n, int /*family*/) { return n > 4096 ? 24 : 16; }

int build_trie(const vc_net* rules, int n, int family, TrieBuilt* out, int root_bits) {
    *out = TrieBuilt{};
    out->key_bits = family == 0 ? 32 : 128;
    out->n_rules = n;
    if (root_bits == 0) root_bits = default_root_bits(n, family);
    if (root_bits != 16 && root_bits != 20 && root_bits != 24) return VC_EINVAL;
    out->root_bits = root_bits;
    const int rb = out->root_bits;
    struct P {
        u128 key;   // left-aligned in 128 bits
        int len;
        uint32_t idx;
    };
    std::vector<P> ps;
    ps.reserve(n);
    for (int i = 0; i < n; ++i) {
        const vc_net& r = rules[i];
        if (!standard_net(r)) return VC_EINVAL;
        if ((family == 0) != (r.ip_len == 4)) return VC_EINVAL;
        int len = mask_int(r.mask, r.mask_len);
        u128 k = key128(r.ip, r.ip_len);
        if (family == 0) k <<= 96;
        ps.push_back({k, len, static_cast<uint32_t>(i)});
    }
    std::stable_sort(ps.begin(), ps.end(), [](const P& a, const P& b) { return a.len < b.len; });
    const size_t root = size_t(1) << rb;
    out->nodes.assign(root, VC_NONE);
    size_t split = 0;
    while (split < ps.size() && ps[split].len <= rb) ++split;
    // 1) prefixes no longer than the root stride: paint root ranges with min,
    //    the root split into slices painted concurrently.
    {
        unsigned T = std::max(1u, std::min(16u, std::thread::hardware_concurrency()));
        if (split < 64) T = 1;
        std::vector<std::thread> th;
        uint32_t* nodes = out->nodes.data();
        for (unsigned t = 0; t < T; ++t) {
            size_t s0 = root * t / T, s1 = root * (t + 1) / T;
            th.emplace_back([&, s0, s1]() {
                for (size_t i = 0; i < split; ++i) {
                    size_t a = static_cast<size_t>(ps[i].key >> (128 - rb));
                    size_t b = a + (size_t(1) << (rb - ps[i].len));
                    a = std::max(a, s0);
                    b = std::min(b, s1);
                    const uint32_t v = ps[i].idx;
                    for (size_t e = a; e < b; ++e)
                        if (v < nodes[e]) nodes[e] = v;
                }
            });
        }
        for (auto& t : th) t.join();
    }
    // 2) a root slot whose subtree holds exactly one longer prefix P (len <=
    //    64) gets a one-prefix record instead of a chain of nodes: match ->
    //    min(P's index, the slot's inherited value), miss -> inherited.  One
    //    16-byte gather replaces up to five dependent node gathers (IPv6
    //    /32-/64 prefixes under a 24-bit root).  The miss value is stored in
    //    24 bits, so records need fewer than 0xFFFFFF rules.
    std::unordered_map<uint32_t, uint32_t> per_slot;      // root slot -> long prefixes
    per_slot.reserve(ps.size() - split);
    for (size_t i = split; i < ps.size(); ++i)
        ++per_slot[static_cast<uint32_t>(ps[i].key >> (128 - rb))];
    const bool records_ok = n < 0xFFFFFF;
    std::vector<uint32_t> rec_words, rec_slots;
    // 3) the other longer prefixes in ascending length: walk/create nodes
    //    (2^trie_stride entries, allocated in 16-entry units); a new node
    //    inherits its parent entry's value (leaf pushing).
    uint32_t n_children = 0;
    for (size_t i = split; i < ps.size(); ++i) {
        const P& p = ps[i];
        size_t entry = static_cast<size_t>(p.key >> (128 - rb));
        if (records_ok && p.len <= 64 && per_slot[static_cast<uint32_t>(entry)] == 1) {
            const uint32_t inh = out->nodes[entry];          // a value: no other long prefix here
            const uint64_t khi = static_cast<uint64_t>(p.key >> 64);
            rec_words.push_back(static_cast<uint32_t>(khi >> 32));
            rec_words.push_back(static_cast<uint32_t>(khi));
            rec_words.push_back(std::min(p.idx, inh));
            rec_words.push_back((inh == VC_NONE ? 0xFFFFFFu : inh) | (uint32_t(p.len) << 24));
            rec_slots.push_back(static_cast<uint32_t>(entry));
            continue;
        }
        int bits = rb;
        for (;;) {
            uint32_t v = out->nodes[entry];
            uint32_t child;
            const int st = 8 - (bits & 7);                   // route_dev.h trie_stride
            const uint32_t width = 1u << st;
            if (v & VC_PTR) {
                child = v & ~VC_PTR;
            } else {
                child = n_children;
                n_children += width / 16;
                if (n_children >= VC_ONE) return VC_ENOMEM;  // ids at VC_ONE and up would read as records
                out->nodes.resize(out->nodes.size() + width, v);
                out->nodes[entry] = VC_PTR | child;
            }
            size_t base = root + size_t(child) * 16;
            int nb = bits + st;
            uint32_t sub = static_cast<uint32_t>(p.key >> (128 - nb)) & (width - 1);
            if (p.len <= nb) {
                uint32_t cnt = 1u << (nb - p.len);
                for (uint32_t e = sub; e < sub + cnt; ++e)
                    if (p.idx < out->nodes[base + e]) out->nodes[base + e] = p.idx;
                break;
            }
            entry = base + sub;
            bits = nb;
        }
    }
    out->n_nodes = static_cast<int32_t>(n_children);   // 16-entry units
    // records after the nodes (the node array is a multiple of 4 words, so
    // they are 16-byte aligned); an entry addresses them in 16-byte units
    const size_t base = out->nodes.size() / 4;
    if (base + rec_slots.size() > VC_ONE_MAX) return VC_ENOMEM;
    for (size_t k = 0; k < rec_slots.size(); ++k)
        out->nodes[rec_slots[k]] = VC_PTR | VC_ONE | static_cast<uint32_t>(base + k);
    out->nodes.insert(out->nodes.end(), rec_words.begin(), rec_words.end());
    out->n_records = static_cast<int32_t>(rec_slots.size());
    return VC_OK;
}

// ---------------------------------------------------------------------------
// Upstream hints
// ---------------------------------------------------------------------------
namespace {

uint32_t pow2_cap(size_t n) {
    uint32_t c = 16;
    while (c < n * 2) c <<= 1;
    return c;
}

// Strings go into the blob 16-byte aligned and zero padded to a multiple of
// 16, so the device compares keys one uint4 at a time (hint_dev.h key_eq).
uint32_t append_blob(std::vector<uint8_t>* blob, const char* s, int len) {
    blob->resize((blob->size() + 15) & ~size_t(15), 0);
    uint32_t off = static_cast<uint32_t>(blob->size());
    blob->insert(blob->end(), s, s + len);
    blob->resize((blob->size() + 15) & ~size_t(15), 0);
    return off;
}

// insert into an open-addressing table (slots + tags); returns the slot index.
// Linear probing that starts at the 4-slot group of the hash, so a lookup
// reads one 16-byte tag group per step (hint_dev.h probe).
uint32_t table_insert(std::vector<KeySlotH>* t, std::vector<uint32_t>* tags, uint32_t h,
                      const KeySlotH& v) {
    uint32_t mask = static_cast<uint32_t>(t->size() - 1);
    uint32_t s = h & mask & ~3u;
    while ((*t)[s].key_len != -1) s = (s + 1) & mask;
    (*t)[s] = v;
    (*tags)[s] = h | 1u;
    return s;
}

}  // namespace

void HostTableBuilt::init(size_t n_keys) {
    const uint32_t cap = pow2_cap(n_keys);
    tags.assign(cap, 0);
    HostRec empty{};
    recs.assign(cap, empty);
    ext.assign(cap, HostExt{0, 0, 0, 0});
    n = 0;
}

uint32_t HostTableBuilt::insert(const std::string& k, int32_t a, int32_t b,
                                std::vector<uint8_t>* blob) {
    const uint32_t h = vck::khash(reinterpret_cast<const uint8_t*>(k.data()),
                                  static_cast<int>(k.size()));
    const uint32_t mask = static_cast<uint32_t>(tags.size() - 1);
    uint32_t s = h & mask & ~3u;
    while (tags[s] != 0) s = (s + 1) & mask;
    tags[s] = h | 1u;
    HostRec& r = recs[s];
    r = HostRec{};
    r.len_pm = static_cast<uint32_t>(k.size());
    r.a = a;
    r.b = b;
    r.key_off = append_blob(blob, k.data(), static_cast<int>(k.size()));
    std::memcpy(r.key, k.data(), std::min<size_t>(k.size(), VC_REC_INLINE));
    ++n;
    return s;
}

// String.length() of the Java string whose UTF-8 (WTF-8 for unpaired
// surrogates) bytes are s: one UTF-16 unit per code point, two for a
// supplementary one (a 4-byte sequence) -- the uriLevel of Hint.matchLevel
// (Hint.java:146-150) counts these, not bytes.
static int32_t utf16_units(const uint8_t* s, int n) {
    int32_t u = 0;
    for (int i = 0; i < n; ++i) {
        if ((s[i] & 0xC0) != 0x80) ++u;        // every byte that starts a code point
        if (s[i] >= 0xF0) ++u;                  // 4-byte sequence: a surrogate pair
    }
    return u;
}

int build_hints(const vc_group_annos* groups, int n, HintBuilt* out) {
    *out = HintBuilt{};
    out->n_groups = n;
    struct KeyAcc {
        std::vector<uint32_t> members;
        std::map<int32_t, int32_t> port_min;   // distinct nonzero hint-port -> min index
        int32_t a = -1, b = -1;
        bool any_uri = false;                  // a member has a hint-uri
    };
    std::map<std::string, KeyAcc> hostk, urik;
    std::vector<std::string> host_order, uri_order;
    out->groups.reserve(size_t(n) * 8);
    for (int g = 0; g < n; ++g) {
        // Hint.matchLevel merge (Hint.java:108-118): first non-null host,
        // first non-zero port, first non-null uri over [handle, group].
        const vc_annos* as[2] = {&groups[g].handle, &groups[g].group};
        const char* H = nullptr; int Hn = 0; int P = 0; const char* U = nullptr; int Un = 0;
        for (const vc_annos* a : as) {
            if (!H && a->host) { H = a->host; Hn = a->host_len; }
            if (P == 0) P = a->port;
            if (!U && a->uri) { U = a->uri; Un = a->uri_len; }
        }
        if ((H && Hn < 0) || (U && Un < 0)) return VC_EINVAL;
        int32_t rec[8] = {-1, 0, -1, 0, P, (H || P != 0 || U) ? 1 : 0, 0, 0};
        if (H) { rec[0] = Hn; rec[1] = static_cast<int32_t>(append_blob(&out->blob, H, Hn)); }
        if (U) {
            rec[2] = Un;
            rec[3] = static_cast<int32_t>(append_blob(&out->blob, U, Un));
            rec[6] = utf16_units(reinterpret_cast<const uint8_t*>(U), Un);
        }
        out->groups.insert(out->groups.end(), rec, rec + 8);
        if (H) {
            std::string k(H, Hn);
            auto it = hostk.find(k);
            if (it == hostk.end()) {
                host_order.push_back(k);
                it = hostk.emplace(k, KeyAcc{}).first;
            }
            KeyAcc& acc = it->second;
            acc.members.push_back(static_cast<uint32_t>(g));
            if (U) acc.any_uri = true;
            if (acc.a < 0) acc.a = g;
            if (P == 0 && acc.b < 0) acc.b = g;
            if (P != 0 && !acc.port_min.count(P)) acc.port_min[P] = g;
        }
        if (U) {
            out->has_uri_keys = 1;
            out->uri_len_mask |= uint64_t(1) << (Un < 63 ? Un : 63);
            std::string k(U, Un);
            auto it = urik.find(k);
            if (it == urik.end()) {
                uri_order.push_back(k);
                it = urik.emplace(k, KeyAcc{}).first;
            }
            it->second.members.push_back(static_cast<uint32_t>(g));
        }
    }
    KeySlotH empty{0, -1, 0, -1, -1, 0, 0};
    for (auto& k : host_order)
        if (k.size() > VC_REC_LEN) return VC_EINVAL;     // the record's length bits
    out->host.init(host_order.size());
    out->uri_slots.assign(pow2_cap(uri_order.size()), empty);
    out->uri_tags.assign(out->uri_slots.size(), 0);
    for (auto& k : host_order) {
        KeyAcc& acc = hostk[k];
        const uint32_t slot = out->host.insert(
            k, acc.a, acc.b < 0 ? static_cast<int32_t>(VC_NONE) : acc.b, &out->blob);
        HostExt& x = out->host.ext[slot];
        x.list_off = static_cast<uint32_t>(out->lists.size());
        x.list_cnt = static_cast<uint32_t>(acc.members.size());
        out->lists.insert(out->lists.end(), acc.members.begin(), acc.members.end());
        x.pm_off = static_cast<uint32_t>(out->port_mins.size() / 2);
        x.pm_cnt = static_cast<uint32_t>(acc.port_min.size());
        if (!acc.port_min.empty()) out->host.recs[slot].len_pm |= VC_REC_HAS_PM;
        if (acc.any_uri) out->host.recs[slot].len_pm |= VC_REC_ANYURI;
        if (acc.any_uri && acc.members.size() > 1) out->host.recs[slot].len_pm |= VC_REC_SPLIT;
        for (auto& pm : acc.port_min) {
            out->port_mins.push_back(pm.first);
            out->port_mins.push_back(pm.second);
        }
        if (k == "*") out->wildcard_slot = static_cast<int32_t>(slot);
    }
    for (auto& k : uri_order) {
        KeyAcc& acc = urik[k];
        KeySlotH s{};
        s.hash = fnv_fwd(reinterpret_cast<const uint8_t*>(k.data()), k.size());
        s.key_len = static_cast<int32_t>(k.size());
        s.key_off = append_blob(&out->blob, k.data(), static_cast<int>(k.size()));
        s.a = acc.members.empty() ? -1 : static_cast<int32_t>(acc.members[0]);
        s.b = -1;
        s.list_off = static_cast<uint32_t>(out->lists.size());
        s.list_cnt = static_cast<uint32_t>(acc.members.size());
        out->lists.insert(out->lists.end(), acc.members.begin(), acc.members.end());
        uint32_t slot = table_insert(&out->uri_slots, &out->uri_tags, uint32_t(s.hash), s);
        if (k == "*") out->uri_star_slot = static_cast<int32_t>(slot);
    }
    if (out->blob.empty()) out->blob.assign(16, 0);
    if (out->lists.empty()) out->lists.push_back(0);
    if (out->port_mins.empty()) { out->port_mins.push_back(0); out->port_mins.push_back(0); }
    if (out->groups.empty()) out->groups.assign(6, 0);
    return VC_OK;
}

int build_hosts(const char* const* keys, const int32_t* key_lens, const int32_t* values, int n,
                HostsBuilt* out) {
    *out = HostsBuilt{};
    std::unordered_map<std::string, int> seen;
    std::vector<int> order;
    for (int i = 0; i < n; ++i) {
        if (key_lens[i] < 0 || (!keys[i] && key_lens[i] > 0)) return VC_EINVAL;
        if (uint32_t(key_lens[i]) > VC_REC_LEN) return VC_EINVAL;
        std::string k(keys[i] ? keys[i] : "", key_lens[i]);
        if (seen.count(k)) continue;     // first key wins
        seen.emplace(k, i);
        order.push_back(i);
    }
    out->table.init(order.size());
    for (int i : order)
        out->table.insert(std::string(keys[i] ? keys[i] : "", key_lens[i]), values[i], 0,
                          &out->blob);
    out->n = out->table.n;
    if (out->blob.empty()) out->blob.assign(16, 0);
    return VC_OK;
}

// SSLContextHolder.compare (SSLContextHolder.java:171-186): "*.S" matches an
// SNI ending in ".S" whose remaining prefix is non-empty and dot-free; any
// other name matches by equality.  choose() returns the first holder with
// any matching name, so each key keeps the minimum holder per kind.
int build_certs(const char* const* names, const int32_t* name_lens, const int32_t* holder, int n,
                int n_holders, HostsBuilt* out) {
    *out = HostsBuilt{};
    std::unordered_map<std::string, std::pair<int32_t, int32_t>> keys;   // key -> (plain, wild)
    std::vector<std::string> order;
    for (int i = 0; i < n; ++i) {
        if (name_lens[i] < 0 || (!names[i] && name_lens[i] > 0)) return VC_EINVAL;
        if (holder[i] < 0 || holder[i] >= n_holders) return VC_EINVAL;
        if (uint32_t(name_lens[i]) > VC_REC_LEN) return VC_EINVAL;
        std::string k(names[i] ? names[i] : "", name_lens[i]);
        const bool wild = k.size() >= 2 && k[0] == '*' && k[1] == '.';
        if (wild) k.erase(0, 1);
        auto it = keys.find(k);
        if (it == keys.end()) {
            it = keys.emplace(k, std::make_pair(int32_t(VC_NONE), int32_t(VC_NONE))).first;
            order.push_back(k);
        }
        int32_t& v = wild ? it->second.second : it->second.first;
        v = std::min(v, holder[i]);
    }
    out->table.init(order.size());
    for (const auto& k : order) {
        const auto& v = keys[k];
        out->table.insert(k, v.first, v.second, &out->blob);
    }
    out->n = out->table.n;
    if (out->blob.empty()) out->blob.assign(16, 0);
    return VC_OK;
}

void build_acl_port(const AclFamilyBuilt& f, uint32_t port, std::vector<uint32_t>* bounds,
                    std::vector<uint32_t>* value) {
    bounds->clear();
    value->clear();
    for (int32_t j = 0; j < f.nb; ++j) {
        // desc (x, y): y == 0 -> x; else pieces[x .. x + y) as (port_start,
        // value), ascending, the first starting at port 0
        const uint32_t x = f.desc[2 * size_t(j)], y = f.desc[2 * size_t(j) + 1];
        uint32_t v = x;
        if (y) {
            v = f.pieces[2 * size_t(x) + 1];
            for (uint32_t k = 1; k < y && f.pieces[2 * size_t(x + k)] <= port; ++k)
                v = f.pieces[2 * size_t(x + k) + 1];
        }
        if (!value->empty() && value->back() == v) continue;
        bounds->push_back(f.bounds4[size_t(j)]);
        value->push_back(v);
    }
    if (bounds->empty()) {                  // no interval at all: one of no rule
        bounds->push_back(0);
        value->push_back(VC_NONE);
    }
}

// Mirror filters.  Java rejects min > max while parsing the config
// (Mirror.java:581-582, 590-591); mirror indices are bits of the result.
int build_mirror(const vc_mirror_filter* f, int n, std::vector<MirrorRec>* out) {
    out->assign(size_t(n), MirrorRec{});
    auto mac = [](const uint8_t* b) {
        uint64_t v = 0;
        for (int k = 0; k < 6; ++k) v |= uint64_t(b[k]) << (8 * k);
        return v;
    };
    auto len_ok = [](int l) { return l == 4 || l == 16; };
    auto net = [](const vc_net& v, MirrorNet* o) {
        const vcn::NetMatch m = vcn::net_matcher(vcn::addr_of(v.ip, v.ip_len),
                                                 vcn::addr_of(v.mask, v.mask_len));
        static_assert(sizeof(MirrorNet) == sizeof(vcn::NetMatch), "NetMatch layout");
        std::memcpy(o, &m, sizeof m);
    };
    for (int i = 0; i < n; ++i) {
        const vc_mirror_filter& s = f[i];
        MirrorRec& r = (*out)[size_t(i)];
        if (s.mirror < 0 || s.mirror > 63) return VC_EINVAL;
        if (s.has_net_x && (!len_ok(s.net_x.ip_len) || !len_ok(s.net_x.mask_len))) return VC_EINVAL;
        if (s.has_net_y && (!len_ok(s.net_y.ip_len) || !len_ok(s.net_y.mask_len))) return VC_EINVAL;
        if (s.has_port_x && s.port_x[0] > s.port_x[1]) return VC_EINVAL;
        if (s.has_port_y && s.port_y[0] > s.port_y[1]) return VC_EINVAL;
        r.origin = s.origin;
        r.mirror = s.mirror;
        r.flags = (s.has_mac_x ? VC_MF_MAC_X : 0) | (s.has_mac_y ? VC_MF_MAC_Y : 0) |
                  (s.has_net_x ? VC_MF_NET_X : 0) | (s.has_net_y ? VC_MF_NET_Y : 0) |
                  (s.has_port_x ? VC_MF_PORT_X : 0) | (s.has_port_y ? VC_MF_PORT_Y : 0);
        r.mac_x = mac(s.mac_x);
        r.mac_y = mac(s.mac_y);
        if (s.has_net_x) net(s.net_x, &r.net_x);
        if (s.has_net_y) net(s.net_y, &r.net_y);
        r.transport = s.transport;
        r.app = s.app;
        r.port_x0 = s.port_x[0];
        r.port_x1 = s.port_x[1];
        r.port_y0 = s.port_y[0];
        r.port_y1 = s.port_y[1];
    }
    return VC_OK;
}

namespace {
uint32_t be32(uint32_t w) { return __builtin_bswap32(w); }

// the key of left-aligned bytes held as little-endian words (netmatch.h)
u128 be128(const uint32_t w[4]) {
    return (u128(be32(w[0])) << 96) | (u128(be32(w[1])) << 64) | (u128(be32(w[2])) << 32) |
           u128(be32(w[3]));
}

// (k & m) == r as the range [r, r | ~m] when m is a run of high ones;
// false when m is not (the per-filter path keeps such a network)
template <class T>
bool prefix_range(T m, T r, std::vector<std::pair<T, T>>* out) {
    const T inv = T(~m);
    if (inv & T(inv + 1)) return false;                    // not a prefix mask
    if ((r & inv) == 0) out->push_back({r, T(r | inv)});   // else: matches nothing
    return true;
}

// Network.contains projected onto 4- and 16-byte inputs (netmatch.h
// NetMatch) as key ranges
bool net_ranges(const MirrorNet& n, std::vector<std::pair<uint32_t, uint32_t>>* r4,
                std::vector<std::pair<u128, u128>>* r6) {
    if (!prefix_range<uint32_t>(be32(n.m4), be32(n.r4), r4)) return false;
    const u128 m = be128(n.m6), r = be128(n.r6);
    if (!n.low6) return prefix_range<u128>(m, r, r6);
    // lowBitsV6V4(input): bytes 0-9 zero, bytes 10-11 both 0x00 or both 0xFF
    const u128 top = ~u128(0) << 32;
    if (r & ~m) return true;                                // matches nothing
    for (const u128 v : {u128(0), u128(0xFFFF) << 32}) {
        if ((r ^ v) & m & top) continue;                    // this form contradicts the rule
        if (!prefix_range<u128>(m | top, (r & ~top) | v, r6)) return false;
    }
    return true;
}

// elementary intervals of the ranges, each with the (x, y) filter masks of
// the ranges covering it; equal neighbours merged
template <class T>
void intervals(const std::vector<std::pair<T, T>>& rg, const std::vector<uint64_t>& bit,
               const std::vector<int>& side, std::vector<T>* starts,
               std::vector<std::pair<uint64_t, uint64_t>>* masks) {
    std::vector<T> b{T(0)};
    for (const auto& p : rg) {
        b.push_back(p.first);
        if (p.second != T(~T(0))) b.push_back(T(p.second + 1));
    }
    std::sort(b.begin(), b.end());
    b.erase(std::unique(b.begin(), b.end()), b.end());
    starts->clear();
    masks->clear();
    for (const T s : b) {
        uint64_t x = 0, y = 0;
        for (size_t k = 0; k < rg.size(); ++k)
            if (rg[k].first <= s && s <= rg[k].second) (side[k] ? y : x) |= bit[k];
        if (!masks->empty() && masks->back() == std::make_pair(x, y)) continue;
        starts->push_back(s);
        masks->push_back({x, y});
    }
}
}  // namespace

bool build_mirror_switch(const std::vector<MirrorRec>& recs, int32_t origin, MirrorSwBuilt* out) {
    *out = MirrorSwBuilt{};
    std::vector<std::pair<uint32_t, uint32_t>> r4;
    std::vector<std::pair<u128, u128>> r6;
    std::vector<uint64_t> bit4, bit6;
    std::vector<int> side4, side6;
    std::map<int32_t, uint64_t> mirs, tmap, amap;
    std::map<uint64_t, std::pair<uint64_t, uint64_t>> macm;  // MAC -> (macX of, macY of)
    std::vector<std::pair<uint32_t, uint32_t>> rp;           // port ranges, x and y
    std::vector<uint64_t> bitp;
    std::vector<int> sidep;
    auto pkey = [](int32_t p) { return uint32_t(p) ^ 0x80000000u; };
    MirrorSwImage& s = out->img;
    int j = 0;
    for (const MirrorRec& f : recs) {
        if (f.origin != origin) continue;
        if (j == 64) return false;
        const uint64_t b = uint64_t(1) << j++;
        s.all |= b;
        mirs[f.mirror] |= b;
        if (f.flags & VC_MF_MAC_X) {
            s.mac |= b;
            out->macs.push_back({b, f.mac_x, f.mac_y, (f.flags & VC_MF_MAC_Y) ? 1u : 0u, 0});
            macm[f.mac_x].first |= b;
            if (f.flags & VC_MF_MAC_Y) {
                macm[f.mac_y].second |= b;
                s.mac_both |= b;
            } else {
                s.mac_xonly |= b;
            }
        }
        for (int y = 0; y < 2; ++y) {
            if (!(f.flags & (y ? VC_MF_NET_Y : VC_MF_NET_X))) continue;
            (y ? s.has_y : s.has_x) |= b;
            if (!net_ranges(y ? f.net_y : f.net_x, &r4, &r6)) return false;
            bit4.resize(r4.size(), b);
            side4.resize(r4.size(), y);
            bit6.resize(r6.size(), b);
            side6.resize(r6.size(), y);
        }
        if (f.flags & VC_MF_PORT_X) {
            s.has_px |= b;
            rp.push_back({pkey(f.port_x0), pkey(f.port_x1)});
            bitp.push_back(b);
            sidep.push_back(0);
        }
        if (f.flags & VC_MF_PORT_Y) {
            s.has_py |= b;
            rp.push_back({pkey(f.port_y0), pkey(f.port_y1)});
            bitp.push_back(b);
            sidep.push_back(1);
        }
        if (f.transport == -1) s.any_t |= b;
        else tmap[f.transport] |= b;
        if (f.app == -1) s.any_a |= b;
        else amap[f.app] |= b;
    }
    if (!j) return false;
    for (const auto& m : mirs) out->mirs.push_back({m.second, uint32_t(m.first), 0});
    std::vector<std::pair<uint64_t, uint64_t>> m4, m6;
    intervals<uint32_t>(r4, bit4, side4, &out->b4, &m4);
    std::vector<u128> b6;
    intervals<u128>(r6, bit6, side6, &b6, &m6);
    for (const auto& m : m4) out->p4.insert(out->p4.end(), {m.first, m.second});
    for (const u128 v : b6) out->b6.insert(out->b6.end(), {uint64_t(v >> 64), uint64_t(v)});
    for (const auto& m : m6) out->p6.insert(out->p6.end(), {m.first, m.second});
    std::vector<std::pair<uint64_t, uint64_t>> mp;
    intervals<uint32_t>(rp, bitp, sidep, &out->bp, &mp);
    for (const auto& m : mp) out->pp.insert(out->pp.end(), {m.first, m.second});
    for (const auto& m : tmap) out->tids.push_back({m.second, m.first, 0});
    for (const auto& m : amap) out->aids.push_back({m.second, m.first, 0});
    for (const auto& m : macm) {
        out->bm.push_back(m.first);
        out->pm.insert(out->pm.end(), {m.second.first, m.second.second});
    }
    s.nbm = int32_t(out->bm.size());
    s.n_t = int32_t(out->tids.size());
    s.n_a = int32_t(out->aids.size());
    s.nbp = int32_t(out->bp.size());
    s.n_mac = int32_t(out->macs.size());
    s.n_mir = int32_t(out->mirs.size());
    s.nb4 = int32_t(out->b4.size());
    s.nb6 = int32_t(b6.size());
    return true;
}

// ---------------------------------------------------------------------------
// ServerGroup source hashing
// ---------------------------------------------------------------------------
namespace {

// sourceReset's comparator (ServerGroup.java:629-642): address length,
// then signed address bytes, then port.
int server_cmp(const vc_server& a, const vc_server& b) {
    if (a.ip_len > b.ip_len) return 1;
    if (b.ip_len > a.ip_len) return -1;
    for (int i = 0; i < a.ip_len; ++i) {
        const int diff = int(int8_t(a.ip[i])) - int(int8_t(b.ip[i]));
        if (diff != 0) return diff;
    }
    return a.port - b.port;
}

}  // namespace

int build_servers(const vc_server* servers, const int32_t* group_off, int n_groups,
                  ServersBuilt* out) {
    *out = ServersBuilt{};
    if (n_groups < 0 || (n_groups > 0 && !group_off)) return VC_EINVAL;
    const int32_t total = n_groups > 0 ? group_off[n_groups] : 0;
    if (n_groups > 0 && group_off[0] != 0) return VC_EINVAL;
    for (int g = 0; g < n_groups; ++g)
        if (group_off[g + 1] < group_off[g]) return VC_EINVAL;
    if (total > 0 && !servers) return VC_EINVAL;
    for (int32_t i = 0; i < total; ++i)
        if (servers[i].ip_len != 4 && servers[i].ip_len != 16) return VC_EINVAL;
    out->n_groups = n_groups;
    out->n_servers = total;
    out->view_off.assign(size_t(n_groups) * 6, 0);
    out->group_base.assign(size_t(n_groups) + 1, 0);
    out->healthy.resize(size_t(total) + 1, 0);
    for (int32_t i = 0; i < total; ++i) out->healthy[i] = servers[i].healthy ? 1 : 0;
    for (int g = 0; g < n_groups; ++g) {
        out->group_base[g] = group_off[g];
        for (int v = 0; v < 3; ++v) {
            std::vector<int32_t> ids;
            for (int32_t i = group_off[g]; i < group_off[g + 1]; ++i) {
                const vc_server& sv = servers[i];
                if (v == 1 && sv.ip_len != 4) continue;    // :622 instanceof IPv4
                if (v == 2 && sv.ip_len != 16) continue;   // :623 instanceof IPv6
                if (sv.weight <= 0) continue;              // :628 weight > 0
                ids.push_back(i);
            }
            std::stable_sort(ids.begin(), ids.end(), [&](int32_t a, int32_t b) {
                return server_cmp(servers[a], servers[b]) < 0;   // List.sort is stable
            });
            out->view_off[size_t(g) * 6 + 2 * v] = static_cast<uint32_t>(out->order.size());
            out->view_off[size_t(g) * 6 + 2 * v + 1] = static_cast<uint32_t>(ids.size());
            out->order.insert(out->order.end(), ids.begin(), ids.end());
        }
    }
    out->group_base[n_groups] = total;
    // the packed form for the kernels' LDS copy (images.h ServerImage.view_pk)
    out->pk_ok = n_groups > 0;
    out->view_pk.assign(size_t(n_groups) * 3 + 1, 0);
    for (int g = 0; g < n_groups && out->pk_ok; ++g)
        for (int v = 0; v < 3; ++v) {
            const uint32_t off = out->view_off[size_t(g) * 6 + 2 * v];
            const uint32_t cnt = out->view_off[size_t(g) * 6 + 2 * v + 1];
            if (off >= (1u << 24) || cnt >= 256u) {
                out->pk_ok = false;
                break;
            }
            out->view_pk[size_t(v) * n_groups + g] = off << 8 | cnt;
        }
    if (out->order.empty()) out->order.push_back(0);
    if (out->view_off.empty()) out->view_off.assign(6, 0);
    source_pick_table(*out, out->healthy.data(), &out->pick);
    return VC_OK;
}

// sourceHashGet's probe (ServerGroup.java:479-490): from idx = hash % size
// it takes the first healthy server at idx, idx + 1, ... cyclically, null
// after a whole round.  That depends only on idx, so each list position
// gets its answer once per health state: a backward pass over the list
// doubled carries the nearest healthy server at or after each position.
void source_pick_table(const ServersBuilt& b, const uint8_t* healthy, std::vector<int32_t>* pick) {
    pick->assign(b.order.size(), -1);
    for (int g = 0; g < b.n_groups; ++g) {
        for (int v = 0; v < 3; ++v) {
            const uint32_t off = b.view_off[size_t(g) * 6 + 2 * v];
            const int64_t size = b.view_off[size_t(g) * 6 + 2 * v + 1];
            int32_t next = -1;
            for (int64_t k = 2 * size - 1; k >= 0; --k) {
                const int32_t s = b.order[off + size_t(k % size)];
                if (healthy[s]) next = s - b.group_base[g];
                if (k < size) (*pick)[off + size_t(k)] = next;
            }
        }
    }
}

namespace {

struct Digest {
    uint64_t h = 14695981039346656037ull;
    void word(uint64_t w) { h = (h ^ w) * 1099511628211ull; }
    void bytes(const void* p, size_t n) {
        const uint8_t* b = static_cast<const uint8_t*>(p);
        word(n);
        size_t i = 0;
        for (; i + 8 <= n; i += 8) {
            uint64_t w;
            std::memcpy(&w, b + i, 8);
            word(w);
        }
        uint64_t w = 0;
        std::memcpy(&w, b + i, n - i);
        word(w);
    }
    template <class T>
    void vec(const std::vector<T>& v) { bytes(v.data(), v.size() * sizeof(T)); }
};

}  // namespace

uint64_t digest(const AclBuilt& b) {
    Digest d;
    for (int l = 0; l < 2; ++l)
        for (int f = 0; f < 2; ++f) {
            const AclFamilyBuilt& x = b.fam[l][f];
            d.vec(x.bounds4);
            d.vec(x.bounds6);
            d.vec(x.desc);
            d.vec(x.rec);
            d.vec(x.pieces);
            d.vec(x.dir4);
            d.word(uint64_t(uint32_t(x.nb)) | uint64_t(uint32_t(x.dir_bits)) << 32);
            d.word(uint64_t(uint32_t(x.v4_only)));
        }
    d.vec(b.allow);
    d.word(uint64_t(uint32_t(b.n_tcp)) | uint64_t(uint32_t(b.n_udp)) << 32);
    d.word(uint64_t(b.default_allow));
    return d.h;
}

uint64_t digest(const TrieBuilt& t4, const TrieBuilt& t6) {
    Digest d;
    for (const TrieBuilt* t : {&t4, &t6}) {
        d.vec(t->nodes);
        d.word(uint64_t(uint32_t(t->root_bits)) | uint64_t(uint32_t(t->key_bits)) << 32);
        d.word(uint64_t(uint32_t(t->n_rules)) | uint64_t(uint32_t(t->n_nodes)) << 32);
        d.word(uint64_t(uint32_t(t->n_records)));
    }
    return d.h;
}

uint64_t digest(const HintBuilt& b) {
    Digest d;
    d.vec(b.blob);
    d.vec(b.host.tags);
    d.vec(b.host.recs);
    d.vec(b.host.ext);
    d.word(uint64_t(uint32_t(b.host.n)));
    d.vec(b.uri_slots);
    d.vec(b.uri_tags);
    d.vec(b.lists);
    d.vec(b.port_mins);
    d.vec(b.groups);
    d.word(uint64_t(uint32_t(b.n_groups)) | uint64_t(uint32_t(b.wildcard_slot)) << 32);
    d.word(uint64_t(uint32_t(b.uri_star_slot)) | uint64_t(uint32_t(b.has_uri_keys)) << 32);
    d.word(b.uri_len_mask);
    return d.h;
}

}  // namespace vc

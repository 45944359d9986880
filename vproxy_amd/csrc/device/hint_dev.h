// hint_dev.h -- device side of Upstream.searchForGroup(Hint) and DNS
// classification.  See hint.hip for the kernels.
//
//   Hint.formatHost / formatUri      base/.../processor/Hint.java:57-90
//   Hint.matchLevel                  Hint.java:100-160
//   Upstream.searchForGroup          core/.../svrgroup/Upstream.java:187-198
//   IP.isIpv6 / isIpLiteral          base/src/main/java/vfd/IP.java:158-300
//   DNSServer.handleRequest (class.) core/src/main/java/vproxy/dns/DNSServer.java:116-166
//
// One lane per hint.  The linear argmax over all groups becomes a handful of
// hash probes: the query host is scanned right-to-left once, producing the
// reversed-FNV hash of every dot-suffix ("." + annoHost candidates) and of
// the whole host; each probe is confirmed by a byte compare.
#pragma once

#include "dev_common.h"

#define VC_HDN __host__ __device__

namespace vcd {


struct DStr {
    const uint8_t* p;
    int n;        // -1 == Java null
};

VC_HD bool bytes_eq(const uint8_t* a, const uint8_t* b, int n) {
    for (int i = 0; i < n; ++i)
        if (a[i] != b[i]) return false;
    return true;
}

// ---------------------------------------------------------------------------
// IP literal validity (IP.java).  Only validity is needed on the device.
// ---------------------------------------------------------------------------

// IP.parseIpv4String(s, bytes, from) with bytes.length == cap: 4 or -1
VC_HDN int d_v4(const uint8_t* s, int n, int from, int cap) {
    int pieces = 0, start = 0;
    for (int i = 0; i <= n; ++i) {
        if (i < n && s[i] != '.') continue;
        int len = i - start;
        if (pieces >= 4) return -1;                      // split length != 4
        if (from + pieces >= cap) return -1;
        if (len > 3 || len == 0) return -1;
        int num = 0;
        for (int k = start; k < i; ++k) {
            uint8_t c = s[k];
            if (c < '0' || c > '9') return -1;
            num = num * 10 + (c - '0');
        }
        if (s[start] == '0' && len > 1) return -1;
        if (num > 255) return -1;
        ++pieces;
        start = i + 1;
    }
    return pieces == 4 ? 4 : -1;
}

VC_HD bool d_hex(uint8_t c) {
    return (c >= '0' && c <= '9') || (c >= 'a' && c <= 'f') || (c >= 'A' && c <= 'F');
}

// IP.parseIpv6ColonPart for a present (non-null) string
VC_HDN int d_colon_part(const uint8_t* s, int n, int from) {
    if (n == 0) return 0;
    if (from < 0) return -1;
    int fields = 0, start = 0;
    for (int i = 0; i <= n; ++i) {
        if (i < n && s[i] != ':') continue;
        int len = i - start;
        if (from + 2 * fields >= 16) return -1;
        if (len > 4 || len == 0) return -1;
        for (int k = start; k < i; ++k)
            if (!d_hex(s[k])) return -1;
        ++fields;
        start = i + 1;
    }
    return fields * 2;
}

VC_HD int d_count(const uint8_t* s, int n, uint8_t c) {
    int k = 0;
    for (int i = 0; i < n; ++i) k += s[i] == c;
    return k;
}

// IP.parseIpv6LastBits, including the `4 + colonPart` sum (IP.java:264)
VC_HDN int d_last_bits(const uint8_t* s, int n) {
    int dot = -1;
    for (int i = 0; i < n; ++i)
        if (s[i] == '.') { dot = i; break; }
    if (dot >= 0) {
        int colon = -1;
        for (int i = dot - 1; i >= 0; --i)
            if (s[i] == ':') { colon = i; break; }
        if (colon < 0) return d_v4(s, n, 12, 16);
        if (d_v4(s + colon + 1, n - colon - 1, 12, 16) == -1) return -1;
        int pieces = 1 + d_count(s, colon, ':');
        return 4 + d_colon_part(s, colon, 16 - 4 - pieces * 2);
    }
    int pieces = 1 + d_count(s, n, ':');
    return d_colon_part(s, n, 16 - pieces * 2);
}

// IP.isIpv6 == parseIpv6String(s) != null (IP.java:158-197)
VC_HDN bool d_is_ipv6(const uint8_t* s, int n) {
    if (n >= 2 && s[0] == '[' && s[n - 1] == ']') {
        s += 1;
        n -= 2;
    }
    int dbl = 0, first = -1;
    for (int i = 0; i + 1 < n;) {
        if (s[i] == ':' && s[i + 1] == ':') {
            if (first < 0) first = i;
            ++dbl;
            i += 2;
        } else {
            ++i;
        }
    }
    if (dbl > 1) return false;
    int c1 = first >= 0 ? d_colon_part(s, first, 0) : 0;
    if (c1 == -1) return false;
    int c2 = first >= 0 ? d_last_bits(s + first + 2, n - first - 2) : d_last_bits(s, n);
    if (c2 == -1) return false;
    return first >= 0 ? (c1 + c2 < 16) : (c1 + c2 == 16);
}

VC_HD bool d_is_ip_literal(const uint8_t* s, int n) {
    return d_is_ipv6(s, n) || d_v4(s, n, 0, 4) == 4;
}

// ---------------------------------------------------------------------------
// Hint.formatHost / formatUri
// ---------------------------------------------------------------------------
VC_HDN DStr format_host(DStr s) {
    if (s.n < 0) return s;
    int colon = -1;
    for (int i = 0; i < s.n; ++i)
        if (s.p[i] == ':') { colon = i; break; }
    if (colon < 0 || d_is_ipv6(s.p, s.n)) return s;
    DStr r{s.p, colon};
    if (r.n >= 4 && r.p[0] == 'w' && r.p[1] == 'w' && r.p[2] == 'w' && r.p[3] == '.') {
        r.p += 4;
        r.n -= 4;
    }
    if (r.n == 0) r.n = -1;
    return r;
}

VC_HDN DStr format_uri(DStr s) {
    if (s.n < 0) return s;
    for (int i = 0; i < s.n; ++i)
        if (s.p[i] == '?') { s.n = i; break; }
    if (s.n == 1 && s.p[0] == '/') return s;
    if (s.n > 0 && s.p[s.n - 1] == '/') s.n -= 1;
    return s;
}

// ---------------------------------------------------------------------------
// key tables
// ---------------------------------------------------------------------------
VC_HD KeySlot load_slot(const KeySlot* t, uint32_t s) {
    const uint4* p = reinterpret_cast<const uint4*>(t + s);
    uint4 a = p[0], b = p[1];
    KeySlot k;
    k.hash = (uint64_t(a.y) << 32) | a.x;
    k.key_len = int32_t(a.z);
    k.key_off = a.w;
    k.a = int32_t(b.x);
    k.b = int32_t(b.y);
    k.list_off = b.z;
    k.list_cnt = b.w;
    return k;
}

// key (16-byte aligned, zero padded in the blob) == query bytes p[0, n)?
// One uint4 key load per 16 bytes and branch-free byte gathers of the query
// (LDS when staged), instead of a byte-by-byte loop of dependent loads.
VC_HD bool key_eq(const uint8_t* key, const uint8_t* q, int n) {
    for (int base = 0; base < n; base += 16) {
        const uint4 kw = *reinterpret_cast<const uint4*>(key + base);
        const uint32_t k[4] = {kw.x, kw.y, kw.z, kw.w};
        uint32_t diff = 0;
#pragma unroll
        for (int w = 0; w < 4; ++w) {
            uint32_t qw = 0;
#pragma unroll
            for (int b = 0; b < 4; ++b) {
                const int i = base + 4 * w + b;
                qw |= uint32_t(i < n ? q[i] : 0) << (8 * b);
            }
            diff |= qw ^ k[w];
        }
        if (diff) return false;
    }
    return true;
}

// slot index of key (p, n) with hash h, or -1.  Linear probing from the
// hash's 4-slot group: one 16-byte tag-group load per step; the 32-byte slot
// and the key are read only on a tag hit.
VC_HDN int probe(const uint32_t* tags, const KeySlot* t, uint32_t mask, const uint8_t* blob,
                 uint32_t h, const uint8_t* p, int n, KeySlot* out) {
    const uint32_t want = h | 1u;
    uint32_t s = h & mask & ~3u;
    for (;;) {
        const uint4 g = *reinterpret_cast<const uint4*>(tags + s);
        const uint32_t tg[4] = {g.x, g.y, g.z, g.w};
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            if (tg[k] == 0) return -1;
            if (tg[k] == want) {
                KeySlot ks = load_slot(t, s + k);
                if (ks.key_len == n && key_eq(blob + ks.key_off, p, n)) {
                    *out = ks;
                    return int(s + k);
                }
            }
        }
        s = (s + 4) & mask;
    }
}

// min handle index of a host key not excluded by the port filter
// (Hint.java:124-128): port == 0 -> any; else hint-port 0 or equal.
VC_HD uint32_t pick(const HintImage& img, int slot, const KeySlot& k, int port) {
    if (port == 0) return uint32_t(k.a);
    uint32_t v = uint32_t(k.b);
    const uint32_t off = img.port_min_off[2 * slot], cnt = img.port_min_off[2 * slot + 1];
    for (uint32_t i = 0; i < cnt; ++i) {
        const PortMin pm = img.port_mins[off + i];
        if (pm.port == port) v = uint32_t(pm.idx) < v ? uint32_t(pm.idx) : v;
    }
    return v;
}

// Continue a probe at group start `s` whose 16-byte tag group `g` is already
// loaded (linear probing moves on only when that group is full of other keys).
VC_HDN int probe_from(const uint32_t* tags, const KeySlot* t, uint32_t mask, const uint8_t* blob,
                      uint32_t h, const uint8_t* p, int n, uint32_t s, uint4 g, KeySlot* out) {
    const uint32_t want = h | 1u;
    for (;;) {
        const uint32_t tg[4] = {g.x, g.y, g.z, g.w};
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            if (tg[k] == 0) return -1;
            if (tg[k] == want) {
                KeySlot ks = load_slot(t, s + k);
                if (ks.key_len == n && key_eq(blob + ks.key_off, p, n)) {
                    *out = ks;
                    return int(s + k);
                }
            }
        }
        s = (s + 4) & mask;
        g = *reinterpret_cast<const uint4*>(tags + s);
    }
}

VC_HD uint4 tag_group(const uint32_t* tags, uint32_t mask, uint32_t h) {
    return *reinterpret_cast<const uint4*>(tags + (h & mask & ~3u));
}

// Sequential form (any number of labels): scan right-to-left, probe at dots.
VC_HDN int32_t hint_host_only_seq(const HintImage& img, DStr host, int port) {
    uint32_t h = kFnvBasis;
    uint32_t best_suffix = VC_NONE;
    KeySlot k;
    for (int j = host.n - 1; j >= 0; --j) {
        const uint8_t c = host.p[j];
        if (c == '.') {   // host.endsWith("." + H) with H = host[j+1..]
            int s = probe(img.host_tags, img.host_slots, img.host_mask, img.blob, h, host.p + j + 1,
                          host.n - j - 1, &k);
            if (s >= 0) {
                uint32_t c2 = pick(img, s, k, port);
                best_suffix = c2 < best_suffix ? c2 : best_suffix;
            }
        }
        h = fnv_step(h, c);
    }
    int s = probe(img.host_tags, img.host_slots, img.host_mask, img.blob, h, host.p, host.n, &k);
    if (s >= 0) {
        uint32_t e = pick(img, s, k, port);
        if (e != VC_NONE) return int32_t(e);
    }
    if (best_suffix != VC_NONE) return int32_t(best_suffix);
    if (img.wildcard_slot >= 0) {
        KeySlot w = load_slot(img.host_slots, uint32_t(img.wildcard_slot));
        uint32_t v = pick(img, img.wildcard_slot, w, port);
        if (v != VC_NONE) return int32_t(v);
    }
    return -1;
}

// Per-probe summary of a loaded 16-byte tag group: bits 0-3 = slots whose
// tag matches, bit 4 = the group holds no empty slot (probing may continue).
VC_HD uint32_t group_code(uint4 g, uint32_t h) {
    const uint32_t want = h | 1u;
    const uint32_t tg[4] = {g.x, g.y, g.z, g.w};
    uint32_t code = 0, open = 0;
#pragma unroll
    for (int k = 0; k < 4; ++k) {
        // slots past the first empty one are never part of this key's chain
        const bool before_empty = open == 0;
        if (tg[k] == 0) open = 1;
        if (before_empty && tg[k] == want) code |= 1u << k;
    }
    if (!open) code |= 16u;
    return code;
}

// Resolve one probe given its first-group summary (slot loads + key compare
// only for tag hits); -1 when absent.  Kept out of line: it runs about once
// per name, and inlining it per suffix multiplied the register footprint.
// Returns pick(...) of the matching host key, or VC_NONE when the key is
// absent (or every member is excluded by the port filter).
// (Takes the image's arrays one by one: passing the HintImage by reference
// to an out-of-line function put a copy of it on the scratch stack.)
__host__ __device__ __noinline__ uint32_t resolve_pick(
    const uint32_t* tags, const KeySlot* slots, uint32_t mask, const uint8_t* blob,
    const uint32_t* pm_off, const PortMin* pms, uint32_t h, const uint8_t* p, int n,
    uint32_t code, int port) {
    const uint32_t s0 = h & mask & ~3u;
    int s = -1;
    KeySlot ks;
#pragma unroll
    for (int k = 0; k < 4; ++k) {
        if (s < 0 && (code & (1u << k))) {
            const KeySlot c = load_slot(slots, s0 + k);
            if (c.key_len == n && key_eq(blob + c.key_off, p, n)) {
                s = int(s0 + k);
                ks = c;
            }
        }
    }
    if (s < 0) {
        if (!(code & 16u)) return VC_NONE;
        // the first group was full of other keys: continue linear probing
        const uint32_t s1 = (s0 + 4) & mask;
        s = probe_from(tags, slots, mask, blob, h, p, n, s1,
                       *reinterpret_cast<const uint4*>(tags + s1), &ks);
        if (s < 0) return VC_NONE;
    }
    if (port == 0) return uint32_t(ks.a);            // pick() (Hint.java:124-128)
    uint32_t v = uint32_t(ks.b);
    const uint32_t off = pm_off[2 * s], cnt = pm_off[2 * s + 1];
    for (uint32_t i = 0; i < cnt; ++i) {
        const PortMin pm = pms[off + i];
        if (pm.port == port) v = uint32_t(pm.idx) < v ? uint32_t(pm.idx) : v;
    }
    return v;
}

// searchForGroup for hints whose uri is null (or no group has a hint-uri):
// level = hostLevel << 10, so exact (3) beats any suffix (2) beats "*" (1),
// and within a level the lowest handle index wins (strict '>' scan).
// Batched form: one register-only scan hashes the whole host and every
// dot-suffix, then all first tag groups are loaded together (independent
// loads in flight) before any slot or key is touched.
constexpr int kMaxSuffix = 6;

VC_HDN int32_t hint_host_only(const HintImage& img, DStr host, int port) {
    if (host.n < 0) return -1;
    uint32_t hs[kMaxSuffix];
    int st[kMaxSuffix];
    int np = 0;
    uint32_t h = kFnvBasis;
    for (int j = host.n - 1; j >= 0; --j) {
        const uint8_t c = host.p[j];
        if (c == '.') {
#pragma unroll
            for (int k = 0; k < kMaxSuffix; ++k)
                if (k == np) {
                    hs[k] = h;
                    st[k] = j + 1;
                }
            ++np;
        }
        h = fnv_step(h, c);
    }
    if (np > kMaxSuffix) return hint_host_only_seq(img, host, port);
    uint4 g[kMaxSuffix + 1];
    g[kMaxSuffix] = tag_group(img.host_tags, img.host_mask, h);
#pragma unroll
    for (int k = 0; k < kMaxSuffix; ++k)
        if (k < np) g[k] = tag_group(img.host_tags, img.host_mask, hs[k]);
    uint32_t code[kMaxSuffix + 1];
    code[kMaxSuffix] = group_code(g[kMaxSuffix], h);
#pragma unroll
    for (int k = 0; k < kMaxSuffix; ++k) code[k] = k < np ? group_code(g[k], hs[k]) : 0u;
    if (code[kMaxSuffix]) {
        const uint32_t e = resolve_pick(img.host_tags, img.host_slots, img.host_mask, img.blob,
                                        img.port_min_off, img.port_mins, h, host.p, host.n,
                                        code[kMaxSuffix], port);
        if (e != VC_NONE) return int32_t(e);
    }
    uint32_t best = VC_NONE;
#pragma unroll
    for (int k = 0; k < kMaxSuffix; ++k) {
        if (code[k]) {
            const uint32_t c = resolve_pick(img.host_tags, img.host_slots, img.host_mask,
                                            img.blob, img.port_min_off, img.port_mins, hs[k],
                                            host.p + st[k], host.n - st[k], code[k], port);
            best = c < best ? c : best;
        }
    }
    if (best != VC_NONE) return int32_t(best);
    if (img.wildcard_slot >= 0) {
        KeySlot w = load_slot(img.host_slots, uint32_t(img.wildcard_slot));
        const uint32_t v = pick(img, img.wildcard_slot, w, port);
        if (v != VC_NONE) return int32_t(v);
    }
    return -1;
}

// Hint.matchLevel for one merged group (Hint.java:100-160)
VC_HDN int match_level(const HintImage& img, uint32_t g, DStr host, int port, DStr uri) {
    const int32_t* r = reinterpret_cast<const int32_t*>(img.groups) + 6 * g;
    const int32_t Hn = r[0], Un = r[2], P = r[4];
    if (!r[5]) return 0;
    if (port != 0 && P != 0 && port != P) return 0;
    const uint8_t* H = img.blob + uint32_t(r[1]);
    const uint8_t* U = img.blob + uint32_t(r[3]);
    int hl = 0;
    if (Hn >= 0 && host.n >= 0) {
        if (host.n == Hn && bytes_eq(host.p, H, Hn)) hl = 3;
        else if (host.n >= Hn + 1 && host.p[host.n - Hn - 1] == '.' &&
                 bytes_eq(host.p + host.n - Hn, H, Hn)) hl = 2;
        else if (Hn == 1 && H[0] == '*') hl = 1;
    }
    int ul = 0;
    if (Un >= 0 && uri.n >= 0) {
        if (uri.n == Un && bytes_eq(uri.p, U, Un)) ul = uri.n + 1;
        else if (uri.n >= Un && bytes_eq(uri.p, U, Un)) ul = Un + 1;
        else if (Un == 1 && U[0] == '*') ul = 1;
    }
    if (ul > 1023) ul = 1023;
    return (hl << 10) + ul;
}

struct Best {
    int level = 0;
    int32_t idx = -1;
    VC_HDN void consider(int lvl, int32_t g) {
        if (lvl > level || (lvl == level && lvl > 0 && g < idx)) {
            level = lvl;
            idx = g;
        }
    }
};

VC_HDN void consider_list(const HintImage& img, const KeySlot& k, DStr host, int port, DStr uri,
                              Best* b) {
    for (uint32_t i = 0; i < k.list_cnt; ++i) {
        uint32_t g = img.lists[k.list_off + i];
        b->consider(match_level(img, g, host, port, uri), int32_t(g));
    }
}

// General searchForGroup: every group with a nonzero level has its hint-host
// equal to / a dot-suffix of / "*" for the host, or its hint-uri a prefix
// of / "*" for the uri; those candidate lists are scored exactly.
VC_HDN int32_t hint_general(const HintImage& img, DStr host, int port, DStr uri) {
    Best b;
    KeySlot k;
    if (host.n >= 0) {
        uint32_t h = kFnvBasis;
        for (int j = host.n - 1; j >= 0; --j) {
            const uint8_t c = host.p[j];
            if (c == '.' && probe(img.host_tags, img.host_slots, img.host_mask, img.blob, h, host.p + j + 1,
                                  host.n - j - 1, &k) >= 0)
                consider_list(img, k, host, port, uri, &b);
            h = fnv_step(h, c);
        }
        if (probe(img.host_tags, img.host_slots, img.host_mask, img.blob, h, host.p, host.n, &k) >= 0)
            consider_list(img, k, host, port, uri, &b);
        if (img.wildcard_slot >= 0)
            consider_list(img, load_slot(img.host_slots, uint32_t(img.wildcard_slot)), host, port,
                          uri, &b);
    }
    if (uri.n >= 0) {
        uint32_t h = kFnvBasis;
        for (int j = 0; j <= uri.n; ++j) {
            if (probe(img.uri_tags, img.uri_slots, img.uri_mask, img.blob, h, uri.p, j, &k) >= 0)
                consider_list(img, k, host, port, uri, &b);
            if (j < uri.n) h = fnv_step(h, uri.p[j]);
        }
        if (img.uri_star_slot >= 0)
            consider_list(img, load_slot(img.uri_slots, uint32_t(img.uri_star_slot)), host, port,
                          uri, &b);
    }
    return b.idx;
}

VC_HD int32_t search_for_group(const HintImage& img, DStr host, int port,
                                                    DStr uri) {
    if (uri.n < 0 || !img.has_uri_keys) return hint_host_only(img, host, port);
    return hint_general(img, host, port, uri);
}

}  // namespace vcd

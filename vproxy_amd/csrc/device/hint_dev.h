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

#include "../common/khash.h"
#include "dev_common.h"

#define VC_HDN __host__ __device__

namespace vcd {

// Profiling builds only (-DVC_HINT_PROF, scripts/hint_prof.py): per-wave
// cycles of the string kernels' phases, accumulated in LDS by every active
// lane (the clock is wave-uniform, so the lanes store equal values).
#if defined(VC_HINT_PROF)
constexpr int kProfPhases = 6;
extern __shared__ uint64_t vc_prof_lds[];
__device__ __forceinline__ void prof_mark(int i) {
    uint64_t* t = vc_prof_lds + (threadIdx.x >> 6) * (kProfPhases + 1);
    const uint64_t now = clock64();
    t[i] += now - t[kProfPhases];
    t[kProfPhases] = now;
}
#endif
#if defined(VC_HINT_PROF) && defined(__HIP_DEVICE_COMPILE__)
#define VC_PMARK(i) prof_mark(i)
#else
#define VC_PMARK(i) ((void)0)
#endif

struct DStr {
    const uint8_t* p;
    int n;        // -1 == Java null
};

// Eight bytes a step with no exit inside a step, so a step's loads issue
// together: compared byte by byte with an exit per byte, every load of an
// annotation string in global memory was its own round trip (the general
// search path compares hint-hosts / hint-uris this way).
VC_HD bool bytes_eq(const uint8_t* a, const uint8_t* b, int n) {
    for (int i = 0; i < n; i += 8) {
        uint32_t d = 0;
#pragma unroll
        for (int k = 0; k < 8; ++k)
            if (i + k < n) d |= uint32_t(a[i + k] ^ b[i + k]);
        if (d) return false;
    }
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
__host__ __device__ __noinline__ bool d_is_ipv6(const uint8_t* s, int n) {
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
// Byte sources.  The fast path reads a name a 32-bit word at a time; PtrSrc
// serves plain pointers (global memory, the host harness) byte by byte and
// never touches bytes outside the requested range; LdsSrc serves a name
// staged in LDS, whose neighbourhood (>= 4 bytes either side) is readable.
// ---------------------------------------------------------------------------

// bytes j of a word at `pos` kept iff lo <= pos + j < hi
VC_HD uint32_t keep_mask(int pos, int lo, int hi) {
    int a = lo - pos, b = hi - pos;
    a = a < 0 ? 0 : (a > 4 ? 4 : a);
    b = b < 0 ? 0 : (b > 4 ? 4 : b);
    const uint32_t m_lo = a >= 4 ? 0u : (~0u << (8 * a));
    const uint32_t m_hi = b >= 4 ? ~0u : ((1u << (8 * b)) - 1u);
    return m_lo & m_hi;
}

// bytes j of a word at `pos` kept iff pos + j >= lo; needs pos > lo - 4
VC_HD uint32_t lo_mask(int pos, int lo) {
    return pos >= lo ? ~0u : (~0u << (8 * (lo - pos)));
}

// the first r bytes of a word; needs r >= 1
VC_HD uint32_t tail_mask(int r) {
    return r >= 4 ? ~0u : ((1u << (8 * r)) - 1u);
}

// Word reads of a source.  word(pos, lo, hi) keeps bytes in [lo, hi).
// down(pos, lo, hi) is for words that end at or before hi (right-to-left
// scans) and masks only the low side.  cursor(pos, hi).get(j) is the word
// at pos + 4j; with LdsSrc its bytes at or past hi are NOT masked, so
// callers mask with tail_mask.
struct PtrSrc {
    const uint8_t* p;
    VC_HD const uint8_t* ptr() const { return p; }
    VC_HD uint32_t word(int pos, int lo, int hi) const {
        uint32_t w = 0;
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            const int i = pos + j;
            if (i >= lo && i < hi) w |= uint32_t(p[i]) << (8 * j);
        }
        return w;
    }
    // word ending at or before hi, bytes below lo zero (pos > lo - 4)
    VC_HD uint32_t down(int pos, int lo, int hi) const { return word(pos, lo, hi); }
    struct Cur {
        const uint8_t* p;
        int pos, hi;
        VC_HD uint32_t get(int j) const { return PtrSrc{p}.word(pos + 4 * j, pos, hi); }
    };
    VC_HD Cur cursor(int pos, int hi) const { return Cur{p, pos, hi}; }
};

// LE word from two aligned words: bytes [sh, sh + 4) of (hi:lo)
VC_HD uint32_t funnel(uint32_t lo, uint32_t hi, uint32_t sh) {
    return uint32_t(((uint64_t(hi) << 32) | lo) >> (8 * sh));
}

struct LdsSrc {
    const uint32_t* w;            // the wave's LDS stage (dword array)
    int off;                      // byte offset of the name's byte 0 in the stage
    VC_HD const uint8_t* ptr() const { return reinterpret_cast<const uint8_t*>(w) + off; }
    VC_HD uint32_t raw(int pos) const {
        const int a = off + pos;                // >= 0: the stage has a 16-byte apron
        return funnel(w[a >> 2], w[(a >> 2) + 1], uint32_t(a & 3));
    }
    VC_HD uint32_t word(int pos, int lo, int hi) const { return raw(pos) & keep_mask(pos, lo, hi); }
    // a word that ends at or before the key's end: only the low side to mask
    VC_HD uint32_t down(int pos, int lo, int hi) const { return raw(pos) & lo_mask(pos, lo); }
    struct Cur {                  // word j at dword p[j], p[j + 1] (immediate offsets)
        const uint32_t* p;
        uint32_t sh;
        VC_HD uint32_t get(int j) const { return funnel(p[j], p[j + 1], sh); }
    };
    VC_HD Cur cursor(int pos, int hi) const {
        const int a = off + pos;
        return Cur{w + (a >> 2), uint32_t(a & 3)};
    }
};

// ---------------------------------------------------------------------------
// Host-name key table: tags + 64-byte records (common/images.h HostRec),
// keyed by vck::khash.
// ---------------------------------------------------------------------------
struct HostTable {
    const uint32_t* tags;
    const HostRec* recs;
    const uint8_t* blob;
    uint32_t mask;
};

struct Rec {                      // a HostRec in registers
    uint4 m, k0, k1, k2;          // meta (len_pm, a, b, key_off), key words 0..11
};

VC_HD Rec load_rec(const HostRec* r, uint32_t s) {
    const uint4* p = reinterpret_cast<const uint4*>(r + s);
    return Rec{p[0], p[1], p[2], p[3]};
}

VC_HD uint32_t rec_word(const Rec& r, int j) {       // j < 12, unrolled callers
    const uint32_t k[12] = {r.k0.x, r.k0.y, r.k0.z, r.k0.w, r.k1.x, r.k1.y,
                            r.k1.z, r.k1.w, r.k2.x, r.k2.y, r.k2.z, r.k2.w};
    return k[j];
}

// True on the device when any active lane of the wave has p (a wave vote,
// so an unrolled loop can stop at the wave's longest key).
VC_HD bool wave_any(bool p) {
#if defined(__HIP_DEVICE_COMPILE__)
    return __ballot(p) != 0;
#else
    return p;
#endif
}

// record key == query bytes [st, st + n)?
template <class Src>
VC_HD bool rec_eq(const Rec& r, const uint8_t* blob, const Src& q, int st, int n) {
    // The word masks use rn, the record's length, made opaque after the
    // check: with n the compiler hoists all twelve masks out of the probe
    // loop and computes them per hit; only the key's last word needs one.
    int rn = int(r.m.x & VC_REC_LEN);
    if (rn != n) return false;
#if defined(__HIP_DEVICE_COMPILE__)
    asm volatile("" : "+v"(rn));
#endif
    uint32_t diff = 0;
    const auto c = q.cursor(st, st + n);
#pragma unroll
    for (int j = 0; j < VC_REC_INLINE / 4; ++j) {
        if (!wave_any(4 * j < rn)) break;         // no lane's key reaches word j
        if (4 * j < rn) {
            uint32_t d = c.get(j) ^ rec_word(r, j);
            if (4 * j + 4 > rn) d &= tail_mask(rn - 4 * j);
            diff |= d;
        }
    }
    if (diff) return false;
    if (n > VC_REC_INLINE) {      // long key: the rest from the blob copy
        const uint32_t* kw = reinterpret_cast<const uint32_t*>(blob + r.m.w);
        for (int j = VC_REC_INLINE / 4; 4 * j < n; ++j)
            if (q.word(st + 4 * j, st, st + n) != kw[j]) return false;
    }
    return true;
}

template <class T>
VC_HD T gload(const T* p);

// Record s's key == query bytes [st, st + n)?  *meta = its meta word on a
// match.  The meta and the first 32 key bytes are loaded together; the last
// 16 inline bytes only when some lane's key is longer.
template <class Src>
VC_HD bool rec_match(const HostRec* recs, uint32_t s, const uint8_t* blob, const Src& q, int st,
                     int n, uint4* meta) {
    const uint4* p = reinterpret_cast<const uint4*>(recs + s);
#if defined(VC_ABL_NOREC)          // timing ablation only: no record load
    if (s != 0xFFFFFFFFu) {
        *meta = uint4{uint32_t(n), 0u, 0u, 0u};
        return true;
    }
#endif
    const uint4 m = gload(p), k0 = gload(p + 1), k1 = gload(p + 2);
    int rn = int(m.x & VC_REC_LEN);
    if (rn != n) return false;
#if defined(__HIP_DEVICE_COMPILE__)
    asm volatile("" : "+v"(rn));
#endif
    uint32_t diff = 0;
    const auto c = q.cursor(st, st + n);
    {
        const uint32_t k[8] = {k0.x, k0.y, k0.z, k0.w, k1.x, k1.y, k1.z, k1.w};
#pragma unroll
        for (int j = 0; j < 8; ++j) {
            if (!wave_any(4 * j < rn)) break;
            if (4 * j < rn) {
                uint32_t d = c.get(j) ^ k[j];
                if (4 * j + 4 > rn) d &= tail_mask(rn - 4 * j);
                diff |= d;
            }
        }
    }
    if (wave_any(rn > 32) && rn > 32) {
        const uint4 k2 = gload(p + 3);
        const uint32_t k[4] = {k2.x, k2.y, k2.z, k2.w};
#pragma unroll
        for (int j = 8; j < 12; ++j) {
            if (4 * j < rn) {
                uint32_t d = c.get(j) ^ k[j - 8];
                if (4 * j + 4 > rn) d &= tail_mask(rn - 4 * j);
                diff |= d;
            }
        }
    }
    if (diff) return false;
    if (n > VC_REC_INLINE) {      // long key: the rest from the blob copy
        const uint32_t* kw = reinterpret_cast<const uint32_t*>(blob + m.w);
        for (int j = VC_REC_INLINE / 4; 4 * j < n; ++j)
            if (q.word(st + 4 * j, st, st + n) != kw[j]) return false;
    }
    *meta = m;
    return true;
}

// Global-memory load through an explicitly global pointer: table pointers
// travel inside image structs, where the compiler cannot infer the address
// space and would emit flat loads.
template <class T>
VC_HD T gload(const T* p) {
#if defined(__HIP_DEVICE_COMPILE__)
    return *(const __attribute__((address_space(1))) T*)(p);
#else
    return *p;
#endif
}

VC_HD uint4 tag_group(const uint32_t* tags, uint32_t mask, uint32_t h) {
#if defined(VC_ABL_NOTAG)          // timing ablation only: every probe misses
    if (h == 0x12345u) return gload(reinterpret_cast<const uint4*>(tags));
    return uint4{0u, 0u, 0u, 0u};
#endif
    return gload(reinterpret_cast<const uint4*>(tags + (h & mask & ~3u)));
}

VC_HD Rec load_rec_g(const HostRec* r, uint32_t s) {
    const uint4* p = reinterpret_cast<const uint4*>(r + s);
    return Rec{gload(p), gload(p + 1), gload(p + 2), gload(p + 3)};
}

// Tag matches of a 4-slot group that belong to the probe chain (before the
// group's first empty slot), bits 0-3; bit 4 set when the group has no
// empty slot (the chain continues into the next group).
VC_HD uint32_t group_hits(uint4 g, uint32_t want) {
    const uint32_t tg[4] = {g.x, g.y, g.z, g.w};
    uint32_t m = 0, open = 0;
#pragma unroll
    for (int k = 0; k < 4; ++k) {
        if (!open && tg[k] == want) m |= 1u << k;
        if (tg[k] == 0) open = 1;
    }
    return open ? m : (m | 16u);
}

// slot of key [st, st + n) with hash h; -1 if absent.  *out = its record.
// m0: group_hits of the first tag group when the caller already holds it
// (host_only_fast loads every probe's first group up front), else ~0u.
template <class Src>
VC_HD int host_find(const HostTable& t, uint32_t h, const Src& q, int st, int n, Rec* out,
                    uint32_t m0 = ~0u) {
    const uint32_t want = h | 1u;
    uint32_t s = h & t.mask & ~3u;
    for (;;) {
        uint32_t m = m0 != ~0u ? m0
                               : group_hits(gload(reinterpret_cast<const uint4*>(t.tags + s)), want);
        m0 = ~0u;
        while (m & 15u) {
            const uint32_t k = __builtin_ctz(m);
            m &= m - 1;
            if (rec_match(t.recs, s + k, t.blob, q, st, n, &out->m)) return int(s + k);
        }
        if (!(m & 16u)) return -1;
        s = (s + 4) & t.mask;
    }
}

VC_HD HostTable host_table(const HintImage& img) {
    return HostTable{img.host_tags, img.host_recs, img.blob, img.host_mask};
}

// port filter over a key's distinct hint-port minima (rare: out of line)
__host__ __device__ __noinline__ uint32_t pick_ports(const HostExt* ext, const PortMin* pms,
                                                      int slot, uint32_t v, int port) {
    const HostExt x = ext[slot];
    for (uint32_t i = 0; i < x.pm_cnt; ++i) {
        const PortMin pm = pms[x.pm_off + i];
        if (pm.port == port) v = uint32_t(pm.idx) < v ? uint32_t(pm.idx) : v;
    }
    return v;
}

// min handle index of a hint-host key not excluded by the port filter
// (Hint.java:124-128): port == 0 -> any; else hint-port 0 or equal.
VC_HD uint32_t pick(const HintImage& img, int slot, const Rec& r, int port) {
    if (port == 0) return r.m.y;
    if (!(r.m.x & VC_REC_HAS_PM)) return r.m.z;
    return pick_ports(img.host_ext, img.port_mins, slot, r.m.z, port);
}

// Hash of [st, e) of a source (khash over a source, a word at a time).
template <class Src>
VC_HD uint32_t src_khash(const Src& q, int st, int e) {
    uint32_t S = vck::kSeed;
    for (int pos = e - 4; pos > st - 4; pos -= 4) S = vck::mix(S, q.down(pos, st, e));
    return vck::fin(S, uint32_t(e - st));
}

// Exact lookup of [st, st + n).
template <class Src>
VC_HD int host_lookup(const HostTable& t, const Src& q, int st, int n, Rec* out) {
    return host_find(t, src_khash(q, st, st + n), q, st, n, out);
}

// the "*" record's meta from the image (HintImage.wild_*: no table load)
VC_HD Rec wildcard_rec(const HintImage& img) {
    Rec r{};
    r.m = uint4{img.wild_len_pm, uint32_t(img.wild_a), uint32_t(img.wild_b), 0u};
    return r;
}

VC_HD uint32_t wildcard_pick(const HintImage& img, int port) {
    if (img.wildcard_slot < 0) return VC_NONE;
    return pick(img, img.wildcard_slot, wildcard_rec(img), port);
}

// The deferring fast path (kDefer below) leaves a lane that needs an
// out-of-line step -- the port filter over a key's distinct hint-port
// minima, a name the word scan does not cover, an unstaged chunk -- marked
// with kDeferred (defined with host_only_fast) for the reference-shaped
// pass that follows the kernel (hint.hip hint_defer_kernel), so the
// kernel's loop contains no call: a call site inside it makes the compiler
// keep the loop's state in scratch and spill SGPRs across the call on every
// chunk.

template <bool kDefer>
VC_HD uint32_t pick_or_defer(const HintImage& img, int slot, const Rec& r, int port,
                             bool* defer) {
    if (!kDefer) return pick(img, slot, r, port);
    if (port == 0) return r.m.y;
    if (!(r.m.x & VC_REC_HAS_PM)) return r.m.z;
    *defer = true;
    return VC_NONE;
}

template <bool kDefer>
VC_HD uint32_t wildcard_pick_or_defer(const HintImage& img, int port, bool* defer) {
    if (!kDefer) return wildcard_pick(img, port);
    if (img.wildcard_slot < 0) return VC_NONE;
    return pick_or_defer<true>(img, img.wildcard_slot, wildcard_rec(img), port, defer);
}

// ---------------------------------------------------------------------------
// Upstream.searchForGroup for hints whose uri is null (or when no group has
// a hint-uri): level = hostLevel << 10, so exact (3) beats any suffix (2)
// beats "*" (1), and within a level the lowest handle index wins (strict
// '>' scan, Upstream.java:187-198).
// ---------------------------------------------------------------------------

// The dots of [s, e), right to left, up to eight (d0 the last found, the
// leftmost; more: the caller scans on left of d0).
// Probing the k-th suffix of every lane in the same loop trip keeps a
// wave's lanes together: probing each at its byte position ran one round
// of dependent table loads per distinct dot position in the wave.
struct Dots {
    int d0 = 0, d1 = 0, d2 = 0, d3 = 0, d4 = 0, d5 = 0, d6 = 0, d7 = 0;
    int n = 0;
    bool more = false;
    VC_HD int at(int k) const {
        return k == 0 ? d0 : k == 1 ? d1 : k == 2 ? d2 : k == 3 ? d3
             : k == 4 ? d4 : k == 5 ? d5 : k == 6 ? d6 : d7;
    }
};

VC_HD Dots find_dots(const uint8_t* p, int s, int e) {
    Dots x;
    for (int j = e - 1; j >= s; --j) {
        if (p[j] != '.') continue;
        if (x.n == 8) {
            x.more = true;
            break;
        }
        x.d7 = x.d6; x.d6 = x.d5; x.d5 = x.d4; x.d4 = x.d3;
        x.d3 = x.d2; x.d2 = x.d1; x.d1 = x.d0; x.d0 = j;
        ++x.n;
    }
    return x;
}

// Reference-shaped form over a formatted host [s, e) of a plain string: any
// number of labels, each dot-suffix probed as it is found.  Out of line: the
// kernels reach it only for names the fast path does not take.
__host__ __device__ __noinline__ int32_t host_only_seq(const HintImage& img, const uint8_t* p,
                                                       int s, int e, int port) {
    const HostTable t = host_table(img);
    const PtrSrc q{p};
    Rec r;
    int slot = host_lookup(t, q, s, e - s, &r);
    if (slot >= 0) {
        const uint32_t v = pick(img, slot, r, port);
        if (v != VC_NONE) return int32_t(v);
    }
    uint32_t best = VC_NONE;
    const Dots dots = find_dots(p, s, e);
    for (int k = 0; k < dots.n; ++k) {
        const int j = dots.at(k);
        slot = host_lookup(t, q, j + 1, e - j - 1, &r);
        if (slot >= 0) {
            const uint32_t v = pick(img, slot, r, port);
            best = v < best ? v : best;
        }
    }
    if (dots.more) {                    // past the eighth dot from the right
        for (int j = dots.d0 - 1; j >= s; --j) {
            if (p[j] != '.') continue;
            slot = host_lookup(t, q, j + 1, e - j - 1, &r);
            if (slot >= 0) {
                const uint32_t v = pick(img, slot, r, port);
                best = v < best ? v : best;
            }
        }
    }
    if (best != VC_NONE) return int32_t(best);
    const uint32_t v = wildcard_pick(img, port);
    return v != VC_NONE ? int32_t(v) : -1;
}

// Formatted host given as a plain string (the general path, the harness).
VC_HDN int32_t hint_host_only(const HintImage& img, DStr host, int port) {
    if (host.n < 0) return -1;
    return host_only_seq(img, host.p, 0, host.n, port);
}

// Hint.formatHost + host-only search on a raw host of a plain string.
__host__ __device__ __noinline__ int32_t host_only_slow(const HintImage& img, const uint8_t* p,
                                                        int n, int port) {
    return hint_host_only(img, format_host(DStr{p, n}), port);
}

constexpr int kMaxSuffix = 6;
constexpr int kProbes = kMaxSuffix + 1;      // [0] = the whole host

// Fast path: one right-to-left word scan of the raw host [0, n) computes
// Hint.formatHost's cut at the first ':' (restarting the scan there) and the
// hash of the host and of every dot-suffix; all first tag groups are then
// loaded together, and only tag hits touch a record.  Names the scan does
// not cover (two or more ':' -- a possible IPv6 literal -- or more than
// kMaxSuffix labels) go to the reference-shaped slow path.
//
// uri (kDefer only): the hint also has a uri and port 0 -- Hint.ofHostUri,
// what HttpContext.connectionHint sends (HttpContext.java:55-71).  Then
// level(g) = hostLevel(g) << 10 + uriLevel(g) (Hint.java:100-160) with
// uriLevel <= 1023, so the winner is among the groups at the top host level
// L, ordered by uriLevel and then index.  When L's groups are one key's
// members and that key is not VC_REC_SPLIT (one member, or none with a
// hint-uri), or several keys none of whose members has a hint-uri
// (VC_REC_ANYURI), every candidate has the same uriLevel and the host-only
// answer -- the lowest index at L -- is the answer.  When they are one
// SPLIT key's members the result is uri_slot_code(slot): the caller scores
// that key's members by uriLevel (uri_in_slot).  Otherwise (several keys at
// L with a hint-uri among them, or no host key at all, L = 0: the uri alone
// decides) the lane is deferred to the general search.
constexpr int32_t kDeferred = INT32_MIN;

// host_only_fast's answer for a uri lane whose top host level is one SPLIT
// key: -2 - slot (below -1, above kDeferred)
VC_HD int32_t uri_slot_code(int slot) { return -2 - slot; }
VC_HD bool is_uri_slot_code(int32_t r) { return r < -1 && r != kDeferred; }

template <bool kDefer = false, class Src>
VC_HD int32_t host_only_fast(const HintImage& img, const HintImage* slow_img, const Src& q, int n,
                             int port, bool uri = false) {
#if defined(VC_ABL_NOSCAN)         // timing ablation only: stage, no scan
    if (n != 0x7FFFFFFF) return int32_t(q.word(0, 0, n) & 1u) - 1;
#endif
    uint32_t h[kProbes];
    uint64_t stp = 0;                 // suffix starts, a byte each: [k] at bits 8k
    int e = n, np = 0, nc = 0;
    uint32_t S = vck::kSeed;
    for (int pos = n - 4; pos > -4;) {
        // every word read here ends at or before e: only bytes below 0 to drop
        const uint32_t valid = lo_mask(pos, 0);
        const uint32_t w = q.down(pos, 0, e);
        const uint32_t cf = vck::byte_eq_flags(w, 0x3A3A3A3Au) & valid;
        if (cf) {                       // restart at the leftmost ':' so far
            nc += __builtin_popcount(cf);
            e = pos + (__builtin_ctz(cf) >> 3);
            pos = e - 4;
            S = vck::kSeed;
            np = 0;
            continue;
        }
        uint32_t df = vck::byte_eq_flags(w, 0x2E2E2E2Eu) & valid;
        while (df) {                    // rightmost dot first: shortest suffix first
            const int b = (31 - __builtin_clz(df)) >> 3;
            df &= ~(0x80u << (8 * b));
            const int sp = pos + b + 1;
            const uint32_t len = uint32_t(e - sp);
            const uint32_t hv = b == 3 ? vck::fin(S, len)
                                       : vck::fin(vck::mix(S, w & (~0u << (8 * (b + 1)))), len);
            ++np;
            // shift in: [1] = the latest (longest) suffix.  Plain moves under
            // the lanes-with-a-dot mask, no per-slot compare and select.
#pragma unroll
            for (int k = kProbes - 1; k > 1; --k) h[k] = h[k - 1];
            h[1] = hv;
            stp = ((stp & 0xFFFFFFFFFF00ull) << 8) | (uint64_t(sp) << 8);
        }
        S = vck::mix(S, w);
        pos -= 4;
    }
    VC_PMARK(1);
    if (nc >= 2 || np > kMaxSuffix || n > 255) {
        if (kDefer) return kDeferred;
        return host_only_slow(*slow_img, q.ptr(), n, port);
    }
    h[0] = vck::fin(S, uint32_t(e));
    if (nc) {
        // cut at the colon; strip "www." (then the whole host is the suffix
        // after the dot at 3, the longest, in [1]); empty -> null
        if (e >= 4 && q.word(0, 0, 4) == 0x2E777777u) {
            h[0] = h[1];
#pragma unroll
            for (int k = 1; k < kProbes - 1; ++k) h[k] = h[k + 1];
            stp = stp >> 8;
            np -= 1;
        }
        if (e - int(stp & 0xFF) <= 0) return kDefer && uri ? kDeferred : -1;   // null host
    }
    const HostTable t = host_table(img);
    // hits: bit k = probe k's first group has a tag match or continues;
    // tm: its 4 match bits at 4k; cont: bit k = it continues (group_hits bit 4)
    uint32_t hits = 0, tm = 0, cont = 0;
    {
        // all first tag groups in flight together; g[k] is read only where
        // it was loaded (k <= np), so it needs no initial value
        uint4 g[kProbes];
#pragma unroll
        for (int k = 0; k < kProbes; ++k)
            if (k <= np) g[k] = tag_group(t.tags, t.mask, h[k]);
#pragma unroll
        for (int k = 0; k < kProbes; ++k) {
            if (k <= np) {
                const uint32_t m = group_hits(g[k], h[k] | 1u);
                tm |= (m & 15u) << (4 * k);
                cont |= ((m >> 4) & 1u) << k;
                hits |= (m != 0u ? 1u : 0u) << k;
            }
        }
    }
    VC_PMARK(2);
    uint32_t best = VC_NONE;
    bool defer = false;
    int nsuf = 0;                     // suffix keys at level 2 (uri lanes)
    uint32_t uflags = 0;              // their len_pm words, or-ed
    int sslot = 0;                    // the (last) one's slot
    while (hits) {
        const int k = __builtin_ctz(hits);
        hits &= hits - 1;
        uint32_t hk = h[0];
#pragma unroll
        for (int j = 1; j < kProbes; ++j) hk = k == j ? h[j] : hk;
        const int sk = int((stp >> (8 * k)) & 0xFF);
        Rec r;
        const uint32_t m0 = ((tm >> (4 * k)) & 15u) | (((cont >> k) & 1u) << 4);
        const int slot = host_find(t, hk, q, sk, e - sk, &r, m0);
        if (slot < 0) continue;
        const uint32_t v = pick_or_defer<kDefer>(img, slot, r, port, &defer);
        if (k == 0) {
            if (v != VC_NONE) {                            // exact level wins
                if (kDefer && uri && (r.m.x & VC_REC_SPLIT)) return uri_slot_code(slot);
                return kDefer && defer ? kDeferred : int32_t(v);
            }
        } else {
            best = v < best ? v : best;
            if (v != VC_NONE) {
                ++nsuf;
                uflags |= r.m.x;
                sslot = slot;
            }
        }
    }
    VC_PMARK(3);
    if (kDefer && uri) {
        if (best != VC_NONE) {
            if (nsuf > 1 && (uflags & VC_REC_ANYURI)) return kDeferred;
            if (nsuf == 1 && (uflags & VC_REC_SPLIT)) return uri_slot_code(sslot);
        } else {
            best = wildcard_pick_or_defer<kDefer>(img, port, &defer);
            if (best == VC_NONE) return kDeferred;        // no host level: the uri decides
            if (img.wild_len_pm & VC_REC_SPLIT) return uri_slot_code(img.wildcard_slot);
        }
    }
    if (best == VC_NONE) best = wildcard_pick_or_defer<kDefer>(img, port, &defer);
    if (kDefer && defer) return kDeferred;
    return best != VC_NONE ? int32_t(best) : -1;
}

// Hint.formatUri's length (Hint.java:75-90: cut at the first '?'; "/"
// stays, else one trailing '/' goes) of a uri in global memory.  Up to 60
// bytes its aligned words are loaded together and searched a word at a time
// (a byte loop with an exit per byte is one dependent load per byte); an
// aligned word holding a byte of the uri never crosses a page.
VC_HD int format_uri_len(const uint8_t* p, int n) {
    if (n > 60) return format_uri(DStr{p, n}).n;
    const uintptr_t a = reinterpret_cast<uintptr_t>(p);
    const uint32_t* w = reinterpret_cast<const uint32_t*>(a & ~uintptr_t(3));
    const int sh = int(a & 3), nw = (sh + n + 3) >> 2;
    uint32_t x[16];
#pragma unroll
    for (int k = 0; k < 16; ++k) x[k] = k < nw ? gload(w + k) : 0u;
    int m = n;
#pragma unroll
    for (int k = 15; k >= 0; --k) {              // the first '?' wins: scan down
        const int b0 = 4 * k - sh;               // uri position of the word's byte 0
        uint32_t f = vck::byte_eq_flags(x[k], 0x3F3F3F3Fu);
        f &= lo_mask(b0, 0) & (b0 + 4 <= n ? ~0u : tail_mask(n - b0 > 0 ? n - b0 : 0));
        if (k < nw && f) m = b0 + (__builtin_ctz(f) >> 3);
    }
    if (m == 1 && p[0] == '/') return 1;
    return m > 0 && p[m - 1] == '/' ? m - 1 : m;
}

// Upstream.searchForGroup for a port-0 uri hint whose top host level is
// one key's members (host_only_fast's uri_slot_code): they share the host
// level, so the highest uriLevel wins and then the lowest index (the list
// ascends; strict '>'), Hint.java:144-157 -- uriLevel = U.length() + 1 when
// the uri starts with U (equal included), 1 for "*", capped at 1023.  A
// member list longer than 32 goes to the general search.
// Scores host slot `slot`'s members by uriLevel against the formatted uri
// up[0, m) into (*lvl, *best): a higher level wins, then the lower index.
VC_HD void score_slot(const HintImage& img, int slot, const uint8_t* up, int m, int* lvl,
                      int32_t* best) {
    const HostExt x = gload(img.host_ext + slot);
    for (uint32_t i = 0; i < x.list_cnt; ++i) {
        const uint32_t g = gload(img.lists + x.list_off + i);
        const int4 r = gload(reinterpret_cast<const int4*>(img.groups) + 2 * g);
        const int4 r2 = gload(reinterpret_cast<const int4*>(img.groups) + 2 * g + 1);
        const int Un = r.z;
        int ul = 0;
        if (Un >= 0) {
            const uint8_t* U = img.blob + uint32_t(r.w);
            if (Un <= m && bytes_eq(U, up, Un)) ul = r2.z + 1;
            else if (Un == 1 && U[0] == '*') ul = 1;
            ul = ul > 1023 ? 1023 : ul;
        }
        if (ul > *lvl || (ul == *lvl && (*best < 0 || int32_t(g) < *best))) {
            *lvl = ul;
            *best = int32_t(g);
        }
    }
}

VC_HD int32_t uri_in_slot(const HintImage& img, int slot, const uint8_t* up, int un) {
    const HostExt x = gload(img.host_ext + slot);
    if (x.list_cnt > 32) return kDeferred;
    const int m = format_uri_len(up, un);
    int32_t best = int32_t(gload(img.lists + x.list_off));
    int lvl = 0;
    for (uint32_t i = 0; i < x.list_cnt; ++i) {
        const uint32_t g = gload(img.lists + x.list_off + i);
        // GroupRec: {host_len, host_off, uri_len, uri_off}, {port, any, uri_units, pad}
        const int4 r = gload(reinterpret_cast<const int4*>(img.groups) + 2 * g);
        const int4 r2 = gload(reinterpret_cast<const int4*>(img.groups) + 2 * g + 1);
        const int Un = r.z;
        if (Un < 0) continue;                                      // no hint-uri: 0
        const uint8_t* U = img.blob + uint32_t(r.w);
        int ul = 0;
        if (Un <= m && bytes_eq(U, up, Un)) ul = r2.z + 1;
        else if (Un == 1 && U[0] == '*') ul = 1;
        ul = ul > 1023 ? 1023 : ul;
        if (ul > lvl) {
            lvl = ul;
            best = int32_t(g);
        }
    }
    return best;
}

// ---------------------------------------------------------------------------
// URI keys (forward FNV-1a, 32-byte KeySlot): general path only
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

VC_HDN int uri_probe(const HintImage& img, uint32_t h, const uint8_t* p, int n, KeySlot* out) {
    const uint32_t want = h | 1u;
    uint32_t s = h & img.uri_mask & ~3u;
    for (;;) {
        const uint4 g = *reinterpret_cast<const uint4*>(img.uri_tags + s);
        const uint32_t tg[4] = {g.x, g.y, g.z, g.w};
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            if (tg[k] == 0) return -1;
            if (tg[k] == want) {
                KeySlot ks = load_slot(img.uri_slots, s + k);
                if (ks.key_len == n && bytes_eq(img.blob + ks.key_off, p, n)) {
                    *out = ks;
                    return int(s + k);
                }
            }
        }
        s = (s + 4) & img.uri_mask;
    }
}

// Hint.matchLevel for one merged group (Hint.java:100-160)
VC_HDN int match_level(const HintImage& img, uint32_t g, DStr host, int port, DStr uri) {
    const int32_t* r = reinterpret_cast<const int32_t*>(img.groups) + 8 * g;
    const int32_t Hn = r[0], Un = r[2], P = r[4], Uu = r[6];
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
        // uri.length() == U.length() when equal: both levels are U's UTF-16
        // length + 1 (strings are UTF-8 here, Java counts UTF-16 units)
        if (uri.n >= Un && bytes_eq(uri.p, U, Un)) ul = Uu + 1;
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

VC_HDN void consider_members(const HintImage& img, uint32_t off, uint32_t cnt, DStr host,
                             int port, DStr uri, Best* b) {
    for (uint32_t i = 0; i < cnt; ++i) {
        uint32_t g = img.lists[off + i];
        b->consider(match_level(img, g, host, port, uri), int32_t(g));
    }
}

VC_HDN void consider_host_slot(const HintImage& img, int slot, DStr host, int port, DStr uri,
                               Best* b) {
    const HostExt x = img.host_ext[slot];
    consider_members(img, x.list_off, x.list_cnt, host, port, uri, b);
}

// General searchForGroup: every group with a nonzero level has its hint-host
// equal to / a dot-suffix of / "*" for the host, or its hint-uri a prefix
// of / "*" for the uri; those candidate lists are scored exactly.
// q serves host's bytes (a PtrSrc on host.p, or the LDS stage holding them)
template <class Src>
__host__ __device__ __noinline__ int32_t hint_general_src(const HintImage& img, DStr host,
                                                          const Src& q, int port, DStr uri) {
    Best b;
    if (host.n >= 0) {
        const HostTable t = host_table(img);
        Rec r;
        const Dots dots = find_dots(host.p, 0, host.n);
        for (int k = 0; k < dots.n; ++k) {
            const int j = dots.at(k);
            const int slot = host_lookup(t, q, j + 1, host.n - j - 1, &r);
            if (slot >= 0) consider_host_slot(img, slot, host, port, uri, &b);
        }
        if (dots.more) {                // past the eighth dot from the right
            for (int j = dots.d0 - 1; j >= 0; --j) {
                if (host.p[j] != '.') continue;
                const int slot = host_lookup(t, q, j + 1, host.n - j - 1, &r);
                if (slot >= 0) consider_host_slot(img, slot, host, port, uri, &b);
            }
        }
        const int slot = host_lookup(t, q, 0, host.n, &r);
        if (slot >= 0) consider_host_slot(img, slot, host, port, uri, &b);
        if (img.wildcard_slot >= 0) consider_host_slot(img, img.wildcard_slot, host, port, uri, &b);
    }
    if (uri.n >= 0) {
        // Members of one hint-uri share its uri level c, so member g scores
        // (hostLevel(g) << 10) + c.  With port 0 no hint-port excludes any,
        // and a member with hostLevel > 0 sits in a host slot probed above,
        // scored exactly there; so the list's first member (scored exactly)
        // decides what the list can add: HTTP hints (port 0) under a "/" or
        // "*" hint-uri shared by thousands of groups no longer scan them all.
        KeySlot k;
        uint32_t h = kFnvBasis;
        const uint64_t lens = uint64_t(img.uri_len_hi) << 32 | img.uri_len_lo;
        for (int j = 0; j <= uri.n; ++j) {
            if (((lens >> (j < 63 ? j : 63)) & 1u) && uri_probe(img, h, uri.p, j, &k) >= 0)
                consider_members(img, k.list_off, port == 0 && k.list_cnt ? 1u : k.list_cnt,
                                 host, port, uri, &b);
            if (j < uri.n) h = fnv_step(h, uri.p[j]);
        }
        if (img.uri_star_slot >= 0) {
            const KeySlot u = load_slot(img.uri_slots, uint32_t(img.uri_star_slot));
            consider_members(img, u.list_off, port == 0 && u.list_cnt ? 1u : u.list_cnt, host,
                             port, uri, &b);
        }
    }
    return b.idx;
}

__host__ __device__ __noinline__ int32_t hint_general(const HintImage& img, DStr host, int port,
                                                      DStr uri) {
    return hint_general_src(img, host, PtrSrc{host.p}, port, uri);
}

// searchForGroup(Hint.ofHostUri(host, uri)) -- port 0, a non-null uri --
// by levels (Hint.java:100-160, Upstream.java:187-198), for the lanes the
// fast path leaves: every group at the top host level L beats every group
// below it (uriLevel <= 1023), so only L's keys are scored, their members
// by uriLevel and then index; with no host level (L = 0) the uri alone
// decides -- the longest hint-uri that prefixes the uri (one level per
// length; "" and "*" share level 1), its first member.  host / uri raw
// (formatted here), in global memory.
// hint_port0_levels: the same over a formatted host and the formatted uri
// up[0, m) (formatUri is not idempotent: "/a//" -> "/a/" -> "/a").
__host__ __device__ __noinline__ int32_t hint_port0_levels(const HintImage& img, DStr host,
                                                           const uint8_t* up, int m) {
    int lvl = 0;
    int32_t best = -1;
    if (host.n >= 0) {
        const HostTable t = host_table(img);
        const PtrSrc q{host.p};
        Rec r;
        int slot = host_lookup(t, q, 0, host.n, &r);
        if (slot >= 0) {                                    // level 3: the exact key
            score_slot(img, slot, up, m, &lvl, &best);
            return best;
        }
        const Dots dots = find_dots(host.p, 0, host.n);
        bool any = false;
        for (int k = 0; k < dots.n; ++k) {                  // level 2: every dot-suffix key
            const int j = dots.at(k);
            slot = host_lookup(t, q, j + 1, host.n - j - 1, &r);
            if (slot >= 0) {
                score_slot(img, slot, up, m, &lvl, &best);
                any = true;
            }
        }
        if (dots.more)
            for (int j = dots.d0 - 1; j >= 0; --j) {
                if (host.p[j] != '.') continue;
                slot = host_lookup(t, q, j + 1, host.n - j - 1, &r);
                if (slot >= 0) {
                    score_slot(img, slot, up, m, &lvl, &best);
                    any = true;
                }
            }
        if (any) return best;
        if (img.wildcard_slot >= 0) {                       // level 1: "*"
            score_slot(img, img.wildcard_slot, up, m, &lvl, &best);
            return best;
        }
    }
    // level 0: the uri alone (port 0: a key's members share its level, the
    // first is the lowest index)
    const uint64_t lens = uint64_t(img.uri_len_hi) << 32 | img.uri_len_lo;
    uint32_t h = kFnvBasis;
    KeySlot k;
    for (int j = 0; j <= m; ++j) {
        if (((lens >> (j < 63 ? j : 63)) & 1u) && uri_probe(img, h, up, j, &k) >= 0 && k.list_cnt) {
            const int32_t g = int32_t(img.lists[k.list_off]);
            const int ul = (j == 0 ? 0 : img.groups[g].uri_units) + 1;
            const int cl = ul > 1023 ? 1023 : ul;
            if (cl > lvl || (cl == lvl && g < best)) {
                lvl = cl;
                best = g;
            }
        }
        if (j < m) h = fnv_step(h, up[j]);
    }
    if (img.uri_star_slot >= 0) {
        const KeySlot u = load_slot(img.uri_slots, uint32_t(img.uri_star_slot));
        if (u.list_cnt) {
            const int32_t g = int32_t(img.lists[u.list_off]);
            if (1 > lvl || (1 == lvl && g < best)) {
                lvl = 1;
                best = g;
            }
        }
    }
    return best;
}

__host__ __device__ __noinline__ int32_t hint_port0_uri(const HintImage& img, DStr host_raw,
                                                        const uint8_t* up, int un) {
    return hint_port0_levels(img, format_host(host_raw), up, format_uri_len(up, un));
}

VC_HD int32_t search_for_group(const HintImage& img, DStr host, int port,
                                                    DStr uri) {
    if (uri.n < 0 || !img.has_uri_keys) return hint_host_only(img, host, port);
    return hint_general(img, host, port, uri);
}

// kind of a DNS query the deferring kernel leaves to its second pass
constexpr uint8_t kDnsDeferred = 0xFF;

// Could [0, n) be an IP literal (IP.isIpLiteral)?  Only hex digits, '.',
// ':', '[' and ']' occur in one; any other byte rules it out.
template <class Src>
VC_HD bool maybe_ip_literal(const Src& q, int n) {
    for (int pos = 0; pos < n; pos += 4) {
        const uint32_t w = q.word(pos, 0, n);
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            if (pos + j >= n) break;
            const uint32_t c = (w >> (8 * j)) & 0xFFu, l = c | 0x20u;
            if (!((c >= '0' && c <= '9') || (l >= 'a' && l <= 'f') || c == '.' || c == ':' ||
                  c == '[' || c == ']'))
                return false;
        }
    }
    return true;
}

// DNSServer.handleRequest classification (DNSServer.java:116-166) on a
// query name in the boundary's string encoding (UTF-8), trailing dot
// included.  kDefer: no out-of-line call -- a name the host scan does not
// cover, or one that may be an IP literal, gets kind kDnsDeferred for the
// second pass (hint.hip dns_defer_kernel).
template <bool kDefer = false, class Src>
VC_HD void dns_flow(const HostsImage& hosts, const HintImage& img, const HintImage* slow_img,
                    const Src& q, int qn, uint8_t* kind, int32_t* value) {
    // (1) hosts.get(qname) on the raw qname (trailing dot kept), :127
    if (hosts.n > 0) {
        Rec r;
        const HostTable t{hosts.tags, hosts.recs, hosts.blob, hosts.mask};
        if (host_lookup(t, q, 0, qn, &r) >= 0) {
            *kind = VC_DNS_HOSTS;
            *value = int32_t(r.m.y);
            return;
        }
    }
    VC_PMARK(4);
    // (2) strip one trailing dot, :133-135
    const uint8_t* qp = q.ptr();
    const int dn = (qn > 0 && (q.word(qn - 1, qn - 1, qn) & 0xFFu) == '.') ? qn - 1 : qn;
    // (3) rrsets.searchForGroup(Hint.ofHost(domain)), :136
    const int32_t g = host_only_fast<kDefer>(img, slow_img, q, dn, 0);
    if (kDefer && (g == kDeferred || (g < 0 && maybe_ip_literal(q, dn)))) {
        *kind = kDnsDeferred;
        *value = 0;
    } else if (g >= 0) {
        *kind = VC_DNS_GROUP;
        *value = g;
    } else if (!kDefer && d_is_ip_literal(qp, dn)) {  // (4) IP literal, :140-149
        *kind = VC_DNS_IP_LITERAL;
        *value = d_count(qp, dn, ':') ? 6 : 4;
    } else {                                          // (5) *.vproxy.local, :150-157
        const char* sfx = ".vproxy.local";
        bool internal = dn >= 13;
        for (int j = 0; internal && j < 13; ++j) internal = qp[dn - 13 + j] == uint8_t(sfx[j]);
        *kind = internal ? VC_DNS_INTERNAL : VC_DNS_RECURSIVE;   // (6) :164
        *value = 0;
    }
}

// Formatter.parseDomainName appends (char) b per wire byte b, a Java byte:
// the cast sign-extends (JLS 5.1.4), so a byte c >= 0x80 is the char
// U+FF00 | c, whose UTF-8 form is EF (BE | BF) (80 | c & 3F).  The rare
// qname with such bytes is transcoded into a private buffer and classified
// from there.  Wire names are at most 255 bytes; a non-ASCII name over 512
// bytes is reported as recursive.
VC_HDN __noinline__ void dns_highbytes(const HostsImage& hosts, const HintImage* slow_img,
                                       const uint8_t* qp, int qn, uint8_t* kind, int32_t* value) {
    uint8_t buf[1536];
    if (qn > 512) {
        *kind = VC_DNS_RECURSIVE;
        *value = 0;
        return;
    }
    int n = 0;
    for (int i = 0; i < qn; ++i) {
        const uint8_t c = qp[i];
        if (c < 0x80) {
            buf[n++] = c;
        } else {
            buf[n++] = 0xEF;
            buf[n++] = uint8_t(0xBC | (c >> 6));
            buf[n++] = uint8_t(0x80 | (c & 0x3F));
        }
    }
    dns_flow(hosts, *slow_img, slow_img, PtrSrc{buf}, n, kind, value);
}

// DNSServer classification on the wire bytes of a query name
// (Formatter.parseDomainName output, trailing dot included).
template <bool kDefer = false, class Src>
VC_HD void dns_one(const HostsImage& hosts, const HintImage& img, const HintImage* slow_img,
                   const Src& q, int qn, uint8_t* kind, int32_t* value) {
    uint32_t hi = 0;
    for (int pos = 0; pos < qn; pos += 4) hi |= q.word(pos, 0, qn);
    if (hi & 0x80808080u) {
        if (kDefer) {
            *kind = kDnsDeferred;
            *value = 0;
        } else {
            dns_highbytes(hosts, slow_img, q.ptr(), qn, kind, value);
        }
    } else {
        dns_flow<kDefer>(hosts, img, slow_img, q, qn, kind, value);
    }
}

// SSLContextHolder.choose(sni) (SSLContextHolder.java:51-79) over the
// CertImage table (common/images.h): no holder -> -1 (null), one holder or
// a null SNI or no match -> 0 (the default, first holder).
template <class Src>
VC_HD int32_t cert_one(const CertImage& c, const Src& q, int n, bool sni_null) {
    if (c.n_holders <= 0) return -1;
    if (c.n_holders == 1 || sni_null || c.names.n == 0) return 0;
    const HostTable t{c.names.tags, c.names.recs, c.names.blob, c.names.mask};
    uint32_t best = VC_NONE;
    Rec r;
    if (host_lookup(t, q, 0, n, &r) >= 0) best = r.m.y;              // plain: sni.equals(name)
    int dot = -1;                                                     // first '.' of the SNI
    for (int pos = 0; pos < n && dot < 0; pos += 4) {
        const uint32_t f = vck::byte_eq_flags(q.word(pos, 0, n), 0x2E2E2E2Eu) &
                           (keep_mask(pos, 0, n) & 0x80808080u);
        if (f) dot = pos + (__builtin_ctz(f) >> 3);
    }
    if (dot > 0 && host_lookup(t, q, dot, n - dot, &r) >= 0)         // wildcard "*" + sni[dot:]
        best = r.m.z < best ? r.m.z : best;
    return best == VC_NONE ? 0 : int32_t(best);
}

}  // namespace vcd

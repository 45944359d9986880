// mirror_dev.h -- the traffic-mirror filter checks:
//
//   FilterConfig.matchEthernet / matchIp / matchTransport / matchApplication
//                               base/src/main/java/vmirror/FilterConfig.java:27-94
//   Mirror.mirror level choice  base/src/main/java/vmirror/Mirror.java:104-117
//   Mirror.switchPacket         Mirror.java:73-87
//   Mirror.checkHelper          Mirror.java:133-139 (set of MirrorConfig)
//
// __host__ __device__ so the test harness runs this exact code on the host.
#pragma once

#include "../common/netmatch.h"
#include "acl_dev.h"
#include "dev_common.h"
#include "packet_dev.h"

namespace vcd {

enum : int { kLvlEther = 0, kLvlIp = 1, kLvlTransport = 2, kLvlApp = 3 };

struct MirrorItem {
    uint64_t mac_src, mac_dst;
    vcn::Addr ip_src, ip_dst;       // len 0 = null
    bool low_src, low_dst;          // lowBitsV6V4 of 16-byte addresses
    int32_t transport, app;         // -1 = null
    int32_t port_src, port_dst;
};

VC_HD bool mf_contains(const MirrorNet& n, const vcn::Addr& a, bool low) {
    return vcn::net_match(*reinterpret_cast<const vcn::NetMatch*>(&n), a, low);
}

VC_HD bool mf_ether(const MirrorRec& f, uint64_t src, uint64_t dst) {           // :27-38
    const bool x = f.flags & VC_MF_MAC_X, y = f.flags & VC_MF_MAC_Y;
    if (x && y) return (f.mac_x == src && f.mac_y == dst) || (f.mac_y == src && f.mac_x == dst);
    if (x) return f.mac_x == src || f.mac_x == dst;
    return true;
}

VC_HD bool mf_ip(const MirrorRec& f, const MirrorItem& it) {                     // :40-55
    if (!mf_ether(f, it.mac_src, it.mac_dst)) return false;
    const bool x = f.flags & VC_MF_NET_X, y = f.flags & VC_MF_NET_Y;
    if (!x && !y) return true;
    const bool xs = x && mf_contains(f.net_x, it.ip_src, it.low_src);
    const bool xd = x && mf_contains(f.net_x, it.ip_dst, it.low_dst);
    if (x && y) {
        const bool ys = mf_contains(f.net_y, it.ip_src, it.low_src);
        const bool yd = mf_contains(f.net_y, it.ip_dst, it.low_dst);
        return (xs && yd) || (ys && xd);
    }
    if (x) return xs || xd;
    return true;                    // netY without netX: the Java else branch
}

VC_HD bool in_range(int32_t lo, int32_t hi, int32_t p) { return lo <= p && p <= hi; }

VC_HD bool mf_transport(const MirrorRec& f, const MirrorItem& it) {              // :57-80
    if (!mf_ip(f, it)) return false;
    if (f.transport != -1 && f.transport != it.transport) return false;
    const bool x = f.flags & VC_MF_PORT_X, y = f.flags & VC_MF_PORT_Y;
    if (x && y)
        return (in_range(f.port_x0, f.port_x1, it.port_src) &&
                in_range(f.port_y0, f.port_y1, it.port_dst)) ||
               (in_range(f.port_y0, f.port_y1, it.port_src) &&
                in_range(f.port_x0, f.port_x1, it.port_dst));
    if (x) return in_range(f.port_x0, f.port_x1, it.port_src) ||
                  in_range(f.port_x0, f.port_x1, it.port_dst);
    return true;
}

VC_HD bool mf_app(const MirrorRec& f, const MirrorItem& it) {                    // :82-94
    if (!mf_transport(f, it)) return false;
    return f.app == -1 || f.app == it.app;
}

// Mirror.mirror: the level its null checks pick (Mirror.java:105-117)
VC_HD int mirror_level(const MirrorItem& it) {
    if (it.ip_src.len == 0 || it.ip_dst.len == 0) return kLvlEther;
    if (it.transport == -1) return kLvlIp;
    if (it.app == -1) return kLvlTransport;
    return kLvlApp;
}

// Filter k through the scalar cache: the loop index is wave-uniform, so
// reading the record through a constant-address-space pointer puts its
// fields in SGPRs and every branch on them is a scalar branch.
VC_HD MirrorRec load_filter(const MirrorImage& img, int k) {
#if defined(__HIP_DEVICE_COMPILE__)
    typedef const __attribute__((address_space(4))) MirrorRec* CRec;
    return ((CRec)(img.f))[k];
#else
    return img.f[k];
#endif
}

// checkHelper: union of the mirrors of the matching filters of `origin`.
VC_HD uint64_t mirror_eval(const MirrorImage& img, int32_t origin, const MirrorItem& it, int lvl) {
    uint64_t m = 0;
    for (int k = 0; k < img.n; ++k) {
        const MirrorRec f = load_filter(img, k);
        if (f.origin != origin) continue;
        bool hit;
        if (lvl == kLvlEther) hit = mf_ether(f, it.mac_src, it.mac_dst);
        else if (lvl == kLvlIp) hit = mf_ip(f, it);
        else if (lvl == kLvlTransport) hit = mf_transport(f, it);
        else hit = mf_app(f, it);
        if (hit) m |= uint64_t(1) << f.mirror;
    }
    return m;
}

VC_HD uint64_t mac48(const uint8_t* p) {
    uint64_t v = 0;
    for (int k = 0; k < 6; ++k) v |= uint64_t(p[k]) << (8 * k);
    return v;
}

// MAC i of a 6-byte-per-item column: three 16-bit loads (6 * i is even;
// the column is at least 2-byte aligned, vc_mirror_match_dev checks)
VC_HD uint64_t mac48_col(const uint8_t* col, int64_t i) {
    const uint16_t* h = reinterpret_cast<const uint16_t*>(col) + 3 * i;
    return uint64_t(h[0]) | (uint64_t(h[1]) << 16) | (uint64_t(h[2]) << 32);
}

VC_HD vcn::Addr item_addr(const uint8_t* base, int64_t i, int len) {
    if (!base || (len != 4 && len != 16)) return vcn::Addr{{0, 0, 0, 0}, 0};
    const uint4 w = reinterpret_cast<const uint4*>(base)[i];       // 16-byte aligned rows
    return len == 16 ? vcn::Addr{{w.x, w.y, w.z, w.w}, 16} : vcn::Addr{{w.x, 0, 0, 0}, 4};
}

// Item i of a vc_mirror_items batch; absent columns take MirrorData's
// defaults (MirrorData.java:16-17: 00:00:00:00:00:00 -> ff:ff:ff:ff:ff:ff)
// or null.  A length other than 4 / 16 reads as a null IP.
VC_HD MirrorItem mirror_item(const vc_mirror_items& in, int64_t i) {
    MirrorItem it;
    it.mac_src = in.mac_src ? mac48_col(in.mac_src, i) : 0;
    it.mac_dst = in.mac_dst ? mac48_col(in.mac_dst, i) : 0xFFFFFFFFFFFFull;
    it.ip_src = item_addr(in.ip_src, i, in.ip_src_len ? in.ip_src_len[i] : 0);
    it.ip_dst = item_addr(in.ip_dst, i, in.ip_dst_len ? in.ip_dst_len[i] : 0);
    it.transport = in.transport ? in.transport[i] : -1;
    it.app = in.app ? in.app[i] : -1;
    it.port_src = in.port_src ? in.port_src[i] : 0;
    it.port_dst = in.port_dst ? in.port_dst[i] : 0;
    it.low_src = vcn::low_bits_v6v4(it.ip_src);
    it.low_dst = vcn::low_bits_v6v4(it.ip_dst);
    return it;
}

// Mirror.switchPacket: frame -> EthernetPacket (dst MAC bytes 0-5, src
// 6-11, EthernetPacket.java:19-20) -> matchIp for IPv4/IPv6 packets,
// matchEthernet otherwise; 0 for a frame the parse rejects.
VC_HD uint64_t mirror_switch_one(const MirrorImage& img, int32_t origin, const uint8_t* p,
                                 int len, int layer) {
    PktOut o;
    parse_packet(p, len, layer, &o);
    if (o.status != VC_PKT_OK) return 0;
    const uint8_t* eth = layer == VC_LAYER_VXLAN ? p + 8 : p;
    MirrorItem it{};
    it.mac_dst = mac48(eth);
    it.mac_src = mac48(eth + 6);
    int lvl = kLvlEther;
    if (o.l3 == VC_L3_IPV4 || o.l3 == VC_L3_IPV6) {
        const bool v6 = o.l3 == VC_L3_IPV6;
        const uint4 s = *reinterpret_cast<const uint4*>(o.src);   // PktOut: 16-byte aligned
        const uint4 d = *reinterpret_cast<const uint4*>(o.dst);
        it.ip_src = v6 ? vcn::Addr{{s.x, s.y, s.z, s.w}, 16} : vcn::Addr{{s.x, 0, 0, 0}, 4};
        it.ip_dst = v6 ? vcn::Addr{{d.x, d.y, d.z, d.w}, 16} : vcn::Addr{{d.x, 0, 0, 0}, 4};
        it.low_src = vcn::low_bits_v6v4(it.ip_src);
        it.low_dst = vcn::low_bits_v6v4(it.ip_dst);
        lvl = kLvlIp;
    }
    return mirror_eval(img, origin, it, lvl);
}

// A uniform record through the scalar cache (as load_filter).
template <class T>
VC_HD T load_uniform(const T* p, int k) {
#if defined(__HIP_DEVICE_COMPILE__)
    typedef const __attribute__((address_space(4))) T* CP;
    return ((CP)(p))[k];
#else
    return p[k];
#endif
}

// The (xmask, ymask) pair of interval j (kL: the table is staged in LDS)
template <bool kL = false>
VC_HD ulonglong2 sw_masks(const uint64_t* p, int j) {
    return tbl_ld<kL>(reinterpret_cast<const ulonglong2*>(p) + j);
}

// The intervals of two keys (an item's source and destination) in one
// loop: the trip count depends on nb only, so the two LDS reads of a step go
// out together (the C2 ACL kernel's lockstep form, classify.hip acl_v4_four)
template <bool kL, class T>
VC_HD void bsearch2(const T* b, int nb, T k0, T k1, int* j0, int* j1) {
    int lo0 = 0, lo1 = 0, len = nb;
    while (len > 1) {
        const int half = len >> 1;
        const T x0 = tbl_ld<kL>(b + lo0 + half), x1 = tbl_ld<kL>(b + lo1 + half);
        lo0 = x0 <= k0 ? lo0 + half : lo0;
        lo1 = x1 <= k1 ? lo1 + half : lo1;
        len -= half;
    }
    *j0 = lo0;
    *j1 = lo1;
}

template <bool kL>
VC_HD void bsearch2_u128(const uint64_t* b, int nb, uint64_t h0, uint64_t l0, uint64_t h1,
                         uint64_t l1, int* j0, int* j1) {
    int lo0 = 0, lo1 = 0, len = nb;
    while (len > 1) {
        const int half = len >> 1;
        const ulonglong2 x0 = tbl_ld<kL>(reinterpret_cast<const ulonglong2*>(b) + lo0 + half);
        const ulonglong2 x1 = tbl_ld<kL>(reinterpret_cast<const ulonglong2*>(b) + lo1 + half);
        lo0 = le128(x0.x, x0.y, h0, l0) ? lo0 + half : lo0;
        lo1 = le128(x1.x, x1.y, h1, l1) ? lo1 + half : lo1;
        len -= half;
    }
    *j0 = lo0;
    *j1 = lo1;
}

// Mirror.switchPacket through the origin's bit-set image (images.h
// MirrorSwImage): the same answer as mirror_switch_one over the origin's
// filters.  matchEthernet (FilterConfig.java:27-38) for every MAC filter,
// then for an IPv4 / IPv6 packet matchIp's network part (:40-55) for all
// filters at once from the interval masks of the two addresses:
//   no netX -> true; netX and netY -> (xs && yd) || (ys && xd); netX only
//   -> xs || xd.
// The interval tables are read from the image, or from the kernel's LDS
// copy of them (kL: t carries the LDS pointers).
struct SwTables {
    const uint32_t* b4;
    const uint64_t *p4, *b6, *p6;
    const uint32_t* bp;            // port intervals (Mirror.mirror's items)
    const uint64_t* pp;
    const uint64_t* bm;            // the origin's MACs (Mirror.mirror's items)
    const uint64_t* pm;
};

VC_HD SwTables sw_tables(const MirrorSwImage& s) {
    return SwTables{s.b4, s.p4, s.b6, s.p6, s.bp, s.pp, s.bm, s.pm};
}

// (macX of, macY of) for a MAC at entry j of the origin's MAC list, or 0s
// when the entry is not that MAC
template <bool kL = false>
VC_HD ulonglong2 sw_mac_at(const SwTables& t, int j, uint64_t mac) {
    if (tbl_ld<kL>(t.bm + j) != mac) return make_ulonglong2(0, 0);
    return sw_masks<kL>(t.pm, j);
}

template <bool kL = false>
VC_HD uint64_t mirror_switch_sw(const MirrorSwImage& s, const SwTables& t, const uint8_t* p,
                                int len, int layer) {
    PktOut o;
    parse_packet(p, len, layer, &o);
    if (o.status != VC_PKT_OK) return 0;
    const uint8_t* eth = layer == VC_LAYER_VXLAN ? p + 8 : p;
    const uint64_t dst = mac48(eth), src = mac48(eth + 6);
    uint64_t hit = s.all & ~s.mac;
    for (int k = 0; k < s.n_mac; ++k) {
        const MirrorSwMac f = load_uniform(s.macs, k);
        const bool ok = f.has_y ? (f.mac_x == src && f.mac_y == dst) || (f.mac_y == src && f.mac_x == dst)
                                : f.mac_x == src || f.mac_x == dst;
        if (ok) hit |= f.bit;
    }
    if (o.l3 == VC_L3_IPV4 || o.l3 == VC_L3_IPV6) {
        ulonglong2 ms, md;
        if (o.l3 == VC_L3_IPV4) {
            int js, jd;
            bsearch2<kL>(t.b4, s.nb4, bswap32(o.src[0]), bswap32(o.dst[0]), &js, &jd);
            ms = sw_masks<kL>(t.p4, js);
            md = sw_masks<kL>(t.p4, jd);
        } else {
            uint64_t sh, sl, dh, dl;
            v6_key(*reinterpret_cast<const uint4*>(o.src), &sh, &sl);
            v6_key(*reinterpret_cast<const uint4*>(o.dst), &dh, &dl);
            int js, jd;
            bsearch2_u128<kL>(t.b6, s.nb6, sh, sl, dh, dl, &js, &jd);
            ms = sw_masks<kL>(t.p6, js);
            md = sw_masks<kL>(t.p6, jd);
        }
        const uint64_t both = s.has_x & s.has_y, xonly = s.has_x & ~s.has_y;
        hit &= ~s.has_x | (both & ((ms.x & md.y) | (ms.y & md.x))) | (xonly & (ms.x | md.x));
    }
    uint64_t m = 0;
    for (int k = 0; k < s.n_mir; ++k) {
        const MirrorSwMir r = load_uniform(s.mirs, k);
        if (hit & r.filters) m |= uint64_t(1) << r.bit;
    }
    return m;
}

// The (xmask, ymask) of one address of a MirrorData item (4 or 16 bytes)
template <bool kL = false>
VC_HD ulonglong2 sw_addr_masks(const MirrorSwImage& s, const SwTables& t, const vcn::Addr& a) {
    if (a.len == 4) return sw_masks<kL>(t.p4, bsearch_u32<kL>(t.b4, s.nb4, bswap32(a.w[0])));
    uint64_t h, l;
    v6_key(make_uint4(a.w[0], a.w[1], a.w[2], a.w[3]), &h, &l);
    return sw_masks<kL>(t.p6, bsearch_u128<kL>(t.b6, s.nb6, h, l));
}

// Filters of a uniform id list whose id is `id`, plus `any`
VC_HD uint64_t sw_ids(const MirrorSwId* ids, int n, uint64_t any, int32_t id) {
    for (int k = 0; k < n; ++k) {
        const MirrorSwId r = load_uniform(ids, k);
        if (r.id == id) any |= r.filters;
    }
    return any;
}

// Mirror.mirror's filter step for one MirrorData item through the origin's
// bit-set image: mirror_eval's answer at the item's level (Mirror.java
// :104-117), with matchTransport's protocol and port part (:57-80) and
// matchApplication's protocol (:82-94) as sets too:
//   transport -1 or equal; no portX -> true; portX and portY ->
//   (pxs && pyd) || (pys && pxd); portX only -> pxs || pxd.
template <bool kL = false>
VC_HD uint64_t mirror_match_sw(const MirrorSwImage& s, const SwTables& t, const MirrorItem& it,
                               int lvl) {
    // matchEthernet: the two MACs looked up in the origin's MAC list;
    // macX and macY -> (xs && yd) || (ys && xd); macX only -> xs || xd
    uint64_t hit = s.all & ~s.mac;
    if (s.nbm) {
        int js, jd;
        bsearch2<kL>(t.bm, s.nbm, it.mac_src, it.mac_dst, &js, &jd);
        const ulonglong2 ms = sw_mac_at<kL>(t, js, it.mac_src);
        const ulonglong2 md = sw_mac_at<kL>(t, jd, it.mac_dst);
        hit |= (s.mac_both & ((ms.x & md.y) | (ms.y & md.x))) | (s.mac_xonly & (ms.x | md.x));
    }
    if (lvl >= kLvlIp) {
        ulonglong2 ms, md;
        if (it.ip_src.len == 4 && it.ip_dst.len == 4) {
            int js, jd;
            bsearch2<kL>(t.b4, s.nb4, bswap32(it.ip_src.w[0]), bswap32(it.ip_dst.w[0]), &js, &jd);
            ms = sw_masks<kL>(t.p4, js);
            md = sw_masks<kL>(t.p4, jd);
        } else {
            ms = sw_addr_masks<kL>(s, t, it.ip_src);
            md = sw_addr_masks<kL>(s, t, it.ip_dst);
        }
        const uint64_t both = s.has_x & s.has_y, xonly = s.has_x & ~s.has_y;
        hit &= ~s.has_x | (both & ((ms.x & md.y) | (ms.y & md.x))) | (xonly & (ms.x | md.x));
    }
    if (lvl >= kLvlTransport) {
        const uint64_t tm = sw_ids(s.tids, s.n_t, s.any_t, it.transport);
        int js, jd;
        bsearch2<kL>(t.bp, s.nbp, uint32_t(it.port_src) ^ 0x80000000u,
                     uint32_t(it.port_dst) ^ 0x80000000u, &js, &jd);
        const ulonglong2 ps = sw_masks<kL>(t.pp, js);
        const ulonglong2 pd = sw_masks<kL>(t.pp, jd);
        const uint64_t both = s.has_px & s.has_py, xonly = s.has_px & ~s.has_py;
        hit &= tm & (~s.has_px | (both & ((ps.x & pd.y) | (ps.y & pd.x))) | (xonly & (ps.x | pd.x)));
    }
    if (lvl == kLvlApp) hit &= sw_ids(s.aids, s.n_a, s.any_a, it.app);
    uint64_t m = 0;
    for (int k = 0; k < s.n_mir; ++k) {
        const MirrorSwMir r = load_uniform(s.mirs, k);
        if (hit & r.filters) m |= uint64_t(1) << r.bit;
    }
    return m;
}

}  // namespace vcd

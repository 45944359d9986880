// imgcheck.hip -- TEST HARNESS ONLY (not part of libvclassify).
//
// Builds the same table images as the product compiler and walks them on the
// host with the kernels' own __host__ __device__ probe functions, so compile
// bugs show up in the CPU test tier before any GPU run.  The product library
// never contains or calls this code.
#include <cstring>
#include <vector>

#include "../../vproxy_amd/csrc/compile/compile.hpp"
#include "../../vproxy_amd/csrc/device/acl_dev.h"
#include "../../vproxy_amd/csrc/device/hint_dev.h"
#include "../../vproxy_amd/csrc/device/mirror_dev.h"
#include "../../vproxy_amd/csrc/device/packet_dev.h"
#include "../../vproxy_amd/csrc/device/route_dev.h"

using namespace vcd;

namespace {
AclFamilyImage fam_img(const vc::AclFamilyBuilt& b) {
    AclFamilyImage f{};
    f.bounds4 = b.bounds4.data();
    f.bounds6 = b.bounds6.data();
    f.rec = b.rec.data();
    f.pieces = b.pieces.data();
    f.dir4 = b.dir4.empty() ? nullptr : b.dir4.data();
    f.dir_bits = b.dir_bits;
    f.nb = b.nb;
    f.np = int32_t(b.pieces.size() / 2);
    f.v4_only = b.v4_only;
    return f;
}

HintImage hint_img(const vc::HintBuilt& b) {
    HintImage h{};
    h.blob = b.blob.data();
    h.host_recs = b.host.recs.data();
    h.host_ext = b.host.ext.data();
    h.host_tags = b.host.tags.data();
    h.uri_slots = reinterpret_cast<const KeySlot*>(b.uri_slots.data());
    h.uri_tags = b.uri_tags.data();
    h.lists = b.lists.data();
    h.port_mins = reinterpret_cast<const PortMin*>(b.port_mins.data());
    h.groups = reinterpret_cast<const GroupRec*>(b.groups.data());
    h.host_mask = uint32_t(b.host.tags.size() - 1);
    h.uri_mask = uint32_t(b.uri_slots.size() - 1);
    h.n_groups = b.n_groups;
    h.wildcard_slot = b.wildcard_slot;
    h.uri_star_slot = b.uri_star_slot;
    h.has_uri_keys = b.has_uri_keys;
    h.uri_len_lo = uint32_t(b.uri_len_mask);
    h.uri_len_hi = uint32_t(b.uri_len_mask >> 32);
    if (b.wildcard_slot >= 0) {
        const auto& w = b.host.recs[size_t(b.wildcard_slot)];
        h.wild_len_pm = w.len_pm;
        h.wild_a = w.a;
        h.wild_b = w.b;
    }
    return h;
}
// A name copied into a buffer with a 16-byte apron of junk either side, the
// way the kernels stage a wave's names in LDS, read through LdsSrc.
struct Staged {
    std::vector<uint32_t> words;
    LdsSrc src;
    Staged(const uint8_t* p, int n, int align) {
        words.assign(size_t(n + 48) / 4 + 2, 0xA5A5A5A5u);
        uint8_t* b = reinterpret_cast<uint8_t*>(words.data());
        std::memcpy(b + 16 + align, p, size_t(n));
        src = LdsSrc{words.data(), 16 + align};
    }
};
}  // namespace

extern "C" {

int ic_acl(const vc_acl_rule* tcp, int nt, const vc_acl_rule* udp, int nu, int dflt, int family,
           const uint8_t* proto, const void* src, const uint16_t* port, int64_t n, int32_t* out,
           uint8_t* allow, int32_t* stats) {
    vc::AclBuilt b;
    int rc = vc::build_acl(tcp, nt, udp, nu, dflt, &b);
    if (rc) return rc;
    for (int l = 0; l < 2; ++l)
        for (int f = 0; f < 2; ++f) {
            stats[(l * 2 + f) * 2] = b.fam[l][f].nb;
            stats[(l * 2 + f) * 2 + 1] = int32_t(b.fam[l][f].pieces.size() / 2);
        }
    for (int64_t i = 0; i < n; ++i) {
        const int l = proto[i] == VC_PROTO_TCP ? 0 : 1;
        AclFamilyImage f = fam_img(b.fam[l][family == 4 ? 0 : 1]);
        int j;
        if (family == 4) {
            // through the bucket directory (when built), checked against the
            // whole binary search
            const uint32_t key = static_cast<const uint32_t*>(src)[i];
            j = acl4_interval(f, key);
            if (j != bsearch_u32(f.bounds4, f.nb, key)) return -100;
        } else {
            uint64_t hi, lo;
            v6_key(static_cast<const uint4*>(src)[i], &hi, &lo);
            j = bsearch_u128(f.bounds6, f.nb, hi, lo);
            // a list of plain IPv4 rules: the kernels' shortcut through the
            // v4 image must give the 128-bit search's answer
            if (f.v4_only &&
                acl6_global(f, fam_img(b.fam[l][0]), hi, lo, port[i]) !=
                    acl_value(f.rec, f.pieces, j, port[i]))
                return -102;
            stats[8 + l] += f.v4_only;
        }
        // the interval's packed record, checked against (x, y) + pieces
        uint32_t v = acl_value(f.rec, f.pieces, j, port[i]);
        const uint2 d = make_uint2(b.fam[l][family == 4 ? 0 : 1].desc[2 * j],
                                   b.fam[l][family == 4 ? 0 : 1].desc[2 * j + 1]);
        if (v != port_lookup(f.pieces, d, port[i])) return -101;
        out[i] = out_index(v);
        allow[i] = v == VC_NONE ? uint8_t(b.default_allow) : b.allow[(l ? b.n_tcp : 0) + v];
    }
    return 0;
}

int ic_route(const vc_net* rules, int nr, int family, const void* keys, int64_t n, int32_t* out,
             int32_t* stats, int root_bits) {
    vc::TrieBuilt t;
    int rc = vc::build_trie(rules, nr, family == 4 ? 0 : 1, &t, root_bits);
    if (rc) return rc;
    stats[0] = t.root_bits;
    stats[1] = t.n_nodes;
    stats[2] = t.n_records;
    // the IPv6 wide root as wide_root_kernel builds it (route_dev.h
    // wide_entry per slot): every key must get the same answer through it
    std::vector<uint32_t> wide;
    if (family == 6) {
        wide.resize((size_t(1) << t.root_bits) * 4);
        for (uint32_t s = 0; s < (1u << t.root_bits); ++s) wide_entry(t.nodes.data(), s, &wide[4 * s]);
    }
    int64_t one_slot = 0;
    for (int64_t i = 0; i < n; ++i) {
        uint32_t e;
        if (family == 4) {
            e = trie_v4(t.nodes.data(), t.root_bits, static_cast<const uint32_t*>(keys)[i]);
        } else {
            uint64_t hi, lo;
            v6_key(static_cast<const uint4*>(keys)[i], &hi, &lo);
            e = trie_v6(t.nodes.data(), t.root_bits, hi, lo);
            if (trie_v6w(t.nodes.data(), wide.data(), t.root_bits, hi, lo) != e) return -201;
            one_slot += wide[4 * (hi >> (64 - t.root_bits)) + 3] != 0;
        }
        out[i] = out_index(e);
    }
    stats[3] = int32_t(one_slot);            // keys the wide root answers in one load
    return 0;
}

// names the deferring fast path left to the follow-up kernel in the last
// ic_hint call
static int64_t g_hint_deferred = 0;
int64_t ic_hint_deferred() { return g_hint_deferred; }

int ic_hint(const vc_group_annos* g, int ng, const uint8_t* hb, const uint32_t* ho,
            const uint8_t* hn, const uint16_t* port, const uint8_t* ub, const uint32_t* uo,
            const uint8_t* un, int64_t n, int32_t* out) {
    vc::HintBuilt b;
    int rc = vc::build_hints(g, ng, &b);
    if (rc) return rc;
    HintImage img = hint_img(b);
    g_hint_deferred = 0;
    for (int64_t i = 0; i < n; ++i) {
        DStr h{nullptr, -1}, u{nullptr, -1};
        if (hb && !(hn && hn[i])) h = DStr{hb + ho[i], int(ho[i + 1] - ho[i])};
        if (ub && !(un && un[i])) u = DStr{ub + uo[i], int(uo[i + 1] - uo[i])};
        const int p = port ? port[i] : 0;
        // reference form: formatHost then the general / sequential search
        const int32_t want = (u.n >= 0 && img.has_uri_keys)
                                 ? hint_general(img, format_host(h), p, format_uri(u))
                                 : hint_host_only(img, format_host(h), p);
        out[i] = want;
        if (u.n >= 0 && img.has_uri_keys) {
            // the uri-aware deferring form (hint_kernel<.., .., true>): a
            // port-0 hint with a host takes the host fast path and gets the
            // same result there, or kDeferred for the general search
            // the follow-up kernel's level-ordered form for port 0
            if (p == 0 && hint_port0_uri(img, h, u.p, u.n) != want) return -106;
            if (p != 0 || h.n < 0) { ++g_hint_deferred; continue; }
            for (int al = 0; al < 4; ++al) {
                Staged st(h.p, h.n, al);
                int32_t d = host_only_fast<true>(img, &img, st.src, h.n, 0, true);
                if (is_uri_slot_code(d)) d = uri_in_slot(img, -2 - d, u.p, u.n);
                if (d != want && d != kDeferred) return -105;
                if (al == 0 && d == kDeferred) ++g_hint_deferred;
            }
            continue;
        }
        if (h.n < 0) { if (want != -1) return -100; continue; }
        // the kernels' fused fast path, from a plain pointer and from a
        // staged copy at every word alignment: all must agree
        if (host_only_fast(img, &img, PtrSrc{h.p}, h.n, p) != want) return -101;
        for (int al = 0; al < 4; ++al) {
            Staged st(h.p, h.n, al);
            if (host_only_fast(img, &img, st.src, h.n, p) != want) return -102;
            // the deferring form (the pool pass's kernel): the same result,
            // or kDeferred for the follow-up kernel
            const int32_t d = host_only_fast<true>(img, &img, st.src, h.n, p);
            if (d != want && d != kDeferred) return -104;
            if (al == 0 && d == kDeferred) ++g_hint_deferred;
        }
    }
    return 0;
}

int ic_dns(const char* const* keys, const int32_t* key_lens, const int32_t* values, int nk,
           const vc_group_annos* g, int ng, const uint8_t* qb, const uint32_t* qo, int64_t n,
           uint8_t* kind, int32_t* value) {
    vc::HostsBuilt hb;
    vc::HintBuilt b;
    int rc = vc::build_hosts(keys, key_lens, values, nk, &hb);
    if (rc == 0) rc = vc::build_hints(g, ng, &b);
    if (rc) return rc;
    HintImage img = hint_img(b);
    HostsImage hosts{hb.blob.data(), hb.table.recs.data(), hb.table.tags.data(),
                     uint32_t(hb.table.tags.size() - 1), hb.n};
    for (int64_t i = 0; i < n; ++i) {
        const uint8_t* q = qb + qo[i];
        const int qn = int(qo[i + 1] - qo[i]);
        dns_one(hosts, img, &img, PtrSrc{q}, qn, kind + i, value + i);
        for (int al = 0; al < 4; ++al) {
            Staged st(q, qn, al);
            uint8_t k2;
            int32_t v2;
            dns_one(hosts, img, &img, st.src, qn, &k2, &v2);
            if (k2 != kind[i] || v2 != value[i]) return -103;
            // the deferring form (dns_kernel / dnsd_kernel): the same
            // classification, or kDnsDeferred for the follow-up kernel
            dns_one<true>(hosts, img, &img, st.src, qn, &k2, &v2);
            if (k2 != kDnsDeferred && (k2 != kind[i] || v2 != value[i])) return -105;
        }
    }
    return 0;
}

// the kernels' parse_packet on the host: 8 ints + 32 address bytes per frame
int ic_packets(const uint8_t* blob, const uint32_t* off, int64_t n, int layer, int32_t* fields,
               uint8_t* addrs) {
    for (int64_t i = 0; i < n; ++i) {
        PktOut o;
        parse_packet(blob + off[i], int(off[i + 1] - off[i]), layer, &o);
        int32_t* f = fields + 8 * i;
        f[0] = o.status; f[1] = o.l3; f[2] = o.l4; f[3] = o.proto;
        f[4] = int32_t(o.vni); f[5] = o.ether_type; f[6] = o.sport; f[7] = o.dport;
        std::memcpy(addrs + 32 * i, o.src, 16);
        std::memcpy(addrs + 32 * i + 16, o.dst, 16);
    }
    return 0;
}

// SSLContextHolder.choose through the compiled certificate table, from a
// plain pointer and from a staged copy at every word alignment.
int ic_certs(const char* const* names, const int32_t* lens, const int32_t* holder, int nn,
             int nh, const uint8_t* qb, const uint32_t* qo, const uint8_t* qnull, int64_t n,
             int32_t* out) {
    vc::HostsBuilt b;
    int rc = vc::build_certs(names, lens, holder, nn, nh, &b);
    if (rc) return rc;
    CertImage c{};
    c.names = HostsImage{b.blob.data(), b.table.recs.data(), b.table.tags.data(),
                         uint32_t(b.table.tags.size() - 1), b.n};
    c.n_holders = nh;
    for (int64_t i = 0; i < n; ++i) {
        const uint8_t* q = qb + qo[i];
        const int qn = int(qo[i + 1] - qo[i]);
        const bool nul = qnull && qnull[i];
        out[i] = cert_one(c, PtrSrc{q}, qn, nul);
        for (int al = 0; al < 4; ++al) {
            Staged st(q, qn, al);
            if (cert_one(c, st.src, qn, nul) != out[i]) return -104;
        }
    }
    return 0;
}

// The UDP list's IPv4 image at a fixed port (compile.cpp build_acl_port,
// the switch kernel's LDS table): for every key, the rule the general image
// gives at that port.  Keys: the given ones plus every interval start of the
// general image and the key below it.  Returns the port table's size.
int ic_acl_port(const vc_acl_rule* udp, int nu, uint32_t port, const uint32_t* keys, int64_t n,
                int32_t* out) {
    vc::AclBuilt b;
    int rc = vc::build_acl(nullptr, 0, udp, nu, 0, &b);
    if (rc) return rc;
    std::vector<uint32_t> pb, pv;
    vc::build_acl_port(b.fam[1][0], port, &pb, &pv);
    const AclFamilyImage f = fam_img(b.fam[1][0]);
    auto check = [&](uint32_t key) {
        const uint32_t g = acl_value(f.rec, f.pieces, acl4_interval(f, key), port);
        const uint32_t v = pv[size_t(bsearch_u32(pb.data(), int(pb.size()), key))];
        return g == v ? int32_t(g == VC_NONE ? -1 : int32_t(g)) : -1000;
    };
    for (int32_t j = 0; j < f.nb; ++j) {
        if (check(f.bounds4[j]) == -1000) return -300;
        if (f.bounds4[j] && check(f.bounds4[j] - 1) == -1000) return -301;
    }
    for (int64_t i = 0; i < n; ++i) {
        out[i] = check(keys[i]);
        if (out[i] == -1000) return -302;
    }
    return int(pb.size());
}

// Mirror filters: the kernels' item loading + mirror_eval, and switchPacket.
int ic_mirror(const vc_mirror_filter* f, int nf, int32_t origin, const vc_mirror_items* items,
              int64_t n, uint64_t* out) {
    std::vector<MirrorRec> recs;
    int rc = vc::build_mirror(f, nf, &recs);
    if (rc) return rc;
    const MirrorImage img{recs.data(), nf};
    for (int64_t i = 0; i < n; ++i) {
        const MirrorItem it = mirror_item(*items, i);
        out[i] = mirror_eval(img, origin, it, mirror_level(it));
    }
    return 0;
}

int ic_mirror_switch(const vc_mirror_filter* f, int nf, int32_t origin, const uint8_t* blob,
                     const uint32_t* off, int64_t n, int layer, uint64_t* out) {
    std::vector<MirrorRec> recs;
    int rc = vc::build_mirror(f, nf, &recs);
    if (rc) return rc;
    const MirrorImage img{recs.data(), nf};
    for (int64_t i = 0; i < n; ++i)
        out[i] = mirror_switch_one(img, origin, blob + off[i], int(off[i + 1] - off[i]), layer);
    return 0;
}

// Mirror.mirror over MirrorData items through the origin's bit-set image
// (mirror_dev.h mirror_match_sw); returns 1, with nothing written, when the
// origin has no such image
int ic_mirror_sw(const vc_mirror_filter* f, int nf, int32_t origin, const vc_mirror_items* items,
                 int64_t n, uint64_t* out) {
    std::vector<MirrorRec> recs;
    int rc = vc::build_mirror(f, nf, &recs);
    if (rc) return rc;
    vc::MirrorSwBuilt b;
    if (!vc::build_mirror_switch(recs, origin, &b)) return 1;
    b.img.macs = b.macs.data();
    b.img.mirs = b.mirs.data();
    b.img.b4 = b.b4.data();
    b.img.p4 = b.p4.data();
    b.img.b6 = b.b6.data();
    b.img.p6 = b.p6.data();
    b.img.tids = b.tids.data();
    b.img.aids = b.aids.data();
    b.img.bp = b.bp.data();
    b.img.pp = b.pp.data();
    b.img.bm = b.bm.data();
    b.img.pm = b.pm.data();
    for (int64_t i = 0; i < n; ++i) {
        const MirrorItem it = mirror_item(*items, i);
        out[i] = mirror_match_sw(b.img, sw_tables(b.img), it, mirror_level(it));
    }
    return 0;
}

// switchPacket through the origin's bit-set image (mirror_dev.h
// mirror_switch_sw over compile.cpp build_mirror_switch); returns 1, with
// nothing written, when the origin has no such image
int ic_mirror_switch_sw(const vc_mirror_filter* f, int nf, int32_t origin, const uint8_t* blob,
                        const uint32_t* off, int64_t n, int layer, uint64_t* out, int32_t* nb) {
    std::vector<MirrorRec> recs;
    int rc = vc::build_mirror(f, nf, &recs);
    if (rc) return rc;
    vc::MirrorSwBuilt b;
    if (!vc::build_mirror_switch(recs, origin, &b)) return 1;
    b.img.macs = b.macs.data();
    b.img.mirs = b.mirs.data();
    b.img.b4 = b.b4.data();
    b.img.p4 = b.p4.data();
    b.img.b6 = b.b6.data();
    b.img.p6 = b.p6.data();
    b.img.tids = b.tids.data();
    b.img.aids = b.aids.data();
    b.img.bp = b.bp.data();
    b.img.pp = b.pp.data();
    b.img.bm = b.bm.data();
    b.img.pm = b.pm.data();
    for (int64_t i = 0; i < n; ++i)
        out[i] = mirror_switch_sw(b.img, sw_tables(b.img), blob + off[i],
                                  int(off[i + 1] - off[i]), layer);
    nb[0] = b.img.nb4;
    nb[1] = b.img.nb6;
    return 0;
}

// the mirror filters' compiled Network.contains (common/netmatch.h NetMatch)
int ic_net_match(const uint8_t* in, int inlen, const uint8_t* rule, int rlen, const uint8_t* mask,
                 int mlen) {
    const vcn::Addr a = vcn::addr_of(in, inlen);
    const vcn::NetMatch m = vcn::net_matcher(vcn::addr_of(rule, rlen), vcn::addr_of(mask, mlen));
    return vcn::net_match(m, a, vcn::low_bits_v6v4(a)) ? 1 : 0;
}

int ic_is_ipv6(const uint8_t* s, int n) { return d_is_ipv6(s, n) ? 1 : 0; }
int ic_is_ip_literal(const uint8_t* s, int n) { return d_is_ip_literal(s, n) ? 1 : 0; }

}  // extern "C"

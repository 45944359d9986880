// packet_dev.h -- header extraction from raw frames,
// the vswitch's parse chain as the Java code runs it:
//
//   VXLanPacket.from      base/src/main/java/vpacket/VXLanPacket.java:16-33
//   EthernetPacket.from   EthernetPacket.java:14-50 (IP errors kept as bytes)
//   ArpPacket.from        ArpPacket.java:22-64
//   Ipv4Packet.from       Ipv4Packet.java:28-101
//   Ipv6Packet.from       Ipv6Packet.java:24-106 (+ ExtHeader.from :248-262)
//   TcpPacket.from        TcpPacket.java:164-227 (+ TcpOption.from :399-434)
//   IcmpPacket.from       IcmpPacket.java:22-33
//
// __host__ __device__ so the test harness runs this exact code on the host.
#pragma once

#include "dev_common.h"

namespace vcd {

enum : int { kPOk = 0, kPErr = 1, kPThrow = 2, kPHang = 3 };

// Addresses are kept as the frame's raw bytes, four to a word in memory
// order (IPv4: word 0 only), so a parse moves 8 words instead of 32 bytes.
struct PktOut {
    uint32_t src[4] __attribute__((aligned(16)));
    uint32_t dst[4] __attribute__((aligned(16)));
    uint32_t vni;
    uint16_t ether_type, sport, dport;
    uint8_t status, l3, l4, proto;
};

VC_HD int pk_u8(const uint8_t* p, int i) { return p[i]; }
VC_HD int pk_u16(const uint8_t* p, int i) { return (int(p[i]) << 8) | p[i + 1]; }
// four bytes at p + i in memory order: one unaligned dword read (LDS or
// global) that stays inside the frame.  Two aligned reads and a byte align
// cut the parse's VALU by a quarter but ran slower (packet 1.32 -> 1.35 ms).
VC_HD uint32_t pk_raw32(const uint8_t* p, int i) {
    uint32_t v;
    __builtin_memcpy(&v, p + i, 4);
    return v;
}

// TcpPacket.from: an option of length 0 or 1 makes TcpOption.from read
// outside its own sub-array (ByteArray.get bounds check) -> throws.
VC_HD int pk_tcp(const uint8_t* p, int len, PktOut* o) {
    if (len < 20) return kPErr;
    o->sport = uint16_t(pk_u16(p, 0));
    o->dport = uint16_t(pk_u16(p, 2));
    const int doff = ((pk_u16(p, 12) >> 12) & 0xf) * 4;
    if (doff > len) return kPErr;
    for (int off = 20; off < doff;) {
        const int kind = int(int8_t(p[off]));
        if (kind == VC_TCPOPT_END || kind == VC_TCPOPT_NOP) {    // CASE_1_OPTION_KINDS
            off += 1;
            if (kind == VC_TCPOPT_END) break;
            continue;
        }
        if (off + 1 >= doff) return kPErr;
        const int olen = pk_u8(p, off + 1);
        if (off + olen > doff) return kPErr;
        if (olen < 2) return kPThrow;
        if (kind == VC_TCPOPT_WS && olen != 3) return kPErr;
        if (kind == VC_TCPOPT_MSS && olen != 4) return kPErr;
        off += olen;
    }
    return kPOk;
}

VC_HD int pk_l4(const uint8_t* p, int len, int proto, bool v6, PktOut* o) {
    if (proto == 1 || (v6 && proto == 58)) {                   // IcmpPacket
        o->l4 = uint8_t(proto == 58 ? 58 : 1);
        return len < 8 ? kPErr : kPOk;
    }
    if (proto == 6) {
        o->l4 = 6;
        return pk_tcp(p, len, o);
    }
    o->l4 = 0;                                                  // PacketBytes
    return kPOk;
}

VC_HD int pk_ipv4(const uint8_t* p, int len, PktOut* o) {
    if (len < 20) return kPErr;
    if (((pk_u8(p, 0) >> 4) & 0xff) != 4) return kPErr;
    const int ihl = pk_u8(p, 0) & 0x0f;
    if (len < ihl * 4) return kPErr;
    if (ihl < 5) return kPErr;
    const int total = pk_u16(p, 2);
    if (total < ihl * 4) return kPErr;
    if (total != len) return kPErr;
    o->proto = uint8_t(pk_u8(p, 9));
    o->src[0] = pk_raw32(p, 12);
    o->dst[0] = pk_raw32(p, 16);
    return pk_l4(p + ihl * 4, total - ihl * 4, o->proto, false, o);
}

VC_HD bool pk_v6_ext(int nh) {                                 // Consts.IPv6_needs_next_header
    return nh == 0 || nh == 60 || nh == 43 || nh == 44 || nh == 51 || nh == 50 || nh == 135 ||
           nh == 139 || nh == 140 || nh == 253 || nh == 254;
}

// The extension-header loop re-parses the first header (xhBuf =
// xhBuf.sub(0, len), Ipv6Packet.java:77): when that header's next header is
// an extension header again, the Java loop never ends.
VC_HD int pk_ipv6(const uint8_t* p, int len, PktOut* o) {
    if (len < 40) return kPErr;
    if (((int(int8_t(p[0])) >> 4) & 0x0f) != 6) return kPErr;
    const int payload = pk_u16(p, 4);
    if (payload == 0) return kPErr;
    if (40 + payload != len) return kPErr;
    for (int k = 0; k < 4; ++k) {
        o->src[k] = pk_raw32(p, 8 + 4 * k);
        o->dst[k] = pk_raw32(p, 24 + 4 * k);
    }
    int proto = pk_u8(p, 6), skip = 0;
    if (pk_v6_ext(proto)) {
        const uint8_t* x = p + 40;
        const int xlen = len - 40;
        if (xlen < 8) return kPErr;
        const int hl = pk_u8(x, 1);
        if (xlen < 8 + hl) return kPErr;
        if (pk_v6_ext(pk_u8(x, 0))) return kPHang;
        skip = 8 + hl;
        proto = pk_u8(x, 0);
    }
    o->proto = uint8_t(proto);
    const int rest = len - 40 - skip;
    if (proto == 59 && rest != 0) return kPErr;                // NO_NEXT_HEADER
    return pk_l4(p + 40 + skip, rest, proto, true, o);
}

VC_HD int pk_arp(const uint8_t* p, int len) {
    if (len < 8) return kPErr;
    return len == 8 + 2 * pk_u8(p, 4) + 2 * pk_u8(p, 5) ? kPOk : kPErr;
}

VC_HD void pk_clear_ip(PktOut* o) {
    o->l4 = o->proto = 0;
    o->sport = o->dport = 0;
    for (int k = 0; k < 4; ++k) o->src[k] = o->dst[k] = 0;
}

VC_HD int pk_ether(const uint8_t* p, int len, PktOut* o) {
    if (len < 14) return kPErr;
    o->ether_type = uint16_t(pk_u16(p, 12));
    const uint8_t* d = p + 14;
    const int dl = len - 14;
    if (o->ether_type == 0x0806) {
        o->l3 = VC_L3_ARP;
        return pk_arp(d, dl);
    }
    if (o->ether_type == 0x0800 || o->ether_type == 0x86dd) {
        const bool v6 = o->ether_type == 0x86dd;
        const int r = v6 ? pk_ipv6(d, dl, o) : pk_ipv4(d, dl, o);
        if (r == kPThrow || r == kPHang) return r;
        if (r == kPErr) {                                      // logged, kept as PacketBytes
            pk_clear_ip(o);
            o->l3 = VC_L3_BAD_IP;
            return kPOk;
        }
        o->l3 = uint8_t(v6 ? VC_L3_IPV6 : VC_L3_IPV4);
        return kPOk;
    }
    o->l3 = VC_L3_OTHER;
    return kPOk;
}

VC_HD uint8_t pk_status(int r, uint8_t err_code) {
    return r == kPOk ? VC_PKT_OK : r == kPErr ? err_code : r == kPThrow ? VC_PKT_EXCEPTION
                                                                     : VC_PKT_LOOP;
}

// One frame, starting at `layer` (VC_LAYER_*).  Fields of a frame whose
// parse failed are zero, except the VXLAN vni and the ether type once read.
VC_HD void parse_packet(const uint8_t* p, int len, int layer, PktOut* o) {
    *o = PktOut{};
    if (layer == VC_LAYER_VXLAN) {
        if (len < 8) {
            o->status = VC_PKT_ERR_VXLAN;
            return;
        }
        o->vni = (uint32_t(p[4]) << 16) | (uint32_t(p[5]) << 8) | p[6];
        o->status = pk_status(pk_ether(p + 8, len - 8, o), VC_PKT_ERR_ETHER);
    } else if (layer == VC_LAYER_ETHER) {
        o->status = pk_status(pk_ether(p, len, o), VC_PKT_ERR_ETHER);
    } else {
        const bool v6 = layer == VC_LAYER_IPV6;
        o->l3 = uint8_t(v6 ? VC_L3_IPV6 : VC_L3_IPV4);
        o->status = pk_status(v6 ? pk_ipv6(p, len, o) : pk_ipv4(p, len, o), VC_PKT_ERR_IP);
    }
    if (o->status != VC_PKT_OK) {
        pk_clear_ip(o);
        o->l3 = 0;
    }
}

}  // namespace vcd

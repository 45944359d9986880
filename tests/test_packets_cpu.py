"""Packet header extraction, CPU tier: the oracle's restatement of the
vpacket parsers (VXLanPacket / EthernetPacket / ArpPacket / Ipv4Packet /
Ipv6Packet / TcpPacket / IcmpPacket .from) pinned by the reference's own
TestPacket vectors (tests/golden/packets.json) and by quirk vectors derived
from the Java source."""
import json
import os

import oracle_ffi as O

G = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


def test_testpacket_vectors():
    with open(os.path.join(G, "packets.json")) as f:
        cases = json.load(f)["cases"]
    for c in cases:
        got = O.parse_packet(bytes.fromhex(c["hex"]), c["layer"])
        for k, v in c["want"].items():
            assert got[k] == v, (c["name"], k, got[k], v)


def _ipv4_tcp(tcp, proto=6):
    total = 20 + len(tcp)
    ip = bytes([0x45, 0, total >> 8, total & 255, 0, 0, 0, 0, 64, proto, 0, 0,
                10, 0, 0, 1, 10, 0, 0, 2])
    return ip + tcp


def _tcp(opts=b"", sport=1234, dport=80):
    doff = 20 + len(opts)
    assert doff % 4 == 0
    return bytes([sport >> 8, sport & 255, dport >> 8, dport & 255]) + bytes(8) + \
        bytes([(doff // 4) << 4, 0x02, 0xff, 0xff, 0, 0, 0, 0]) + opts


def test_quirks_from_source():
    # TCP option of length 0 / 1: TcpOption.from reads past its sub-array -> throws
    assert O.parse_packet(_ipv4_tcp(_tcp(bytes([8, 0, 1, 1]))), 4)["status"] == 4
    assert O.parse_packet(_ipv4_tcp(_tcp(bytes([8, 1, 1, 1]))), 4)["status"] == 4
    # ... and under an Ethernet frame the exception escapes mayIgnoreError
    eth = bytes(12) + b"\x08\x00"
    assert O.parse_packet(eth + _ipv4_tcp(_tcp(bytes([8, 0, 1, 1]))), 1)["status"] == 4
    # MSS option with the wrong length: an error string -> IP kept as bytes
    r = O.parse_packet(eth + _ipv4_tcp(_tcp(bytes([2, 3, 0, 0]))), 1)
    assert (r["status"], r["l3"]) == (0, 5)
    # END option stops option parsing
    r = O.parse_packet(_ipv4_tcp(_tcp(bytes([0, 0, 0, 0]))), 4)
    assert (r["status"], r["sport"], r["dport"]) == (0, 1234, 80)
    # UDP is PacketBytes in the reference: no ports
    r = O.parse_packet(_ipv4_tcp(bytes(8), proto=17), 4)
    assert (r["status"], r["l4"], r["sport"]) == (0, 0, 0)
    # IPv6 extension header whose next header is again an extension header:
    # Ipv6Packet.java:63-78 re-parses the same header forever
    v6 = bytes([0x60, 0, 0, 0, 0, 16, 0, 64]) + bytes(32) + bytes([43, 8]) + bytes(14)
    assert O.parse_packet(v6, 6)["status"] == 5
    # NO_NEXT_HEADER (59) with trailing bytes -> error
    v6 = bytes([0x60, 0, 0, 0, 0, 8, 59, 64]) + bytes(32) + bytes(8)
    assert O.parse_packet(v6, 6)["status"] == 3
    # too short at every layer
    assert O.parse_packet(bytes(7), 0)["status"] == 1
    assert O.parse_packet(bytes(8 + 13), 0)["status"] == 2
    # IPv4 totalLength must equal the buffer length
    assert O.parse_packet(_ipv4_tcp(_tcp()) + b"\0", 4)["status"] == 3


def test_device_parser_on_host_vs_oracle():
    """The kernels' parse_packet (device/packet_dev.h, run on the host by
    tests/native/imgcheck.hip) against the oracle, every layer."""
    import numpy as np
    import imgcheck_ffi as IC
    from cases import gen_frames
    frames = gen_frames(np.random.default_rng(7), 6000)
    for layer, cut in ((0, 0), (1, 8), (4, 22), (6, 22)):
        fr = [f[cut:] for f in frames]
        got = IC.packets(fr, layer)
        for f, g in zip(fr, got):
            assert g == O.parse_packet(f, layer), (layer, f.hex())
    st = [g["status"] for g in IC.packets(frames, 0)]
    assert all(st.count(k) > 0 for k in (0, 1, 2, 4, 5)), st   # every outcome exercised

#!/usr/bin/env python3
"""Writes tests/golden/packets.json: the packet byte vectors of the
reference's TestPacket (test/src/test/java/vproxy/test/cases/TestPacket.java)
with the outcomes its assertions state, plus the structures its generators
build (genIpv6 :76-95, vxlan(genEther(genArp)) :227-233) laid out by hand.

Run here (the reference tree exists only in this container); the JSON is
committed.  The byte values are data transcribed from the test file; no
reference code is run.
"""
import json
import os
import re

REF = "/root/reference/test/src/test/java/vproxy/test/cases/TestPacket.java"
OUT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "packets.json")


def byte_block(text, start_marker):
    """hex bytes of the first ByteArray.from( ... ) after start_marker"""
    i = text.index(start_marker)
    j = text.index("ByteArray.from(", i)
    k = text.index(");", j)
    return bytes(int(x, 16) for x in re.findall(r"0x([0-9a-fA-F]{2})", text[j:k]))


def main():
    text = open(REF).read()
    icmp4 = byte_block(text, "public void ipv4ByIcmpExample()")
    icmp6 = byte_block(text, "public void ipv6ByIcmpExample()")
    syn = byte_block(text, "public void tcpIpv4SynExample()")
    psh_i = text.index("public void tcpIpv4PshExample()")
    psh_h = byte_block(text[psh_i:], "ByteArray header")
    psh_d = byte_block(text[psh_i:], "ByteArray dataPart")
    cases = [
        # TestPacket.ipv4ByIcmpExample :135-158 -- parsed, payload IcmpPacket
        {"name": "ipv4ByIcmpExample", "layer": 4, "hex": icmp4.hex(),
         "want": {"status": 0, "l3": 4, "l4": 1, "proto": 1,
                  "src": "c0a80360", "dst": "c0a80301"}},
        # TestPacket.ipv6ByIcmpExample :167-193 -- parsed, payload IcmpPacket (ICMPv6)
        {"name": "ipv6ByIcmpExample", "layer": 6, "hex": icmp6.hex(),
         "want": {"status": 0, "l3": 6, "l4": 58, "proto": 58,
                  "src": "00" * 15 + "01", "dst": "00" * 15 + "01"}},
        # TestPacket.tcpIpv4SynExample :252-281 -- srcPort 62824, dstPort 443, 8 options
        {"name": "tcpIpv4SynExample", "layer": 1, "hex": syn.hex(),
         "want": {"status": 0, "l3": 4, "l4": 6, "proto": 6, "ether_type": 0x0800,
                  "sport": 62824, "dport": 443}},
        # TestPacket.tcpIpv4PshExample :283-350 -- srcPort 62824, dstPort 443, 517 data bytes
        {"name": "tcpIpv4PshExample", "layer": 1, "hex": (psh_h + psh_d).hex(),
         "want": {"status": 0, "l3": 4, "l4": 6, "proto": 6, "ether_type": 0x0800,
                  "sport": 62824, "dport": 443}},
    ]
    # genIpv6 (:76-95): next header 43 (routing) -> one ext header
    # (nextHeader 233, hdrExtLen 10, 8 + 10 bytes) -> 57 payload bytes
    v6 = bytes([0x60 | (28 >> 4), ((28 & 15) << 4) | 0x3, 0xab, 0xcd, 0, 75, 43, 123])
    v6 += bytes(range(1, 17)) + bytes(range(17, 33))
    v6 += bytes([233, 10]) + bytes(range(16)) + bytes(57)
    cases.append({"name": "genIpv6", "layer": 6, "hex": v6.hex(),
                  "want": {"status": 0, "l3": 6, "l4": 0, "proto": 233}})
    # vxlan(genEther(genArp)) (:220-233): vni 1314, ARP 6/4 sizes, 28 bytes
    arp = bytes([0, 1, 0x08, 0x00, 6, 4, 0, 1]) + bytes(range(6)) + bytes([10, 0, 0, 1]) + \
        bytes(range(6, 12)) + bytes([10, 0, 0, 2])
    eth = bytes(range(12)) + bytes([0x08, 0x06]) + arp
    vx = bytes([0b01000000, 0, 0, 0]) + (1314).to_bytes(3, "big") + b"\0" + eth
    cases.append({"name": "vxlan", "layer": 0, "hex": vx.hex(),
                  "want": {"status": 0, "l3": 1, "vni": 1314, "ether_type": 0x0806}})
    with open(OUT, "w") as f:
        json.dump({"source": "TestPacket.java", "cases": cases}, f, indent=1)
    print("wrote", OUT, len(cases), "cases")


if __name__ == "__main__":
    main()

"""DNSServer's drain loop per datagram (DNSServer.java:457-500): the oracle's
restatement (vo_dns_datagram) against the hand-derived datagram KATs in
tests/golden/kats.json (TestResolver.packet's packet among them), and the
wire builder's round trip."""
import json
import os
import random

import numpy as np

from vproxy_amd import dnswire as DW
import oracle_ffi as O
from vproxy_amd import workloads as W

HERE = os.path.dirname(os.path.abspath(__file__))


def kats():
    with open(os.path.join(HERE, "golden", "kats.json")) as f:
        return json.load(f)["dns_datagrams"]


def udp_rules(spec):
    """[[alias, net, min_port, max_port, allow]] -> RULE_DT array"""
    arr = O.sg_rule_arr([O.sg_rule(n, lo, hi, allow) for _, n, lo, hi, allow in spec])
    return np.frombuffer(bytes(arr), W.RULE_DT)[:len(spec)].copy()


def remotes(addrs):
    """IP strings -> (family, remote4, remote6[n, 16])"""
    n = len(addrs)
    fam, r4, r6 = np.zeros(n, np.uint8), np.zeros(n, np.uint32), np.zeros((n, 16), np.uint8)
    for i, a in enumerate(addrs):
        b = O.parse_ip(a)
        if len(b) == 4:
            fam[i], r4[i] = 4, int.from_bytes(b, "big")
        else:
            fam[i], r6[i] = 6, np.frombuffer(b, np.uint8)
    return fam, r4, r6


def kat_inputs(k):
    cases = k["cases"]
    blob, off = W.pack([bytes.fromhex(c["datagram"]) for c in cases])
    fam, r4, r6 = remotes([c["remote"] for c in cases])
    port = np.array([c["port"] for c in cases], np.uint16)
    return cases, blob, off, fam, r4, r6, port


def check_against_kats(res, cases):
    for i, c in enumerate(cases):
        got = (int(res["status"][i]), int(res["nq"][i]),
               [[int(res["qtype"][i][q]), int(res["kind"][i][q]), int(res["value"][i][q])]
                for q in range(int(res["nq"][i]))])
        assert got == (c["status"], c["nq"], c["questions"]), c["what"]


def test_oracle_dns_datagram_kats():
    k = kats()
    cases, blob, off, fam, r4, r6, port = kat_inputs(k)
    res = O.dnsd_batch_np(np.zeros(0, W.RULE_DT), udp_rules(k["udp_rules"]),
                          k["default_allow"], [tuple(x) for x in k["hosts"]], k["groups"], blob,
                          off, fam, r4, r6, port)
    check_against_kats(res, cases)
    # the rejected ones name the UDP rule that matched
    for i, c in enumerate(cases):
        if c["status"] == 3:
            assert res["acl"][i] in (0, 1), c["what"]


def test_wire_builder_layout():
    """dnswire.name is Formatter.formatDomainName (Formatter.java:98-127)."""
    assert DW.name("www.example.com.") == b"\x03www\x07example\x03com\x00"
    assert DW.name("www.example.com") == DW.name("www.example.com.")
    assert DW.name("") == b"\x00"
    assert DW.name("a.", ptr=12) == b"\x01a\xc0\x0c"
    p = DW.reference_packet()
    assert p[:4] == bytes([0xAB, 0xCD, 0x85, 0x80])    # response | aa | rd ; ra, NoError
    assert p[4:12] == bytes([0, 1, 0, 2, 0, 1, 0, 1])


def test_oracle_random_datagrams_are_total():
    """Every random and mutated datagram gets exactly one outcome; statuses
    that evaluate no question report nq == 0."""
    rng = random.Random(5)
    names = ["example.com.", "a.test.com.", "1.2.3.4.", "::1.", "x.vproxy.local.", "nope.org.",
             "db.example.com.", b"caf\xe9.com.", "."]
    dg = [DW.random_datagram(rng, names) for _ in range(3000)]
    blob, off = W.pack(dg)
    n = len(dg)
    res = O.dnsd_batch_np(np.zeros(0, W.RULE_DT), np.zeros(0, W.RULE_DT), True,
                          [("db.example.com.", 5)], [({}, {"host": "example.com"}),
                                                      ({}, {"host": "test.com"})],
                          blob, off, None, np.zeros(n, np.uint32), None,
                          np.full(n, 53, np.uint16), nthreads=4)
    st = res["status"]
    assert set(np.unique(st)) <= set(range(7))
    assert np.all(res["nq"][st >= 2] == 0)
    assert np.all(res["nq"] <= 4)
    for s in (0, 1, 2, 5, 6):          # answer, recursive, response, malformed, host all occur
        assert (st == s).sum() > 0, s

"""Pins the CPU oracle against the reference's own test vectors.

Fixtures in tests/golden/ are transcribed from the reference's JUnit tests
(TestNetMask, TestIpParser, TestRouteTable, TestSocks5, TestProtocols,
TestTcpLB, CI) and SURVEY.md Appendix B; see tests/golden/make_golden.py.
"""
import json
import os

import pytest

import oracle_ffi as O

G = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


def load(name):
    with open(os.path.join(G, name)) as f:
        return json.load(f)


def _bits(b):
    return "".join(format(x, "08b") for x in b)


def test_parse_mask():
    for v in load("netmask.json")["mask"]:
        assert _bits(O.parse_mask(v["m"])) == v["bits"], v
    with pytest.raises(ValueError):
        O.parse_mask(129)


def test_valid_network():
    for v in load("netmask.json")["valid_network"]:
        addr = O.parse_ip(v["addr"])
        assert addr is not None
        assert O.valid_network(addr, O.parse_mask(v["mask"])) == v["expect"], v


def _mm(v):
    inp = O.parse_ip(v["input"])
    ip_s, m = v["net"].rsplit("/", 1)
    rule = O.parse_ip(ip_s)
    assert inp is not None and rule is not None, v
    return O.mask_match(inp, rule, O.parse_mask(int(m)))


def test_ip_net_mask():
    for v in load("netmask.json")["mask_match"]:
        assert _mm(v) == v["expect"], v


def test_appendix_b_mask_match():
    for v in load("kats.json")["mask_match"]:
        assert _mm(v) == v["expect"], v


def test_ip_parser():
    d = load("ip_parser.json")
    for v in d["v4_ok"]:
        assert list(O.parse_ipv4(v["s"])) == v["bytes"]
    for s in d["v4_fail"]:
        assert O.parse_ipv4(s) is None, s
    for v in d["v6_ok"]:
        assert list(O.parse_ipv6(v["s"])) == v["bytes"], v
    for s in d["bogus"]:
        assert O.parse_ip(s) is None, s


def test_route_table_ordering():
    for case in load("route_table.json")["cases"]:
        t = O.RouteTable()
        for n in case["add"]:
            assert t.add(n)
        assert t.rules() == case["expect"], case["source"]
        for ip, want in case["lookups"]:
            assert t.lookup(O.parse_ip(ip)) == want, (case["source"], ip)


def test_route_table_duplicate():
    t = O.RouteTable()
    assert t.add("10.0.0.0/8")
    assert not t.add("10.0.0.0/8")


def test_hint_kats():
    for case in load("kats.json")["hints"]:
        g = O.Groups(case["groups"])
        for q, want in case["queries"]:
            got = O.search_for_group(g, q.get("host"), q.get("port", 0), q.get("uri"))
            assert got == want, (case["source"], q)


def test_dns_kats():
    for case in load("kats.json")["dns"]:
        g = O.Groups(case["groups"])
        h = O.Hosts(case["hosts"])
        for q, kind, value in case["queries"]:
            assert O.dns_classify(h, g, q) == (kind, value), (case["source"], q)


def test_dns_wire_kats():
    """qnames as wire bytes: (char) b per byte (Formatter.java:225-257), which
    sign-extends a byte >= 0x80 to U+FF80..U+FFFF, against UTF-8 annotations
    / hosts keys."""
    for case in load("kats.json")["dns_wire"]:
        g = O.Groups(case["groups"])
        h = O.Hosts(case["hosts"])
        for q, kind, value in case["queries"]:
            assert O.dns_classify(h, g, bytes.fromhex(q)) == (kind, value), (case["source"], q)


def test_match_level_counts_utf16_units():
    """Hint.matchLevel's uriLevel = String.length() + 1 (Hint.java:146-150):
    "/\u00e9" is 2 units (3 UTF-8 bytes), "/\U0001f600" 3 units (a surrogate
    pair; 5 bytes)."""
    for uri, units in (("/\u00e9", 2), ("/\U0001f600", 3), ("/a\u00e9\U0001f600b", 6)):
        ub = uri.encode()
        annos = (O.VoAnnos * 1)()
        annos[0].uri, annos[0].uri_len = ub, len(ub)
        for q in (uri, uri + "/tail"):
            h, keep = O.hint_of(None, 0, q)
            assert O.lib().vo_match_level(O.C.byref(h), annos, 1) == units + 1, (uri, q)


def test_security_group_scenarios():
    for case in load("kats.json")["security_group"]:
        tcp, udp, dflt = [], [], True
        names = {}
        for st in case["steps"]:
            if st[0] == "default":
                dflt = st[1]
            elif st[0] == "add":
                _, alias, n, proto, lo, hi, allow = st
                r = O.sg_rule(n, lo, hi, allow)
                (tcp if proto == "TCP" else udp).append(r)
                names[alias] = (proto, r)
            elif st[0] == "remove":
                proto, r = names.pop(st[1])
                lst = tcp if proto == "TCP" else udp
                lst[:] = [x for x in lst if x is not r]
            else:
                _, proto, ip, port, want = st
                _, verdict = O.sg_allow(tcp, udp, dflt, 6 if proto == "TCP" else 17,
                                        O.parse_ip(ip), port)
                assert verdict == want, (case["source"], st)


def test_hosts_parse():
    text = ("# comment\n127.0.0.1 localhost localhost.localdomain\n"
            "10.0.0.1\tdb.example.com. db # trailing\n"
            "bad line\n::1 localhost ip6-localhost\r\n\n10.0.0.2 db\n")
    pairs, ips = O.hosts_parse(text)
    d = dict(pairs)
    # Resolver.java:122-141: both x and x. keys, first occurrence wins
    assert d["localhost"] == 0 and d["localhost."] == 0
    assert d["db.example.com."] == 1 and d["db.example.com"] == 1
    assert d["db"] == 1 and d["db."] == 1
    assert d["ip6-localhost"] == 2
    assert ips[0] == bytes([127, 0, 0, 1]) and len(ips[2]) == 16
    # "10.0.0.2 db" parses but adds no key: "db" was already present
    assert all(v != 3 for _, v in pairs)


def test_cert_kats():
    """SSLContextHolder.choose with TestSSL.TEST_CERT's name and the
    certificates SSLContextHolder.checkSNI documents (kats.json certs)."""
    for case in load("kats.json")["certs"]:
        c = O.Certs(case["holders"])
        for sni, want in case["queries"]:
            assert c.choose(sni) == want, (case["source"], sni)


def test_hosts_text_kats():
    """Resolver.getHosts over an /etc/hosts text, then DNSServer's
    classification: TestResolver.resolve's localhost -> 127.0.0.1 line."""
    for case in load("kats.json")["hosts_text"]:
        pairs, ips = O.hosts_parse(case["text"])
        h = O.Hosts(pairs)
        g = O.Groups(case["groups"])
        for q, kind, value in case["queries"]:
            assert O.dns_classify(h, g, q) == (kind, value), (case["source"], q)
        assert ips[0] == bytes([127, 0, 0, 1])


def _ip_bytes(s):
    import ipaddress
    return ipaddress.ip_address(s).packed


def test_source_kats():
    """ServerGroup source hashing vs TestTcpLB.proxySource: the 127.0.0.1
    clients all reach svr0 (kats.json source)."""
    for case in load("kats.json")["source"]:
        servers = [(_ip_bytes(ip), port, w, h) for ip, port, w, h in case["servers"]]
        for client, view, want in case["queries"]:
            assert O.source_select(servers, view, _ip_bytes(client)) == want, case["source"]


def _hx(v):
    return bytes.fromhex(v) if v is not None else None


def test_http1_heads():
    """HttpSubContext's theUri / theHostHeader (TestHttp1Parser's request
    heads and the derived state-machine KATs, tests/golden/http1.json)."""
    for c in load("http1.json")["cases"]:
        assert O.http_extract(_hx(c["head"])) == (_hx(c["uri"]), _hx(c["host"])), c["what"]


def test_http1_connection_hint():
    """HttpContext.connectionHint (HttpContext.java:55-71): the hint kind
    follows which fields are set, and Upstream.searchForGroup sees the
    formatted host (port and 'www.' cut, Hint.java:57-73) and uri ('?' cut,
    trailing '/' cut, :75-90)."""
    groups = [({"host": "example.com"}, {}), ({"uri": "/hello"}, {}),
              ({"host": "*"}, {"uri": "/api"})]
    cases = [
        (b"GET /hello/url HTTP/1.1\r\nHost: www.example.com:8080\r\n\r\n", 0, 3),
        (b"GET /hello/url HTTP/1.1\r\n\r\n", 1, 1),
        (b"GET /api/?q=1 HTTP/1.1\r\nHost: other\r\n\r\n", 2, 3),
        (b"GET /none HTTP/1.1\r\nHost: other\r\n\r\n", 2, 3),      # "*" host: level 1 << 10
        (b"GET /none HTTP/1.1\r\n\r\n", -1, 1),
        (b"", -1, 0),
        (b"GET /hello/url HTTP/1.1\r\nHost: :80\r\n\r\n", 1, 3),   # formatHost -> null
    ]
    for head, group, kind in cases:
        assert O.http_hint(groups, head) == (group, kind), head
    # the batch form equals the single form
    blob = b"".join(h for h, _, _ in cases)
    import numpy as np
    off = np.cumsum([0] + [len(h) for h, _, _ in cases]).astype(np.uint32)
    kind, grp = O.http_batch_np(groups, np.frombuffer(blob, np.uint8), off, nthreads=2)
    assert list(grp) == [g for _, g, _ in cases] and list(kind) == [k for _, _, k in cases]

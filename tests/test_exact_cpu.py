"""CPU tier: the whole-batch checkers of tests/exact.py against the oracle.

The GPU tests compare every output of the headline batches with these
checkers, so each is first shown equal to the oracle's linear scans
(oracle/vc_oracle.c: vo_rt_lookup_list, vo_sg_allow, vo_search_for_group)
on random rule sets: the 255-rule C1 route table in RouteTable.addRule
order, a 20k-rule arbitrary-priority list with duplicate networks, IPv6
lists with 4-byte masks and ::/0, 64- to 10k-rule ACLs with both defaults
and every protocol, IPv6 sources against IPv4 rules (the cross-family
cases), and Upstream groups with hint-ports, "*" and suffix chains.
"""
import numpy as np
import pytest
import torch

import oracle_ffi as O
from exact import AclChecker, HintChecker, RouteChecker
from vproxy_amd import workloads as W

from cases import hint_cases_random, hint_cases_shapes, rule_row, v6_edge_inputs, ip_like_strings

CPU = torch.device("cpu")
THREADS = 8


def _np(t):
    return t.cpu().numpy()


def test_route_c1_order_vs_oracle():
    rng = np.random.default_rng(11)
    ot = O.RouteTable()
    ot.add("10.0.0.0/8")
    plen = rng.integers(8, 31, 600)
    net = rng.integers(0, 2**32, 600, dtype=np.uint64).astype(np.uint32) & W._mask32(plen)
    added = 0
    for i in range(600):
        s = "%d.%d.%d.%d/%d" % (net[i] >> 24, (net[i] >> 16) & 255, (net[i] >> 8) & 255,
                                net[i] & 255, plen[i])
        added += bool(ot.add(s))
        if added == 255:
            break
    v4, _ = O.rt_table_np(ot)
    q = W.v4_lookups(net, plen, 200_000, 12)
    np.testing.assert_array_equal(_np(RouteChecker(v4, 4, CPU)(q)),
                                  O.rt_batch_v4_np(v4, q, nthreads=THREADS))


def test_route_arbitrary_priority_vs_oracle():
    """20k prefixes /0-/32 in random list order, some networks listed twice
    (the earlier one must win), lookups inside and outside."""
    rng = np.random.default_rng(21)
    plen = rng.integers(0, 33, 20000)
    net = rng.integers(0, 2**32, 20000, dtype=np.uint64).astype(np.uint32) & W._mask32(plen)
    nets = W.v4_nets(net, plen)
    nets = np.concatenate([nets, nets[rng.integers(0, len(nets), 500)]])
    rng.shuffle(nets)
    q = W.v4_lookups(net, plen, 200_000, 22)
    q[:64] = [0, 0xFFFFFFFF] * 32
    np.testing.assert_array_equal(_np(RouteChecker(nets, 4, CPU)(q)),
                                  O.rt_batch_v4_np(nets, q, nthreads=THREADS))
    np.testing.assert_array_equal(_np(RouteChecker(nets[:0], 4, CPU)(q[:100])),
                                  np.full(100, -1, np.int32))


def test_route_shortest_first_vs_oracle():
    """The C3 generator's shape (BGP-like, shortest-first list)."""
    net, plen = W.gen_v4_prefixes(30000, 3)
    nets = W.v4_nets(net, plen)
    q = W.v4_lookups(net, plen, 100_000, 4)
    np.testing.assert_array_equal(_np(RouteChecker(nets, 4, CPU)(q)),
                                  O.rt_batch_v4_np(nets, q, nthreads=THREADS))


def test_route_v6_vs_oracle():
    hi, lo, p6 = W.gen_v6_prefixes(5000, 31)
    nets6 = np.concatenate([W.v6_nets(hi, lo, p6), W.v6_nets([0], [0], [0]),
                            W.v6_nets(hi[:50], lo[:50], np.minimum(p6[:50], 24))])
    rng = np.random.default_rng(3)
    rng.shuffle(nets6)
    assert (nets6["mask_len"] == 4).any()
    q = W.v6_lookups(hi, lo, p6, 100_000, 23)
    got = _np(RouteChecker(nets6, 6, CPU)(q))
    np.testing.assert_array_equal(got, O.rt_batch_v6_np(nets6, q, nthreads=THREADS))
    # without the ::/0 rule some lookups miss
    keep = nets6[~((nets6["mask_len"] == 4) & (nets6["mask"][:, 0] == 0))]
    got = _np(RouteChecker(keep, 6, CPU)(q))
    np.testing.assert_array_equal(got, O.rt_batch_v6_np(keep, q, nthreads=THREADS))
    assert (got == -1).any()


@pytest.mark.parametrize("n_rules,p_range,weighted,seed", [
    (64, 0.5, False, 1), (2000, 0.3, True, 2), (10000, 0.3, True, 3), (3000, 0.95, False, 4)])
def test_acl_v4_vs_oracle(n_rules, p_range, weighted, seed):
    tcp, udp = W.gen_sg_rules(n_rules, seed, p_range=p_range, weighted=weighted)
    # a network listed several times with different port ranges (a run of
    # equal keys the checker scans) and a catch-all late in the list
    extra = np.concatenate([rule_row("10.1.0.0/16", lo, lo + 9, lo % 2) for lo in range(0, 200, 7)]
                           + [rule_row("0.0.0.0/0", 0, 65535, True)])
    tcp = np.concatenate([tcp[: len(tcp) // 2], extra, tcp[len(tcp) // 2:]])
    proto, src, port = W.gen_acl_queries(tcp, udp, 200_000, seed + 100)
    proto[::97] = 1                                    # not TCP: the UDP list
    src[::89] = 0x0A010000 | (src[::89] & 0xFFFF)
    for dflt in (False, True):
        chk = AclChecker(tcp, udp, dflt, CPU)
        got, allow = chk.v4(proto, src, port)
        want, wv = O.sg_batch_v4_np(tcp, udp, dflt, proto, src, port, nthreads=THREADS)
        np.testing.assert_array_equal(_np(got), want)
        np.testing.assert_array_equal(_np(allow), wv)
    for t, u in ((tcp[:0], udp), (tcp, udp[:0])):
        got, allow = AclChecker(t, u, True, CPU).v4(proto[:5000], src[:5000], port[:5000])
        want, wv = O.sg_batch_v4_np(t, u, True, proto[:5000], src[:5000], port[:5000])
        np.testing.assert_array_equal(_np(got), want)
        np.testing.assert_array_equal(_np(allow), wv)


def test_acl_v6_sources_on_v4_rules_vs_oracle():
    tcp, udp = W.gen_sg_rules(1500, 8)
    extra = np.concatenate([rule_row(s, 0, 65535, a) for s, a in (
        ("127.0.0.1/32", True), ("8.8.8.0/24", False), ("0.0.0.0/0", True))])
    tcp = np.concatenate([extra[:2], tcp, extra[2:]])
    udp = np.concatenate([udp, extra])
    rng = np.random.default_rng(9)
    src6, proto, port = v6_edge_inputs(rng, 100_000)
    # some mapped addresses inside real rule networks
    ip, mk = W.rule_v4_fields(tcp[2:])
    r = rng.integers(0, len(ip), 100_000)
    inside = (ip[r] | (rng.integers(0, 2**32, 100_000, dtype=np.uint64).astype(np.uint32) & ~mk[r]))
    pick = (src6[:, :10] == 0).all(1) & (rng.random(100_000) < 0.5)
    src6[pick, 12:] = W.v4_to_bytes(inside[pick])
    for dflt in (False, True):
        got, allow = AclChecker(tcp, udp, dflt, CPU).v6(proto, src6, port)
        want, wv = O.sg_batch_v6_np(tcp, udp, dflt, proto, src6, port, nthreads=THREADS)
        np.testing.assert_array_equal(_np(got), want)
        np.testing.assert_array_equal(_np(allow), wv)
    assert (want >= 0).mean() > 0.1


def test_hint_dict_vs_oracle_generated():
    groups, ghosts = W.gen_groups(3000, 17, port_frac=0.3)
    # repeated hosts (member lists), a second "*", handle annotations
    groups += [({}, {"host": ghosts[5]}), ({}, {"host": "*", "port": "80"}),
               ({"host": ghosts[9]}, {"host": "zz.none"}), ({}, {"port": "443"})]
    names = W.gen_hostnames(ghosts, 60_000, 18, port_frac=0.3)
    names += [b"www.", b":80", b"www.:80", b"", b"*", b"a.*", b"." + ghosts[3].encode()]
    blob, off = W.pack(names)
    rng = np.random.default_rng(19)
    ports = rng.choice(np.array([0, 0, 80, 443, 8080], np.uint16), len(names))
    gp = [int(g[1]["port"]) for g in groups[:3000] if "port" in g[1]]
    ports[::7] = rng.choice(np.array(gp, np.uint16), len(ports[::7]))
    chk = HintChecker(groups)
    og = O.Groups(groups)
    for p in (None, ports):
        want = O.hint_batch_np(og, blob, off, p, nthreads=THREADS)
        np.testing.assert_array_equal(chk.batch(blob, off, p), want)
    assert (want >= 0).mean() > 0.5


def test_hint_dict_vs_oracle_edge_cases():
    rng = np.random.default_rng(23)
    groups, _, queries = hint_cases_random(rng, 400, 20000)
    names = [(h, p) for h, p, _ in queries if h is not None]
    g2, n2 = hint_cases_shapes(rng, 20000)
    chk, og = HintChecker(groups), O.Groups(groups)
    for h, p in names:
        assert chk(h.encode(), p) == O.search_for_group(og, h, p), (h, p)
    chk, og = HintChecker(g2), O.Groups(g2)
    blob, off = W.pack(n2)
    np.testing.assert_array_equal(chk.batch(blob, off), O.hint_batch_np(og, blob, off, None,
                                                                        nthreads=THREADS))


def test_java_ip_predicates_vs_oracle():
    """exact.java_is_ipv6 / java_is_ip_literal (IP.isIpv6 / isIpLiteral
    restated on bytes) against the oracle's parser: the TestIpParser vectors
    (tests/golden/ip_parser.json) and 200k literal-shaped strings, the
    parser's quirks included ("::" twice, a bad colon part before a dotted
    tail, brackets, 1-4 hex digits)."""
    import json
    import os
    from exact import java_is_ip_literal, java_is_ipv6
    with open(os.path.join(os.path.dirname(__file__), "golden", "ip_parser.json")) as f:
        d = json.load(f)
    fixed = [v["s"] for v in d["v4_ok"] + d["v6_ok"]] + d["v4_fail"] + d["bogus"]
    fixed = [x.encode() for x in fixed] + [b"", b":", b"::", b":::", b"[]", b"[::]", b"::1.2.3.4",
                                           b"::a:zz:1.2.3.4", b"1::2::3", b"a:b:c:d:e:f:1.2.3.4"]
    strings = fixed + ip_like_strings(np.random.default_rng(41), 200_000)
    v6 = [java_is_ipv6(x) for x in strings]
    assert v6 == [O.parse_ipv6(x) is not None for x in strings]
    assert [java_is_ip_literal(x) for x in strings] == [O.is_ip_literal(x) for x in strings]
    assert 0.05 < np.mean(v6) < 0.95
    for v in d["v6_ok"]:
        assert java_is_ipv6(v["s"].encode())


def test_hosts_map_vs_oracle_parser():
    """exact.hosts_map (dict restatement of Resolver.getHosts) equals the
    oracle's parser on comments, CRLF, tabs, invalid IPs, dot-twins and
    first-occurrence-wins lines, and on the kats.json hosts texts."""
    import json
    import os
    from exact import hosts_map
    texts = [("# comment\n127.0.0.1 localhost localhost.localdomain\n"
              "10.0.0.1\tdb.example.com. db # trailing\n"
              "bad line\n::1 localhost ip6-localhost\r\n\n10.0.0.2 db\n"
              "300.1.1.1 nope.example\n  \t\n10.1.1.1   spaced.example\t\ttab.example.\r"
              "fe80::1%eth0 scoped.example\n10.2.2.2 db. fresh.example # x\n01.2.3.4 lead.zero\n")]
    with open(os.path.join(os.path.dirname(__file__), "golden", "kats.json")) as f:
        texts += [c["text"] for c in json.load(f)["hosts_text"]]
    for text in texts:
        pairs, _ = O.hosts_parse(text)
        want = {}
        for k, v in pairs:
            want.setdefault(k.encode(), v)
        assert hosts_map(text, O.is_ip_literal) == want


def test_dns_checker_vs_oracle():
    """DnsChecker against vo_dns_classify on the DNS-flavoured C4 names
    (trailing dots), hosts keys in both forms, IP literals, .vproxy.local
    names and misses, with and without a "*" group."""
    from exact import DnsChecker
    groups, ghosts = W.gen_groups(2000, 31, port_frac=0.1)
    hosts = "\n".join("10.0.%d.%d h%d.hosts.local%s" % (i >> 8 & 255, i & 255, i,
                                                         "." if i % 3 == 0 else "")
                      for i in range(3000)) + "\n# c\n::1 six.hosts.local\n"
    names = W.gen_hostnames(ghosts, 20000, 32, dns=True, port_frac=0)
    names += [b"h%d.hosts.local" % i for i in range(0, 3000, 7)]
    names += [b"h%d.hosts.local." % i for i in range(1, 3000, 7)]
    names += [b"1.2.3.4", b"1.2.3.4.", b"::1", b"::1.", b"[::1]", b"2001:db8::1.",
              b"a.vproxy.local.", b"vproxy.local", b"x.vproxy.local", b"six.hosts.local.",
              b"01.2.3.4.", b"", b".", b"..", b"miss.nowhere.", b"www.x:80", b"1.2.3.256."]
    for gs in (groups, [g for g in groups if g[1].get("host") != "*"]):
        oh, og = O.Hosts(O.hosts_parse(hosts)[0]), O.Groups(gs)
        chk = DnsChecker(hosts, gs)
        blob, off = W.pack(names)
        kind, val = chk.batch(blob, off)
        wk, wv = O.dns_batch_np(oh, og, blob, off, nthreads=THREADS)
        np.testing.assert_array_equal(kind, wk)
        np.testing.assert_array_equal(val, wv)
        assert len(set(wk.tolist())) >= (2 if gs is groups else 4)


def test_hint_level_checker_vs_oracle():
    """HintLevelChecker (searchForGroup with hint-uri levels, the port filter
    and every host level) against vo_search_for_group: the random edge-case
    groups and queries of cases.hint_cases_random (overlapping hosts,
    handle/group merging, ports, uris with '?', '/', '*', nulls), and the
    generated C4 groups with hint-uris added."""
    from exact import HintLevelChecker
    rng = np.random.default_rng(71)
    groups, _, queries = hint_cases_random(rng, 400, 20000)
    og = O.Groups(groups)
    chk = HintLevelChecker(groups)
    enc = lambda x: None if x is None else x.encode()
    for h, p, u in queries:
        assert chk(enc(h), p, enc(u)) == O.search_for_group(og, h, p, u), (h, p, u)
    # generated groups with uris (a quarter), uri-only groups, queries with paths
    g2, hosts = W.gen_groups(3000, 72, port_frac=0.1)
    paths = ["/", "/api", "/api/v1", "/api/v1/users", "/static", "/static/img/a.png", "*",
             "/api/", "/x?y=1"]
    for i in range(0, len(g2), 4):
        g2[i][1]["uri"] = paths[i % len(paths)]
    g2 += [({}, {"uri": p}) for p in paths]
    names = W.gen_hostnames(hosts, 20000, 73, port_frac=0.2)
    qp = rng.choice(np.array([0, 0, 80, 443]), len(names))
    qu = [None if rng.random() < 0.2 else
          paths[int(rng.integers(0, len(paths)))] + ("/" + str(int(rng.integers(0, 5)))
                                                      if rng.random() < 0.5 else "")
          for _ in names]
    og2 = O.Groups(g2)
    chk2 = HintLevelChecker(g2)
    got = [chk2(n, int(p), enc(u)) for n, p, u in zip(names, qp, qu)]
    want = [O.search_for_group(og2, n, int(p), u) for n, p, u in zip(names, qp, qu)]
    assert got == want
    assert len(set(want)) > 1000


def test_cert_checker_vs_oracle():
    """CertChecker against vo_cert_choose: generated holders with plain,
    wildcard and shared names, SNIs that hit plain names, wildcard depths
    (one extra label, two, none), empty labels and nulls; one- and
    zero-holder tables."""
    from exact import CertChecker
    _, hosts = W.gen_groups(6000, 61, wildcard=False)
    holders = [[hosts[i], "*." + hosts[i + 1], "shared%d.example" % (i % 37)]
               for i in range(0, len(hosts), 2)]
    holders += [["*.x.example", "a.x.example"], ["*.example", "*"], [""], ["*."]]
    names = W.gen_hostnames(hosts, 20000, 62)
    snis = [n.split(b":")[0] for n in names]
    snis += [b"a." + h.encode() for h in hosts[1:400:2]] + [b"a.b." + h.encode() for h in hosts[1:200:2]]
    snis += [b"x.example", b"q.x.example", b".x.example", b"a.example", b"", b".", b"*", b"*.",
             b"shared3.example", b"a.shared3.example"]
    for hs in (holders, holders[:1], []):
        chk, oc = CertChecker(hs), O.Certs(hs)
        got = [chk(s) for s in snis] + [chk(None)]
        want = [oc.choose(s) for s in snis] + [oc.choose(None)]
        assert got == want


def test_source_checker_vs_oracle():
    """SourceChecker against vo_source_batch: groups of 0-31 servers with
    duplicate addresses (the stable sort), zero weights, IPv6 servers in the
    all-view, unhealthy runs (the forward probe) and all-unhealthy groups;
    clients with high-bit bytes (signed sdbm), 0 and 255.255.255.255."""
    from exact import SourceChecker
    rng = np.random.default_rng(83)
    groups = []
    for k in range(600):
        g = []
        for _ in range(int(rng.integers(0, 32))):
            ip = bytes(rng.integers(0, 256, 4 if rng.random() < 0.9 else 16).astype(np.uint8))
            if g and rng.random() < 0.1:
                ip = g[int(rng.integers(0, len(g)))][0]           # duplicate address
            g.append((ip, int(rng.choice([80, 443, 8080])), int(rng.random() < 0.9),
                      bool(rng.random() < (0.0 if k % 50 == 0 else 0.7))))
        groups.append(g)
    n = 200_000
    grp = rng.integers(0, len(groups), n).astype(np.int32)
    src = rng.integers(0, 2**32, n, dtype=np.uint64).astype(np.uint32)
    src[:4] = [0, 0xFFFFFFFF, 0x80000000, 0x7F000001]
    got = SourceChecker(groups, CPU).v4(grp, src).numpy()
    want = O.source_batch_np(groups, 0, grp, src, nthreads=THREADS)
    np.testing.assert_array_equal(got, want)
    assert (want >= 0).mean() > 0.5 and (want < 0).any()


def test_hint_level_table_vs_checker_and_oracle():
    """HintLevelChecker.table (the whole-batch form the c4uri checks use:
    port 0, every (name, uri) pair) against the per-item checker on every
    pair and against vo_hint_uri_batch on a sample: the c4uri generator at
    3,000 groups (a fifth with hint-uris, 200 uri-only groups) and 2,000
    names with the 66 uris and a null one."""
    import bench
    from exact import HintLevelChecker
    groups, names, uris, nidx, uidx = bench.c4uri_workload(20000, n_groups=3000, n_names=2000)
    og = O.Groups(groups)
    chk = HintLevelChecker(groups)
    cols = uris + [None]
    tab = chk.table(names, cols)
    for i, name in enumerate(names[:600]):
        assert [chk(name, 0, u) for u in cols] == list(tab[i]), name
    u = np.where(uidx < 0, len(uris), uidx)
    want = tab[nidx, u]
    hb, ho = W.pack([names[i] for i in nidx])
    ub, uo = W.pack([uris[max(j, 0)] for j in uidx])
    got = O.hint_uri_batch_np(og, hb, ho, ub, uo, (uidx < 0).astype(np.uint8), nthreads=8)
    np.testing.assert_array_equal(got, want)
    assert len(np.unique(want)) > 500 and (want >= 0).mean() > 0.5
    # the uri decides: some names change group with the uri
    assert (tab[:, :-1] != tab[:, -1:]).any(axis=1).mean() > 0.02

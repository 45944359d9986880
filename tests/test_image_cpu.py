"""CPU tier: the product's table compilers + the kernels' own probe code
(walked on the host by the test harness) against the oracle.

The GPU tier (test_gpu_*.py) repeats these comparisons with the real HIP
kernels; this tier catches compile/image bugs without a GPU.
"""
import numpy as np
import pytest

import imgcheck_ffi as IC
import oracle_ffi as O
from vproxy_amd import workloads as W
from vproxy_amd.classifier import group_array, pack_strings

from cases import acl_edge_rules, rule_row, v6_edge_inputs, hint_cases_random


@pytest.mark.parametrize("n_rules,p_range,weighted,seed", [
    (64, 0.5, False, 1),        # C1 shape
    (2000, 0.3, True, 2),       # C2 generator, reduced
    (300, 0.9, True, 3),        # wide port ranges -> multi-piece port functions
])
def test_acl_v4_random(n_rules, p_range, weighted, seed):
    tcp, udp = W.gen_sg_rules(n_rules, seed, p_range=p_range, weighted=weighted)
    proto, src, port = W.gen_acl_queries(tcp, udp, 40000, seed + 100)
    for dflt in (False, True):
        got, allow, _ = IC.acl(tcp, udp, dflt, 4, proto, src, port)
        want, wv = O.sg_batch_v4_np(tcp, udp, dflt, proto, src, port, nthreads=4)
        np.testing.assert_array_equal(got, want)
        np.testing.assert_array_equal(allow, wv)


@pytest.mark.parametrize("n_rules", [25000, 70000])
def test_acl_v4_directory_and_records_large(n_rules):
    """Lists of ~25k and ~70k intervals: the bucket directory (images.h
    dir4, built for 17-65535 intervals: here 16-bit buckets holding ~0.4 or
    none) and the 16-byte interval records; the harness checks every lookup
    against a whole binary search and the (x, y) + pieces form, and the
    results against the oracle on a sample."""
    tcp, udp = W.gen_sg_rules(n_rules, 9, p_range=0.3, weighted=True)
    proto, src, port = W.gen_acl_queries(tcp, udp, 6000, 109)
    got, allow, stats = IC.acl(tcp, udp, False, 4, proto, src, port)
    want, wv = O.sg_batch_v4_np(tcp, udp, False, proto, src, port, nthreads=8)
    np.testing.assert_array_equal(got, want)
    np.testing.assert_array_equal(allow, wv)


@pytest.mark.parametrize("n_rules,p_range,seed", [(64, 0.5, 11), (10000, 0.3, 12), (3000, 0.95, 13)])
def test_acl_port_image(n_rules, p_range, seed):
    """The UDP list's IPv4 image at one bind port (build_acl_port: the switch
    kernel's LDS table, Switch.java:679 allow(UDP, remote, bind port)) equals
    the general image at that port at every interval edge, and the oracle's
    SecurityGroup.allow scan on sample keys; C5's list (10k rules) at the
    VXLAN port stays within the kernel's 256-interval LDS copy."""
    tcp, udp = W.gen_sg_rules(n_rules, seed, p_range=p_range, weighted=True)
    rng = np.random.default_rng(seed)
    nets = W.rule_v4_fields(udp)[0] if len(udp) else np.zeros(1, np.uint32)
    keys = np.concatenate([rng.integers(0, 2**32, 3000, dtype=np.uint64).astype(np.uint32),
                           nets[rng.integers(0, len(nets), 3000)]])
    for port in (4789, 53, 0, 65535, int(udp["min_port"][0])):
        got, nb = IC.acl_port(udp, port, keys)
        proto = np.full(len(keys), 17, np.uint8)
        pr = np.full(len(keys), port, np.uint16)
        want, _ = O.sg_batch_v4_np(tcp, udp, False, proto, keys, pr, nthreads=4)
        np.testing.assert_array_equal(got, want)
        if n_rules == 10000 and port == 4789:
            assert nb <= 256, nb


def test_acl_edges_v4_v6():
    tcp, udp = acl_edge_rules()
    rng = np.random.default_rng(7)
    src6, proto6, port6 = v6_edge_inputs(rng, 20000)
    src4 = src6[:, 12:].copy().view(">u4").reshape(-1).astype(np.uint32)
    for dflt in (False, True):
        got, allow, _ = IC.acl(tcp, udp, dflt, 6, proto6, src6, port6)
        want, wv = O.sg_batch_v6_np(tcp, udp, dflt, proto6, src6, port6)
        np.testing.assert_array_equal(got, want)
        np.testing.assert_array_equal(allow, wv)
        got, allow, _ = IC.acl(tcp, udp, dflt, 4, proto6, src4, port6)
        want, wv = O.sg_batch_v4_np(tcp, udp, dflt, proto6, src4, port6)
        np.testing.assert_array_equal(got, want)
        np.testing.assert_array_equal(allow, wv)


@pytest.mark.parametrize("n_rules,seed", [(64, 1), (2000, 2), (10000, 3)])
def test_acl_v6_sources_on_v4_only_lists(n_rules, seed):
    """Lists of plain IPv4 rules (every bench workload's) take the kernels'
    shortcut for IPv6 sources (acl_dev.h acl6_global, AclFamilyImage.v4_only):
    the ::a.b.c.d / ::ffff:a.b.c.d forms classified through the v4 image on
    their low 32 bits, every other key as no rule.  The harness checks each
    lookup against the 128-bit search over the same list's v6 image, and the
    results against the oracle's Network.maskMatch restatement."""
    tcp, udp = W.gen_sg_rules(n_rules, seed)
    rng = np.random.default_rng(seed + 50)
    src6, proto, port = v6_edge_inputs(rng, 30000)
    ip, mk = W.rule_v4_fields(tcp)
    r = rng.integers(0, len(ip), 30000)
    inside = ip[r] | (rng.integers(0, 2**32, 30000, dtype=np.uint64).astype(np.uint32) & ~mk[r])
    pick = (src6[:, :10] == 0).all(1) & (rng.random(30000) < 0.6)
    src6[pick, 12:] = W.v4_to_bytes(inside[pick])
    proto[pick] = 6
    lo, hi = tcp["min_port"][r].astype(np.int64), tcp["max_port"][r].astype(np.int64)
    port[pick] = (lo + (rng.random(30000) * (hi - lo + 1)).astype(np.int64))[pick].astype(np.uint16)
    for dflt in (False, True):
        got, allow, stats = IC.acl(tcp, udp, dflt, 6, proto, src6, port)
        want, wv = O.sg_batch_v6_np(tcp, udp, dflt, proto, src6, port)
        np.testing.assert_array_equal(got, want)
        np.testing.assert_array_equal(allow, wv)
        assert stats[8] + stats[9] == len(port)          # every lookup took the shortcut
    assert (want >= 0).mean() > 0.05
    # one IPv6 rule in the TCP list turns its shortcut off (the UDP one stays)
    tcp6 = np.concatenate([tcp, rule_row("::ffff:10.0.0.0/104", 0, 65535, True)])
    got, allow, stats = IC.acl(tcp6, udp, False, 6, proto, src6, port)
    want, wv = O.sg_batch_v6_np(tcp6, udp, False, proto, src6, port)
    np.testing.assert_array_equal(got, want)
    assert stats[8] == 0 and stats[9] == (proto != 6).sum()


def test_acl_empty_lists():
    tcp, udp = W.gen_sg_rules(20, 5)
    empty = tcp[:0]
    proto, src, port = W.gen_acl_queries(tcp, udp, 5000, 6)
    for t, u in ((empty, udp), (tcp, empty), (empty, empty)):
        for dflt in (False, True):
            got, allow, _ = IC.acl(t, u, dflt, 4, proto, src, port)
            want, wv = O.sg_batch_v4_np(t, u, dflt, proto, src, port)
            np.testing.assert_array_equal(got, want)
            np.testing.assert_array_equal(allow, wv)


def _c1_route_table(seed):
    """RouteTable(Table{10.0.0.0/8}) + 255 CIDRs /8-/30 in random order,
    through the oracle's exact addRule heuristic."""
    rng = np.random.default_rng(seed)
    plen = rng.integers(8, 31, 400)
    net = rng.integers(0, 2**32, 400, dtype=np.uint64).astype(np.uint32) & W._mask32(plen)
    t = O.RouteTable()
    t.add("10.0.0.0/8")
    nets = W.v4_nets(net, plen)
    added = 0
    for i in range(len(nets)):
        if added == 255:
            break
        n = O.VoNet.from_buffer_copy(nets[i].tobytes())
        if O.lib().vo_rt_add(O.C.byref(t.t), O.C.byref(n)) == 0:
            added += 1
    return t


def test_route_c1_random_order():
    t = _c1_route_table(11)
    v4, _ = O.rt_table_np(t)
    q = W.v4_lookups(v4["ip"][:, :4].copy().view(">u4").reshape(-1).astype(np.uint32),
                     np.array([O.lib().vo_mask_int((O.C.c_uint8 * 16)(*r["mask"]), 4) for r in v4]),
                     50000, 12)
    got, stats = IC.route(v4, 4, q)
    want = O.rt_batch_v4_np(v4, q, nthreads=4)
    np.testing.assert_array_equal(got, want)


def test_route_v4_deep_and_long():
    """prefixes longer than the root stride (/25-/32) and nested chains."""
    rng = np.random.default_rng(21)
    plen = rng.integers(0, 33, 6000)
    net = rng.integers(0, 2**32, 6000, dtype=np.uint64).astype(np.uint32) & W._mask32(plen)
    net[:200] = net[200] & W._mask32(plen[:200])   # nested chain around one address
    key = (net.astype(np.uint64) << 8) | plen.astype(np.uint64)
    _, first = np.unique(key, return_index=True)
    first = np.sort(first)
    nets = W.v4_nets(net[first], plen[first])
    rng.shuffle(nets)     # arbitrary list order: priority = index, not length
    q = W.v4_lookups(net[first], plen[first], 40000, 22)
    for nr in (len(nets), 1000):   # 24-bit and 16-bit roots by default
        want = O.rt_batch_v4_np(nets[:nr], q, nthreads=4)
        for rb in (0, 16, 20, 24):
            got, stats = IC.route(nets[:nr], 4, q, rb)
            np.testing.assert_array_equal(got, want)
            assert rb == 0 or stats[0] == rb


def test_route_root_20_edges():
    """A 20-bit root strides 4 bits to the byte boundary, then 8: prefixes
    of every length 16-32 nested in a few root slots, list order shuffled,
    queries with each bit 18-25 flipped (the first node's edges)."""
    rng = np.random.default_rng(23)
    base = rng.integers(0, 2**32, 12, dtype=np.uint64).astype(np.uint32)
    plen = rng.integers(16, 33, 3000)
    net = (base[rng.integers(0, 12, 3000)] ^ rng.integers(0, 2**16, 3000).astype(np.uint32))
    net = net & W._mask32(plen)
    key = (net.astype(np.uint64) << 8) | plen.astype(np.uint64)
    _, first = np.unique(key, return_index=True)
    nets = W.v4_nets(net[first], plen[first])
    rng.shuffle(nets)
    q = W.v4_lookups(net[first], plen[first], 20000, 24, inside=1.0)
    q = np.concatenate([q] + [q[:2000] ^ np.uint32(1 << (31 - b)) for b in range(18, 26)])
    want = O.rt_batch_v4_np(nets, q, nthreads=4)
    got, stats = IC.route(nets, 4, q, 20)
    np.testing.assert_array_equal(got, want)
    assert stats[0] == 20 and stats[1] > 0, stats
    hi, lo, p6 = W.gen_v6_prefixes(3000, 25)
    n6 = W.v6_nets(hi, lo, p6)
    q6 = W.v6_lookups(hi, lo, p6, 20000, 26)
    q6 = np.concatenate([q6] + [_flip(q6[:2000], b) for b in (19, 20, 23, 24, 31)])
    want6 = O.rt_batch_v6_np(n6, q6, nthreads=4)
    for rb in (16, 20, 24):
        got, stats = IC.route(n6, 6, q6, rb)
        np.testing.assert_array_equal(got, want6)
        assert stats[0] == rb


def test_route_v6():
    hi, lo, plen = W.gen_v6_prefixes(3000, 31)
    nets = W.v6_nets(hi, lo, plen)
    nets = np.concatenate([nets, W.v6_nets([0], [0], [0])])   # ::/0 last
    q = W.v6_lookups(hi, lo, plen, 30000, 32)
    got, _ = IC.route(nets, 6, q)
    want = O.rt_batch_v6_np(nets, q, nthreads=4)
    np.testing.assert_array_equal(got, want)


def _flip(q6, bit):
    """q6 [n,16] with address bit `bit` (0 = most significant) flipped"""
    out = q6.copy()
    out[:, bit // 8] ^= np.uint8(0x80 >> (bit % 8))
    return out


def test_route_one_prefix_records():
    """Root slots holding a single longer prefix compile to one-prefix
    records (images.h VC_ONE).  Edges: length 64 (the record limit) and 65
    (nodes), a covering shorter prefix listed before and after the long one
    (the record's match value is the min), slots with two long prefixes
    (nodes), and queries one bit inside / outside each prefix.  Every IPv6
    key is also looked up through the wide root (images.h TrieImage.wide,
    built per slot by route_dev.h wide_entry) and must get the same answer."""
    rng = np.random.default_rng(51)
    n = 1500
    plen = rng.choice(np.array([25, 30, 32, 40, 47, 48, 56, 63, 64, 65, 80]), n)
    hi = rng.integers(0, 2**64, n, dtype=np.uint64)
    lo = rng.integers(0, 2**64, n, dtype=np.uint64)
    hm = np.where(plen >= 64, np.uint64(2**64 - 1),
                  np.uint64(2**64 - 1) << (64 - np.minimum(plen, 64)).astype(np.uint64))
    lm = np.where(plen > 64, np.uint64(2**64 - 1) << (128 - np.maximum(plen, 65)).astype(np.uint64),
                  np.uint64(0))
    hi &= hm
    lo &= lm
    hi[:100] = (hi[100:200] & np.uint64(0xFFFFFF0000000000)) | (hi[:100] & np.uint64(0xFFFFFFFFFF))
    hi[:100] &= hm[:100]                                  # 100 slots with two long prefixes
    cover_p = rng.integers(16, 24, 300)                   # shorter covering prefixes
    cover_h = hi[200:500] & (np.uint64(2**64 - 1) << (64 - cover_p).astype(np.uint64))
    all_hi = np.concatenate([hi, cover_h])
    all_lo = np.concatenate([lo, np.zeros(300, np.uint64)])
    all_p = np.concatenate([plen, cover_p])
    nets = W.v6_nets(all_hi, all_lo, all_p)
    rng.shuffle(nets)                                     # list order = priority
    q = W.v6_lookups(all_hi, all_lo, all_p, 20000, 52, inside=1.0)
    qb = np.concatenate([q] + [_flip(q[:3000], b) for b in (23, 24, 31, 39, 46, 47, 55, 62, 63, 64)])
    got, stats = IC.route(nets, 6, qb)
    want = O.rt_batch_v6_np(nets, qb, nthreads=4)
    np.testing.assert_array_equal(got, want)
    assert stats[0] == 16 and stats[2] > 500 and stats[1] > 0, stats
    # 24-bit root: pad the table past 4096 rules with far-away /12s
    pad = W.v6_nets(np.arange(4000, dtype=np.uint64) << np.uint64(52),
                    np.zeros(4000, np.uint64), np.full(4000, 12))
    big = np.concatenate([nets, pad])
    got, stats = IC.route(big, 6, qb)
    np.testing.assert_array_equal(got, O.rt_batch_v6_np(big, qb, nthreads=4))
    assert stats[0] == 24 and stats[2] > 500, stats
    # the IPv6 wide root (every key above also went through it, harness rc
    # -201 otherwise) answers the one-prefix slots' keys in one load
    assert stats[3] > len(qb) // 4, stats
    # IPv4 with a 16-bit root: /17-/32 prefixes alone in their slot
    p4 = rng.integers(17, 33, 2000)
    n4 = rng.integers(0, 2**32, 2000, dtype=np.uint64).astype(np.uint32) & W._mask32(p4)
    c4p = rng.integers(8, 17, 200)
    c4 = n4[:200] & W._mask32(c4p)
    v4n = W.v4_nets(np.concatenate([n4, c4]), np.concatenate([p4, c4p]))
    rng.shuffle(v4n)
    q4 = W.v4_lookups(np.concatenate([n4, c4]), np.concatenate([p4, c4p]), 20000, 53, inside=1.0)
    q4 = np.concatenate([q4, q4 ^ np.uint32(1 << 15), q4 ^ np.uint32(1), q4 ^ np.uint32(1 << 8)])
    got, stats = IC.route(v4n, 4, q4)
    np.testing.assert_array_equal(got, O.rt_batch_v4_np(v4n, q4, nthreads=4))
    assert stats[0] == 16 and stats[2] > 1000, stats
    # the same under a 20-bit root (records for /21-/32 alone in their slot)
    got, stats = IC.route(v4n, 4, q4, 20)
    np.testing.assert_array_equal(got, O.rt_batch_v4_np(v4n, q4, nthreads=4))
    assert stats[0] == 20 and stats[2] > 1000, stats
    got, stats = IC.route(nets, 6, qb, 20)
    np.testing.assert_array_equal(got, O.rt_batch_v6_np(nets, qb, nthreads=4))
    assert stats[0] == 20 and stats[2] > 500, stats


def test_hint_random():
    groups, hosts, queries = hint_cases_random(np.random.default_rng(41), 800, 20000)
    arr, ng, keep = group_array(groups)
    h = pack_strings([q[0] for q in queries])
    ports = np.array([q[1] for q in queries], np.uint16)
    u = pack_strings([q[2] for q in queries])
    got = IC.hint(arr, ng, h, ports, u)
    og = O.Groups(groups)
    want = np.array([O.search_for_group(og, q[0], q[1], q[2]) for q in queries], np.int32)
    np.testing.assert_array_equal(got, want)
    # host-only batch (uri null everywhere) exercises the summary fast path
    got2 = IC.hint(arr, ng, h, ports, None)
    want2 = np.array([O.search_for_group(og, q[0], q[1], None) for q in queries], np.int32)
    np.testing.assert_array_equal(got2, want2)


def test_hint_kats_on_image():
    import json
    import os
    with open(os.path.join(os.path.dirname(__file__), "golden", "kats.json")) as f:
        kats = json.load(f)
    for case in kats["hints"]:
        arr, ng, keep = group_array(case["groups"])
        qs = case["queries"]
        h = pack_strings([q.get("host") for q, _ in qs])
        u = pack_strings([q.get("uri") for q, _ in qs])
        p = np.array([q.get("port", 0) for q, _ in qs], np.uint16)
        got = IC.hint(arr, ng, h, p, u)
        assert list(got) == [w for _, w in qs], case["source"]


def test_device_ip_literal_parser():
    import json
    import os
    with open(os.path.join(os.path.dirname(__file__), "golden", "ip_parser.json")) as f:
        d = json.load(f)
    strs = [v["s"] for v in d["v6_ok"]] + d["bogus"] + [v["s"] for v in d["v4_ok"]] + d["v4_fail"]
    strs += ["::x:1.2.3.4", "::hello:1.2.3.4", "1:2:3:4:5:6:7:1.2.3.4", "::1:2:3:4:5:6:7:1.2.3.4",
             "[::1]", "[", "]", "[]", "::", ":::", "1::2:", "::ffff:1.2.3.4", "a.b:80",
             "www.example.com:8080", "fe80::1%eth0", "1.2.3.04", "0.0.0.0", "255.255.255.255"]
    rng = np.random.default_rng(3)
    alpha = list("0123456789abcdefABCDEF:.[]xg")
    for _ in range(4000):
        strs.append("".join(rng.choice(alpha, int(rng.integers(0, 20)))))
    for s in strs:
        assert IC.is_ipv6(s) == (O.parse_ipv6(s) is not None), s
        assert IC.is_ip_literal(s) == O.is_ip_literal(s), s


def test_hint_dense_table():
    """~30k distinct hint-hosts in a 64K-slot table: full 4-slot tag groups,
    so probes continue past the first group (the batched probe path)."""
    groups, ghosts = W.gen_groups(30000, 61)
    arr, ng, keep = group_array(groups)
    names = W.gen_hostnames(ghosts, 4000, 62)
    h = pack_strings(names)
    ports = np.random.default_rng(63).choice(np.array([0, 0, 80, 8080], np.uint16), len(names))
    got = IC.hint(arr, ng, h, ports, None)
    og = O.Groups(groups)
    blob, off = W.pack(names)
    want = O.hint_batch_np(og, blob, off, ports, nthreads=8)
    np.testing.assert_array_equal(got, want)


def test_dns_image():
    groups, ghosts = W.gen_groups(20000, 71)
    arr, ng, keep = group_array(groups)
    pairs = [(h + ".", i) for i, h in enumerate(ghosts[:5000])] + [("localhost.", 999)]
    names = W.gen_hostnames(ghosts, 3000, 72, dns=True)
    names += [b"1.2.3.4.", b"::1.", b"[::1].", b"a.vproxy.local.", b".", b"", b"::ffff:1.2.3.4.",
              b"::x:1.2.3.4.", b"www.x.com:80."]
    qb, qo = W.pack(names)
    kind, val = IC.dns(pairs, arr, ng, qb, qo)
    og = O.Groups(groups)
    oh = O.Hosts(pairs)
    want = [O.dns_classify(oh, og, q) for q in names]
    assert [(int(k), int(v)) for k, v in zip(kind, val)] == want


def test_dns_hosts_dot_forms():
    """The hosts table holds names without one trailing dot (.b tells them
    apart): a name and the name + "." are distinct keys, first entry wins,
    and the probe is made on the dotted qname's scan hash, on a colon
    name's own hash, and before the slow group path (many labels)."""
    groups, ghosts = W.gen_groups(2000, 75)
    arr, ng, keep = group_array(groups)
    pairs = [("a.example.", 1), ("a.example", 2), ("b.example", 3), ("c.example..", 4),
             ("c.example.", 5), ("a.example.", 9), ("x:1.", 6), ("p.q.r.s.t.u.v.w.", 7),
             ("", 8), (".", 10), ("\u00e9.example.", 11), (ghosts[0] + ".", 12), (ghosts[1], 13),
             ("www.y.com:80.", 14), ("e.f::1.", 15)]
    names = [b"a.example.", b"a.example", b"b.example.", b"b.example", b"c.example..",
             b"c.example.", b"c.example", b"x:1.", b"x:1", b"p.q.r.s.t.u.v.w.", b"p.q.r.s.t.u.v.w",
             b".", b"", b"..", b"\xe9.example.", b"\xe9.example", (ghosts[0] + ".").encode(),
             ghosts[0].encode(), (ghosts[1] + ".").encode(), ghosts[1].encode(),
             b"www.y.com:80.", b"www.y.com:80", b"e.f::1.", b"e.f::1"]
    qb, qo = W.pack(names)
    kind, val = IC.dns(pairs, arr, ng, qb, qo)
    og = O.Groups(groups)
    oh = O.Hosts(pairs)
    want = [O.dns_classify(oh, og, q) for q in names]
    assert [(int(k), int(v)) for k, v in zip(kind, val)] == want
    assert sum(1 for k, _ in want if k == 1) >= 12        # VC_DNS_HOSTS hits


def test_hint_fast_path_shapes():
    """The kernels' word-at-a-time fast path (plain and LDS-staged sources at
    every alignment, checked inside the harness) vs the oracle on the hard
    hostname shapes of cases.hint_cases_shapes."""
    from cases import hint_cases_shapes
    groups, names = hint_cases_shapes(np.random.default_rng(91), 6000)
    arr, ng, keep = group_array(groups)
    h = pack_strings(names)
    ports = np.random.default_rng(92).choice(np.array([0, 0, 80, 8080], np.uint16), len(names))
    got = IC.hint(arr, ng, h, ports, None)
    og = O.Groups(groups)
    blob, off = W.pack(names)
    want = O.hint_batch_np(og, blob, off, ports, nthreads=8)
    np.testing.assert_array_equal(got, want)


def test_hint_bench_names_are_never_deferred():
    """The C4 / C5 hostname generator's names (exact, sub-domain, miss, with
    ':port' and 'www.') all take the kernel's fast path: the deferring form
    leaves none of them to the follow-up kernel, so that kernel only reads
    its count and exits in the benchmarks.  Shapes the fast path does not
    cover (IPv6 literals, many labels, port filters) are deferred."""
    from vproxy_amd import workloads as W
    groups, ghosts = W.gen_groups(20000, W.SEED + 5)
    arr, ng, keep = group_array(groups)
    names = W.gen_hostnames(ghosts, 20000, W.SEED + 6, pool=20000)
    blob, off = W.pack(names)
    h = (blob, off.astype(np.uint32), None)
    og = O.Groups(groups)
    got = IC.hint(arr, ng, h, None, None)
    assert IC.hint_deferred() == 0
    want = O.hint_batch_np(og, blob, off, None, nthreads=4)
    np.testing.assert_array_equal(got, want)
    odd = [b"[::1]:8080", b"fe80::1", b"a.b.c.d.e.f.g.h", b"x.com:80"]
    blob, off = W.pack(odd)
    IC.hint(arr, ng, (blob, off.astype(np.uint32), None), np.full(len(odd), 80, np.uint16), None)
    assert IC.hint_deferred() >= 3


@pytest.mark.parametrize("wildcards", [0.0, 0.02])
def test_hint_uri_fast_path_on_image(wildcards):
    """The uri-aware fast path (host_only_fast with `uri`: the host answer,
    a SPLIT key's slot for uri_in_slot, or deferred) and the follow-up's
    level-ordered port-0 search (hint_port0_uri) against the general search
    on every port-0 uri hint (imgcheck ic_hint: -105 / -106 on a mismatch),
    over groups that share hint-hosts with and without hint-uris, several
    matching suffix keys, "*" groups, hosts no key lists and uris with '?',
    '*', '' and over 60 bytes; a sample against the oracle."""
    import test_gpu_c4uri as T
    rng = np.random.default_rng(17)
    hosts = ["a.com", "b.a.com", "c.b.a.com", "x.org", "y.x.org", "z.net", "com", "org"]
    g = T._split_groups(rng, hosts, 300, wildcards)
    qh = hosts + ["d.c.b.a.com", "q.z.net", "nope.io", "www.a.com:80", "a.com:8080", ":80",
                  "m.y.x.org", "[::1]:80"]
    qu = ["/a/b/c/x", "/a/b", "/a/", "/a?x=1", "/", "/b/q", "/zz", "*", "/a/b/c/d/e/f?g", "*x",
          "", "?", "/" + "/".join("abcdefghijklmnopqrstuvwxyz0123456")]
    n = 12000
    hs = [None if rng.random() < 0.05 else qh[int(rng.integers(0, len(qh)))] for _ in range(n)]
    us = [qu[int(rng.integers(0, len(qu)))] for _ in range(n)]
    arr, ng, keep = group_array(g)
    out = IC.hint(arr, ng, pack_strings(hs), np.zeros(n, np.uint16), pack_strings(us))
    og = O.Groups(g)
    s = rng.integers(0, n, 1500)
    assert [int(out[i]) for i in s] == [O.search_for_group(og, hs[i], 0, us[i]) for i in s]
    assert 0 < IC.hint_deferred() < n

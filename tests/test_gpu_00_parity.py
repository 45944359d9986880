"""GPU tier: the HIP kernels, called through the C ABI, against the oracle.

Bit-exact comparisons on seeded inputs at oracle-friendly sizes, plus full
BASELINE-size tables with oracle-checked samples and size-independent
properties.  Everything here runs on the MI355X box (`-m gpu`).
"""
import json
import os

import numpy as np
import pytest

import oracle_ffi as O
import vproxy_amd as V
from exact import AclChecker, HintChecker, RouteChecker
from vproxy_amd import workloads as W
from vproxy_amd.classifier import group_array, pack_strings

from cases import acl_edge_rules, hint_cases_random, v6_edge_inputs

pytestmark = pytest.mark.gpu
G = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")
THREADS = min(16, os.cpu_count() or 1)


@pytest.fixture(scope="module")
def clf():
    c = V.Classifier(0)
    yield c
    c.close()


def _acl_rules(tcp, udp):
    a, na, ka = W.as_ctypes(tcp, V._lib.VcAclRule)
    b, nb, kb = W.as_ctypes(udp, V._lib.VcAclRule)
    return (a, na, ka), (b, nb, kb)


def compile_acl_np(clf, tcp, udp, dflt):
    (a, na, _), (b, nb, _) = _acl_rules(tcp, udp)
    V.check(V.lib().vc_compile_acl(clf.h, a, na, b, nb, 1 if dflt else 0))


# ---------------------------------------------------------------------------
# SecurityGroup ACL
# ---------------------------------------------------------------------------
@pytest.mark.parametrize("n_rules,p_range,weighted,nq,seed", [
    (64, 0.5, False, 1 << 20, 1),      # C1: 64 rules over 1M 5-tuples (full)
    (2000, 0.3, True, 200000, 2),
    (300, 0.9, True, 100003, 3),       # odd n: vector tail
])
def test_acl_v4_vs_oracle(clf, n_rules, p_range, weighted, nq, seed):
    tcp, udp = W.gen_sg_rules(n_rules, seed, p_range=p_range, weighted=weighted)
    proto, src, port = W.gen_acl_queries(tcp, udp, nq, seed + 100)
    for dflt in (False, True):
        compile_acl_np(clf, tcp, udp, dflt)
        got, allow = clf.acl_v4(proto, src, port)
        want, wv = O.sg_batch_v4_np(tcp, udp, dflt, proto, src, port, nthreads=THREADS)
        np.testing.assert_array_equal(got, want)
        np.testing.assert_array_equal(allow, wv)


def test_acl_c2_full_size(clf):
    """C2: 10k-rule ACL, 64M IPv4 5-tuples resident in HBM; oracle-checked
    sample, whole-batch properties, and every output equal to the exact
    first-match checker."""
    import torch
    tcp, udp = W.gen_sg_rules(10000, W.SEED + 2, p_range=0.3)
    compile_acl_np(clf, tcp, udp, False)
    n = 64 << 20
    proto, src, port = W.gen_acl_queries(tcp, udp, n, W.SEED + 20)
    d = [torch.from_numpy(x).cuda() for x in (proto, src, port)]
    idx, allow = clf.acl_v4(*d)
    torch.cuda.synchronize()
    idx_h, allow_h = idx.cpu().numpy(), allow.cpu().numpy()
    rng = np.random.default_rng(5)
    s = rng.integers(0, n, 100000)
    want, wv = O.sg_batch_v4_np(tcp, udp, False, proto[s], src[s], port[s], nthreads=THREADS)
    np.testing.assert_array_equal(idx_h[s], want)
    np.testing.assert_array_equal(allow_h[s], wv)
    # properties over all 64M: the index names a rule of the item's protocol
    # that really matches it, and allow == that rule's bit (default when -1)
    tcp_n = len(tcp)
    hit = idx_h >= 0
    is_tcp = proto == 6
    assert np.all(idx_h[is_tcp] < tcp_n) and np.all(idx_h[~is_tcp] < len(udp))
    for lst, sel in ((tcp, is_tcp & hit), (udp, ~is_tcp & hit)):
        ip, mk = W.rule_v4_fields(lst)
        r = idx_h[sel]
        assert np.all((src[sel] & mk[r]) == ip[r])
        assert np.all((port[sel] >= lst["min_port"][r]) & (port[sel] <= lst["max_port"][r]))
        assert np.all(allow_h[sel] == lst["allow"][r])
    assert np.all(allow_h[~hit] == 0)
    # every one of the 64M: the first match (tests/exact.py, oracle-validated)
    want_i, want_a = AclChecker(tcp, udp, False, d[0].device).v4(*d)
    assert torch.equal(idx, want_i), int((idx != want_i).sum())
    assert torch.equal(allow, want_a)


@pytest.mark.parametrize("n", [(1 << 22) + (1 << 20) + 3,        # the verdict's size
                               4 * (11 * 131072 + 777) + 1,     # odd pass count, tail 1
                               4 * (2 * 131072) + 2])           # just at the two-quad threshold
def test_acl_two_quad_passes_and_tail(clf, n):
    """vc_acl_classify_v4_dev on the C2 tables at sizes that run the
    two-quad kernel (acl_v4_kernel<true, 2>: launch_acl_v4 picks it once
    n / 4 >= grid x 256 x 2) with a partial last pass -- its second quad past
    the end is searched but not stored -- and the n & 3 tail: every output
    against the exact checker, the last 20k and a spread sample against the
    oracle (SecurityGroup.java:30-45)."""
    import torch
    tcp, udp = W.gen_sg_rules(10000, W.SEED + 2, p_range=0.3)
    compile_acl_np(clf, tcp, udp, False)
    proto, src, port = W.gen_acl_queries(tcp, udp, n, n & 0xFFFF)
    d = [torch.from_numpy(x).cuda() for x in (proto, src, port)]
    idx, allow = clf.acl_v4(*d)
    torch.cuda.synchronize()
    want_i, want_a = AclChecker(tcp, udp, False, d[0].device).v4(*d)
    assert torch.equal(idx, want_i), int((idx != want_i).sum())
    assert torch.equal(allow, want_a)
    s = np.concatenate([np.arange(n - 20000, n), np.random.default_rng(n).integers(0, n, 20000)])
    want, wv = O.sg_batch_v4_np(tcp, udp, False, proto[s], src[s], port[s], nthreads=THREADS)
    np.testing.assert_array_equal(idx.cpu().numpy()[s], want)
    np.testing.assert_array_equal(allow.cpu().numpy()[s], wv)


def test_acl_edges_and_paths(clf):
    import torch
    tcp, udp = acl_edge_rules()
    rng = np.random.default_rng(7)
    src6, proto, port = v6_edge_inputs(rng, 50001)
    src4 = src6[:, 12:].copy().view(">u4").reshape(-1).astype(np.uint32)
    for dflt in (False, True):
        compile_acl_np(clf, tcp, udp, dflt)
        want6, wv6 = O.sg_batch_v6_np(tcp, udp, dflt, proto, src6, port)
        got, allow = clf.acl_v6(proto, src6, port)
        np.testing.assert_array_equal(got, want6)
        np.testing.assert_array_equal(allow, wv6)
        want4, wv4 = O.sg_batch_v4_np(tcp, udp, dflt, proto, src4, port)
        got, allow = clf.acl_v4(proto, src4, port)
        np.testing.assert_array_equal(got, want4)
        np.testing.assert_array_equal(allow, wv4)
        # device path, aligned (vector kernel) and misaligned (scalar kernel)
        dp, ds, dq = (torch.from_numpy(x).cuda() for x in (proto, src4, port))
        gi, ga = clf.acl_v4(dp, ds, dq)
        np.testing.assert_array_equal(gi.cpu().numpy(), want4)
        np.testing.assert_array_equal(ga.cpu().numpy(), wv4)
        gi, ga = clf.acl_v4(dp[1:], ds[1:], dq[1:])
        np.testing.assert_array_equal(gi.cpu().numpy(), want4[1:])
        d6 = torch.from_numpy(src6).cuda()
        gi, ga = clf.acl_v6(dp, d6, dq)
        np.testing.assert_array_equal(gi.cpu().numpy(), want6)


def test_acl_empty_and_tiny_batches(clf):
    tcp, udp = W.gen_sg_rules(30, 5)
    for t, u in ((tcp[:0], udp), (tcp, udp[:0]), (tcp[:0], udp[:0])):
        compile_acl_np(clf, t, u, True)
        for n in (0, 1, 2, 3, 4, 5, 1023):
            proto, src, port = W.gen_acl_queries(tcp, udp, n, n + 9)
            got, allow = clf.acl_v4(proto, src, port)
            want, wv = O.sg_batch_v4_np(t, u, True, proto, src, port)
            np.testing.assert_array_equal(got, want)
            np.testing.assert_array_equal(allow, wv)


def test_security_group_scenarios_on_gpu(clf):
    """TestTcpLB/CI security-group flows through the C++ mirror + GPU."""
    with open(os.path.join(G, "kats.json")) as f:
        kats = json.load(f)
    for case in kats["security_group"]:
        sg = V.SecurityGroup("secg", True)
        for st in case["steps"]:
            if st[0] == "default":
                sg.default_allow = st[1]
            elif st[0] == "add":
                _, alias, n, proto, lo, hi, allow = st
                sg.add_rule(alias, n, proto, lo, hi, allow)
            elif st[0] == "remove":
                sg.remove_rule(st[1])
            else:
                _, proto, ip, port, want = st
                clf.compile_security_group(sg)
                ipb = V.parse_ip(ip)
                src = np.frombuffer(ipb, ">u4").astype(np.uint32)
                _, allow = clf.acl_v4(np.array([6 if proto == "TCP" else 17], np.uint8), src,
                                      np.array([port], np.uint16))
                assert bool(allow[0]) == want, (case["source"], st)


# ---------------------------------------------------------------------------
# RouteTable
# ---------------------------------------------------------------------------
def test_route_golden_and_f3(clf):
    with open(os.path.join(G, "route_table.json")) as f:
        cases = json.load(f)["cases"]
    for case in cases:
        rt = V.RouteTable()
        for i, n in enumerate(case["add"]):
            rt.add_rule("r%d" % i, n)
        assert [str(x) for x in rt.get_rules()] == case["expect"]
        clf.compile_route_table(rt)
        if case["lookups"]:
            ips = np.array([int.from_bytes(V.parse_ip(ip), "big") for ip, _ in case["lookups"]],
                           np.uint32)
            assert list(clf.route_v4(ips)) == [w for _, w in case["lookups"]]


def test_route_c1_random_order(clf):
    rng = np.random.default_rng(11)
    rt = V.RouteTable("10.0.0.0/8", None, 1)
    ot = O.RouteTable()
    ot.add("10.0.0.0/8")
    plen = rng.integers(8, 31, 600)
    net = rng.integers(0, 2**32, 600, dtype=np.uint64).astype(np.uint32) & W._mask32(plen)
    added = 0
    for i in range(600):
        s = "%d.%d.%d.%d/%d" % (net[i] >> 24, (net[i] >> 16) & 255, (net[i] >> 8) & 255,
                                net[i] & 255, plen[i])
        if ot.add(s):
            rt.add_rule("r%d" % i, s)
            added += 1
        if added == 255:
            break
    assert [str(x) for x in rt.get_rules()] == ot.rules()
    clf.compile_route_table(rt)
    v4, _ = O.rt_table_np(ot)
    q = W.v4_lookups(net, plen, 1 << 20, 12)
    np.testing.assert_array_equal(clf.route_v4(q), O.rt_batch_v4_np(v4, q, nthreads=THREADS))


def test_route_arbitrary_priority_and_v6(clf):
    rng = np.random.default_rng(21)
    plen = rng.integers(0, 33, 6000)
    net = rng.integers(0, 2**32, 6000, dtype=np.uint64).astype(np.uint32) & W._mask32(plen)
    key = (net.astype(np.uint64) << 8) | plen.astype(np.uint64)
    _, first = np.unique(key, return_index=True)
    nets4 = W.v4_nets(net[np.sort(first)], plen[np.sort(first)])
    rng.shuffle(nets4)
    hi, lo, p6 = W.gen_v6_prefixes(5000, 31)
    nets6 = np.concatenate([W.v6_nets(hi, lo, p6), W.v6_nets([0], [0], [0])])
    rng.shuffle(nets6)
    a, na, ka = W.as_ctypes(nets4, V._lib.VcNet)
    b, nb, kb = W.as_ctypes(nets6, V._lib.VcNet)
    clf.compile_routes_raw(a, na, b, nb)
    q4 = W.v4_lookups(net, plen, 300001, 22)
    np.testing.assert_array_equal(clf.route_v4(q4), O.rt_batch_v4_np(nets4, q4, nthreads=THREADS))
    q6 = W.v6_lookups(hi, lo, p6, 100000, 23)
    np.testing.assert_array_equal(clf.route_v6(q6), O.rt_batch_v6_np(nets6, q6, nthreads=THREADS))


def test_route_c3_full_size(clf):
    """C3: ~1M IPv4 + 200k IPv6 prefixes inserted shortest-first through the
    RouteTable mirror (first match == LPM there); 16M device-resident
    lookups; oracle-checked sample, LPM properties, and every v4 and v6
    output equal to the exact per-length checker."""
    import torch
    net, plen = W.gen_v4_prefixes(1000000, W.SEED + 3)
    hi, lo, p6 = W.gen_v6_prefixes(200000, W.SEED + 4)
    rt = V.RouteTable()
    allnets = np.concatenate([W.v4_nets(net, plen), W.v6_nets(hi, lo, p6)])
    arr, n, keep = W.as_ctypes(allnets, V._lib.VcNet)
    assert rt.add_rules("bgp", arr, n=n)
    clf.compile_route_table(rt)
    a4, n4 = rt.rules_raw(4)
    a6, n6 = rt.rules_raw(6)
    v4 = np.frombuffer(bytes(a4)[:n4 * 40], W.NET_DT)
    v6 = np.frombuffer(bytes(a6)[:n6 * 40], W.NET_DT)
    q4 = W.v4_lookups(net, plen, 16 << 20, 41)
    clf.counters_enable(True)
    clf.counters_reset()
    got4 = clf.route_v4(torch.from_numpy(q4).cuda()).cpu().numpy()
    torch.cuda.synchronize()
    # hit counters (bucketed histogram path: ~30 chunks of 32K rules)
    cr = clf.counters_read(V.COUNTERS_ROUTE)
    exp = np.bincount(np.where(got4 >= 0, got4, n4 + n6), minlength=n4 + n6 + 2)
    np.testing.assert_array_equal(cr, exp.astype(np.uint64))
    clf.counters_enable(False)
    s = np.random.default_rng(1).integers(0, len(q4), 3000)
    np.testing.assert_array_equal(got4[s], O.rt_batch_v4_np(v4, q4[s], nthreads=THREADS))
    # every hit's prefix contains the address; 90% of lookups were drawn inside one
    ip, mk = v4["ip"][:, :4].copy().view(">u4").reshape(-1), v4["mask"][:, :4].copy().view(
        ">u4").reshape(-1)
    h = got4 >= 0
    assert np.all((q4[h] & mk[got4[h]]) == ip[got4[h]])
    assert h.mean() > 0.9
    # every one of the 16M: the first match in list order (tests/exact.py)
    dev = torch.device("cuda", 0)
    want4 = RouteChecker(v4, 4, dev)(q4).cpu().numpy()
    np.testing.assert_array_equal(got4, want4)
    q6 = W.v6_lookups(hi, lo, p6, 1 << 20, 42)
    got6 = clf.route_v6(torch.from_numpy(q6).cuda()).cpu().numpy()
    s = np.random.default_rng(2).integers(0, len(q6), 2000)
    np.testing.assert_array_equal(got6[s], O.rt_batch_v6_np(v6, q6[s], nthreads=THREADS))
    np.testing.assert_array_equal(got6, RouteChecker(v6, 6, dev)(q6).cpu().numpy())


# ---------------------------------------------------------------------------
# Upstream hints / DNS
# ---------------------------------------------------------------------------
def test_hint_kats(clf):
    with open(os.path.join(G, "kats.json")) as f:
        kats = json.load(f)
    for case in kats["hints"]:
        clf.compile_upstream(case["groups"])
        qs = case["queries"]
        got = clf.hint_search([q.get("host") for q, _ in qs],
                              np.array([q.get("port", 0) for q, _ in qs], np.uint16),
                              [q.get("uri") for q, _ in qs])
        assert list(got) == [w for _, w in qs], case["source"]


def test_hint_random_vs_oracle(clf):
    groups, hosts, queries = hint_cases_random(np.random.default_rng(41), 800, 50000)
    clf.compile_upstream(groups)
    og = O.Groups(groups)
    hs = [q[0] for q in queries]
    ps = np.array([q[1] for q in queries], np.uint16)
    us = [q[2] for q in queries]
    got = clf.hint_search(hs, ps, us)
    want = np.array([O.search_for_group(og, q[0], q[1], q[2]) for q in queries], np.int32)
    np.testing.assert_array_equal(got, want)
    got = clf.hint_search(hs, ps, None)
    want = np.array([O.search_for_group(og, q[0], q[1], None) for q in queries], np.int32)
    np.testing.assert_array_equal(got, want)


def test_hint_work_tickets_wrap(clf):
    """The string kernels take work tickets from a ring of 4096 per-launch
    device counters (launch.h TicketRing) that each launch's last wave
    resets: over 4500 launches (every slot reused) of sizes around the
    64-item chunk and the tail- and big-ticket edges, on two streams, every
    result equals the oracle's."""
    import ctypes as C
    import torch
    groups, hosts, queries = hint_cases_random(np.random.default_rng(43), 300, 7000)
    clf.compile_upstream(groups)
    og = O.Groups(groups)
    hs = [q[0] for q in queries if q[0] is not None][:6000]
    want = np.array([O.search_for_group(og, h, 0, None) for h in hs], np.int32)
    blob, off, _ = pack_strings(hs)
    bd = torch.from_numpy(blob).cuda()
    od = torch.from_numpy(off.astype(np.int32)).cuda()
    # chunk (64 items), tail-ticket (8 chunks) and big-ticket (24 chunks)
    # edges (chunks.h)
    sizes = [1, 63, 64, 65, 511, 512, 513, 1535, 1536, 1537, 3000, 6000]
    streams = [torch.cuda.Stream(), torch.cuda.Stream()]
    outs = []
    for k in range(4500):
        n = sizes[k % len(sizes)]
        s = streams[k % 2]
        with torch.cuda.stream(s):
            o = torch.empty(n, dtype=torch.int32, device="cuda")
            V.check(V.lib().vc_hint_search_dev(
                clf.h, C.c_void_p(bd.data_ptr()), C.c_void_p(od.data_ptr()), None, None, None,
                None, None, n, C.c_void_p(o.data_ptr()), C.c_void_p(s.cuda_stream)))
        if k % 500 == 0 or k >= 4490:
            outs.append((n, o))
    torch.cuda.synchronize()
    for n, o in outs:
        np.testing.assert_array_equal(o.cpu().numpy(), want[:n])


def test_hint_deferred_lanes_over_slot_reuse(clf):
    """The host-only pool pass leaves lanes that need an out-of-line step
    (port filters over hint-port minima, IPv6 literals and other names the
    word scan does not cover, chunks too long for the stage) to a second
    kernel, counted in the launch's ticket slot, which that kernel resets.
    Over 4300 launches (every slot reused) of batches with and without such
    lanes, on two streams, every result equals the oracle's."""
    import ctypes as C
    import torch
    from cases import hint_cases_shapes
    groups, names = hint_cases_shapes(np.random.default_rng(97), 6000)
    clf.compile_upstream(groups)
    og = O.Groups(groups)
    ports = np.random.default_rng(98).choice(np.array([0, 0, 80, 8080], np.uint16), len(names))
    blob, off = W.pack(names)
    want = O.hint_batch_np(og, blob, off, ports, nthreads=THREADS)
    zero = O.hint_batch_np(og, blob, off, np.zeros_like(ports), nthreads=THREADS)
    bd = torch.from_numpy(blob.astype(np.uint8)).cuda()
    od = torch.from_numpy(off.astype(np.int32)).cuda()
    pd = torch.from_numpy(ports.astype(np.int16)).cuda()
    sizes = [1, 64, 65, 1025, 3000, 6000]
    streams = [torch.cuda.Stream(), torch.cuda.Stream()]
    outs = []
    for k in range(4300):
        n = sizes[k % len(sizes)]
        s = streams[k % 2]
        with_ports = (k // len(sizes)) % 2 == 0
        with torch.cuda.stream(s):
            o = torch.empty(n, dtype=torch.int32, device="cuda")
            V.check(V.lib().vc_hint_search_dev(
                clf.h, C.c_void_p(bd.data_ptr()), C.c_void_p(od.data_ptr()), None,
                C.c_void_p(pd.data_ptr()) if with_ports else None, None, None, None, n,
                C.c_void_p(o.data_ptr()), C.c_void_p(s.cuda_stream)))
        if k % 300 < 12 or k >= 4288:
            outs.append((n, with_ports, o))
    torch.cuda.synchronize()
    for n, with_ports, o in outs:
        np.testing.assert_array_equal(o.cpu().numpy(), (want if with_ports else zero)[:n])


def test_dns_deferred_queries_over_slot_reuse(clf):
    """dns_kernel leaves the queries that may be IP literals, carry bytes
    >= 0x80 or have names the host scan does not cover to a second kernel
    (counted in the launch's ticket slot, which that kernel resets).  Over
    4300 launches of batches with and without such queries, on two streams,
    every result equals the one-shot host call's (itself checked against the
    oracle by test_dns_kats_and_random)."""
    import ctypes as C
    import torch
    groups, ghosts = W.gen_groups(2000, 87)
    clf.compile_upstream(groups)
    clf.compile_hosts([(h + ".", i) for i, h in enumerate(ghosts[:40])])
    rng = np.random.default_rng(88)
    plain = W.gen_hostnames(ghosts, 3000, 89, dns=True)
    odd = [b"1.2.3.4.", b"::1.", b"[::1].", b"fe80::1.", b"::ffff:1.2.3.4.", b"abc.def.",
           b"\xc3\xa9t\xc3\xa9.com.", b"\xff.", b"a.b.c.d.e.f.g.h.i.j.", b"dead.beef."]
    mixed = [odd[int(k)] if rng.random() < 0.1 else plain[i]
             for i, k in enumerate(rng.integers(0, len(odd), 3000))]
    wants = []
    for names in (plain, mixed):
        wants.append(clf.dns_classify(names))
    devs = []
    for names in (plain, mixed):
        blob, off, _ = pack_strings(names)
        devs.append((torch.from_numpy(blob).cuda(), torch.from_numpy(off.astype(np.int32)).cuda()))
    sizes = [1, 65, 1025, 3000]
    streams = [torch.cuda.Stream(), torch.cuda.Stream()]
    outs = []
    for k in range(4300):
        n = sizes[k % len(sizes)]
        which = (k // len(sizes)) % 2
        s = streams[k % 2]
        qb, qo = devs[which]
        with torch.cuda.stream(s):
            kd = torch.empty(n, dtype=torch.uint8, device="cuda")
            vl = torch.empty(n, dtype=torch.int32, device="cuda")
            V.check(V.lib().vc_dns_classify_dev(
                clf.h, C.c_void_p(qb.data_ptr()), C.c_void_p(qo.data_ptr()), n,
                C.c_void_p(kd.data_ptr()), C.c_void_p(vl.data_ptr()), C.c_void_p(s.cuda_stream)))
        if k % 300 < 8 or k >= 4292:
            outs.append((n, which, kd, vl))
    torch.cuda.synchronize()
    for n, which, kd, vl in outs:
        np.testing.assert_array_equal(kd.cpu().numpy(), wants[which][0][:n])
        np.testing.assert_array_equal(vl.cpu().numpy(), wants[which][1][:n])


def test_hint_c4_scale(clf):
    """C4: 100k hint-host groups (5 % with a hint-port) vs 1M hostnames with
    hint ports on 20 %: every result equal to exact.HintChecker, plus an
    oracle sample (each oracle query scans all 100k groups)."""
    groups, ghosts = W.gen_groups(100000, W.SEED + 5)
    clf.compile_upstream(groups)
    names = W.gen_hostnames(ghosts, 1 << 20, W.SEED + 6, pool=1 << 18)
    rng = np.random.default_rng(3)
    ports = np.where(rng.random(len(names)) < 0.2, rng.integers(1, 65536, len(names)), 0)
    ports = ports.astype(np.uint16)
    clf.counters_enable(True)
    clf.counters_reset()
    got = clf.hint_search(names, ports)
    cg = clf.counters_read(V.COUNTERS_GROUP)
    exp = np.bincount(np.where(got >= 0, got, len(groups)), minlength=len(groups) + 1)
    np.testing.assert_array_equal(cg, exp.astype(np.uint64))
    clf.counters_enable(False)
    # every name, hint-port filter included (Hint.java:124-128): exact.HintChecker
    blob, off = W.pack(names)
    np.testing.assert_array_equal(got, HintChecker(groups).batch(blob, off, ports))
    og = O.Groups(groups)
    s = rng.integers(0, len(names), 500)
    want = [O.search_for_group(og, names[i], int(ports[i]), None) for i in s]
    np.testing.assert_array_equal(got[s], np.array(want, np.int32))
    assert (got >= 0).mean() > 0.5
    assert (ports > 0).mean() > 0.15


def test_hint_uri_levels_at_scale(clf):
    """R9 at scale with hint-uris: 100k C4 groups, a fifth with a hint-uri
    (paths, prefixes of each other, '*'), 200 uri-only groups, 5 % with a
    hint-port; 500k hostnames with ports on 20 % and uris on 80 % (formatUri
    cases: '?', trailing '/').  Every result equal to exact.HintLevelChecker
    (the whole Hint.matchLevel, Hint.java:100-160, and searchForGroup's
    strict '>', Upstream.java:187-198), plus an oracle sample."""
    from exact import HintLevelChecker
    groups, ghosts = W.gen_groups(100000, W.SEED + 5)
    paths = ["/", "/api", "/api/v1", "/api/v1/users", "/api/v2", "/static", "/static/img",
             "/static/img/a.png", "*", "/login", "/a/b/c/d/e/f"]
    rng = np.random.default_rng(81)
    for i in np.nonzero(rng.random(len(groups)) < 0.2)[0]:
        groups[i][1]["uri"] = paths[int(rng.integers(0, len(paths)))]
    groups += [({}, {"uri": paths[k % len(paths)] + ("/u%d" % k if k > len(paths) else "")})
               for k in range(200)]
    clf.compile_upstream(groups)
    names = W.gen_hostnames(ghosts, 500_000, W.SEED + 6, pool=1 << 18)
    ports = np.where(rng.random(len(names)) < 0.2, rng.integers(1, 65536, len(names)), 0)
    ports = ports.astype(np.uint16)
    tails = ["", "/", "/x", "?q=1", "/?q=2", "/users/7"]
    uris = [None if rng.random() < 0.2 else
            (paths[int(rng.integers(0, len(paths)))] + tails[int(rng.integers(0, len(tails)))])
            for _ in range(len(names))]
    got = clf.hint_search([n.decode() for n in names], ports, uris)
    og = O.Groups(groups)
    chk = HintLevelChecker(groups)
    enc = lambda x: None if x is None else x.encode()
    want = np.array([chk(n, int(p), enc(u)) for n, p, u in zip(names, ports, uris)], np.int32)
    np.testing.assert_array_equal(got, want)
    s = rng.integers(0, len(names), 300)
    np.testing.assert_array_equal(got[s], [O.search_for_group(og, names[i], int(ports[i]), uris[i])
                                           for i in s])
    assert (got >= 0).mean() > 0.5 and len(np.unique(got)) > 10000


def test_hint_shapes(clf):
    """Fast-path shapes (lengths mod 4, > 6 labels, waves whose names
    overflow the LDS stage, ':port' / 'www.' / IPv6 forms) vs the oracle,
    from the host entry point and from an unaligned device blob."""
    import torch
    from cases import hint_cases_shapes
    groups, names = hint_cases_shapes(np.random.default_rng(93), 40000)
    clf.compile_upstream(groups)
    ports = np.random.default_rng(94).choice(np.array([0, 0, 80, 8080], np.uint16), len(names))
    og = O.Groups(groups)
    blob, off = W.pack(names)
    want = O.hint_batch_np(og, blob, off, ports, nthreads=THREADS)
    np.testing.assert_array_equal(clf.hint_search(names, ports), want)
    # device blob at an odd address: the launcher's unstaged kernel
    raw = torch.zeros(len(blob) + 1, dtype=torch.uint8, device="cuda")
    raw[1:] = torch.from_numpy(blob.astype(np.uint8)).cuda()
    o = torch.from_numpy(off.astype(np.int32)).cuda()
    got = clf.hint_search((raw[1:], o, None), torch.from_numpy(ports.astype(np.int16)).cuda())
    torch.cuda.synchronize()
    np.testing.assert_array_equal(got.cpu().numpy(), want)


def test_dns_kats_and_random(clf):
    with open(os.path.join(G, "kats.json")) as f:
        kats = json.load(f)
    for case in kats["dns"]:
        clf.compile_upstream(case["groups"])
        clf.compile_hosts([tuple(x) for x in case["hosts"]])
        kind, val = clf.dns_classify([q for q, _, _ in case["queries"]])
        assert [(int(k), int(v)) for k, v in zip(kind, val)] == \
            [(k, v) for _, k, v in case["queries"]], case["source"]
    # qnames as wire bytes: (char) b sign-extends (U+FF80..) vs UTF-8 annotations (Formatter.java:225-257)
    for case in kats["dns_wire"]:
        clf.compile_upstream(case["groups"])
        clf.compile_hosts([tuple(x) for x in case["hosts"]])
        kind, val = clf.dns_classify([bytes.fromhex(q) for q, _, _ in case["queries"]])
        assert [(int(k), int(v)) for k, v in zip(kind, val)] == \
            [(k, v) for _, k, v in case["queries"]], case["source"]
    groups, ghosts = W.gen_groups(3000, 77)
    clf.compile_upstream(groups)
    pairs = [(h + ".", i) for i, h in enumerate(ghosts[:50])] + [("localhost.", 999)]
    clf.compile_hosts(pairs)
    names = W.gen_hostnames(ghosts, 30000, 78, dns=True)
    names += [b"1.2.3.4.", b"::1.", b"[::1].", b"a.vproxy.local.", b".", b"", b"::ffff:1.2.3.4.",
              b"::x:1.2.3.4.", b"www.x.com:80."]
    kind, val = clf.dns_classify(names)
    og = O.Groups(groups)
    oh = O.Hosts(pairs)
    want = [O.dns_classify(oh, og, q) for q in names]
    assert [(int(k), int(v)) for k, v in zip(kind, val)] == want


def test_hosts_text(clf):
    clf.compile_upstream([({}, {"host": "example.com"})])
    text = "127.0.0.1 localhost\n10.0.0.1 db.example.com. db # x\n::1 localhost ip6\n"
    clf.compile_hosts_text(text)
    pairs, _ = O.hosts_parse(text)
    kind, val = clf.dns_classify(["localhost.", "db.example.com.", "db.", "ip6.", "example.com."])
    oh = O.Hosts(pairs)
    og = O.Groups([({}, {"host": "example.com"})])
    want = [O.dns_classify(oh, og, q) for q in
            ["localhost.", "db.example.com.", "db.", "ip6.", "example.com."]]
    assert [(int(k), int(v)) for k, v in zip(kind, val)] == want


# ---------------------------------------------------------------------------
# Pipeline + counters
# ---------------------------------------------------------------------------
def test_pipeline_and_counters(clf):
    import torch
    tcp, udp = W.gen_sg_rules(1000, 51)
    compile_acl_np(clf, tcp, udp, False)
    net, plen = W.gen_v4_prefixes(20000, 52)
    nets = W.v4_nets(net, plen)
    a, na, ka = W.as_ctypes(nets, V._lib.VcNet)
    clf.compile_routes_raw(a, na, (V._lib.VcNet * 1)(), 0)
    groups, ghosts = W.gen_groups(5000, 53)
    clf.compile_upstream(groups)
    names = W.gen_hostnames(ghosts, 20000, 54)
    pool = clf.hint_search(names)
    n = 1000003
    proto, src, port = W.gen_acl_queries(tcp, udp, n, 55)
    dst = W.v4_lookups(net, plen, n, 56)
    hid = np.random.default_rng(57).integers(0, len(names), n).astype(np.uint32)
    hid[::97] = 0xFFFFFFFF
    clf.counters_enable(True)
    clf.counters_reset()
    T = lambda x: torch.from_numpy(x).cuda()
    out = clf.pipeline_v4(T(proto), T(src), T(dst), T(port), T(hid), T(pool), want_allow=True)
    torch.cuda.synchronize()
    acl, route, grp, allow = (o.cpu().numpy() for o in out)
    want_acl, want_allow = O.sg_batch_v4_np(tcp, udp, False, proto, src, port, nthreads=THREADS)
    np.testing.assert_array_equal(acl, want_acl)
    np.testing.assert_array_equal(allow, want_allow)
    s = np.random.default_rng(58).integers(0, n, 20000)
    np.testing.assert_array_equal(route[s], O.rt_batch_v4_np(nets, dst[s], nthreads=THREADS))
    np.testing.assert_array_equal(grp, np.where(hid == 0xFFFFFFFF, -1, pool[np.minimum(
        hid, len(pool) - 1)]))
    # counters: exact histograms of the outputs
    ca = clf.counters_read(V.COUNTERS_ACL)
    nt, nu = len(tcp), len(udp)
    exp = np.zeros(nt + nu + 2, np.uint64)
    is_t = proto == 6
    np.add.at(exp, np.where(acl >= 0, np.where(is_t, acl, nt + acl), nt + nu + (~is_t)), 1)
    np.testing.assert_array_equal(ca, exp)
    cr = clf.counters_read(V.COUNTERS_ROUTE)
    exp = np.bincount(np.where(route >= 0, route, len(nets)), minlength=len(nets) + 2)
    np.testing.assert_array_equal(cr, exp.astype(np.uint64))
    cg = clf.counters_read(V.COUNTERS_GROUP)
    assert int(cg.sum()) == n
    clf.counters_enable(False)


def test_hosts_text_kats_on_gpu(clf):
    """kats.json hosts_text: an /etc/hosts text through vc_compile_hosts_text
    (Resolver.getHosts: first line wins, x and x. keys, comments and non-IP
    lines skipped) and vc_dns_classify -- TestResolver.resolve's localhost
    is the 127.0.0.1 line."""
    with open(os.path.join(G, "kats.json")) as f:
        kats = json.load(f)
    for case in kats["hosts_text"]:
        clf.compile_upstream(case["groups"])
        clf.compile_hosts_text(case["text"])
        kind, value = clf.dns_classify([q for q, _, _ in case["queries"]])
        assert list(zip(kind.tolist(), value.tolist())) == \
            [(k, v) for _, k, v in case["queries"]], case["source"]


def test_hosts_with_ipv6_literals_at_scale(clf):
    """formatHost's IPv6 branch (Hint.java:57-73: an IPv6 string is the host
    as it is, any other name with a ':' is cut at the first one) and the DNS
    IP-literal step (DNSServer.java:116-166), item by item over 400k names --
    generated hostnames, IPv6 / IPv4 literals and near misses
    (cases.ip_like_strings), bracketed, with ports -- against
    exact.HintChecker and exact.DnsChecker, whose IP predicates restate
    IP.java (checked against the oracle on the CPU tier)."""
    from cases import ip_like_strings
    from exact import DnsChecker, HintChecker
    rng = np.random.default_rng(47)
    groups, ghosts = W.gen_groups(5000, 48, port_frac=0.2)
    groups = [g for g in groups if g[1].get("host") != "*"]    # so misses reach the literal step
    lits = [b"::1", b"2001:db8::1", b"fe80::1", b"::ffff:1.2.3.4", b"[::1]", b"a::b",
            b"1:2:3:4:5:6:7:8", b"10.1.2.3"]
    groups += [({}, {"host": h.decode()}) for h in lits]
    clf.compile_upstream(groups)
    names = W.gen_hostnames(ghosts, 200_000, 49, port_frac=0.2)
    names += ip_like_strings(rng, 200_000)
    names += lits + [x + b":80" for x in lits] + [b"[" + x + b"]:443" for x in lits]
    ports = rng.choice(np.array([0, 0, 80, 443, 8080], np.uint16), len(names))
    chk = HintChecker(groups)
    blob, off = W.pack(names)
    for p in (None, ports):
        got = clf.hint_search(names, p)
        want = chk.batch(blob, off, p)
        np.testing.assert_array_equal(got, want)
    lit_groups = set(range(len(groups) - len(lits), len(groups)))
    assert len(lit_groups & set(want.tolist())) >= 5
    # the DNS classification of the same names (as qnames, half with the
    # trailing dot), over a hosts file with IPv6 and IPv4 entries
    text = "::1 six.hosts.local\n10.0.0.1 four.hosts.local\n2001:db8::2 v6.hosts.local.\n"
    clf.compile_hosts_text(text)
    qn = [x + b"." if i % 2 else x for i, x in enumerate(names)]
    qn += [b"six.hosts.local", b"v6.hosts.local", b"four.hosts.local."]
    kind, val = clf.dns_classify(qn)
    wk, wv = DnsChecker(text, groups).batch(*W.pack(qn))
    np.testing.assert_array_equal(kind, wk)
    np.testing.assert_array_equal(val, wv)
    assert {V.DNS_HOSTS, V.DNS_GROUP, V.DNS_IP_LITERAL} <= set(np.unique(kind).tolist())

"""GPU tier: the general pipeline entry points vc_pipeline_dev / vc_pipeline.

IPv4 and IPv6 packets in one batch, as the vswitch drain loop hands them
to L3.route (core/src/main/java/vswitch/Switch.java:744-776,
core/src/main/java/vswitch/stack/L3.java:423-444): each packet's family is
the `instanceof IPv4` dispatch of RouteTable.lookup
(core/src/main/java/vswitch/RouteTable.java:44-58), so IPv4-mapped
(::ffff:a.b.c.d) and IPv4-compatible (::a.b.c.d) addresses are IPv6 packets:
they go to rulesV6 and to the v6 projection of the SecurityGroup rules
(Network.maskMatch's cross-family cases, Network.java:183-278).  Every
output is compared with the oracle's per-family restatements; hit counters
with exact histograms; the host entry point (chunked staging and zero-copy
over registered buffers) with the device entry point.
"""
import os

import numpy as np
import pytest

import oracle_ffi as O
import vproxy_amd as V
from vproxy_amd import workloads as W

from cases import acl_edge_rules, v6_edge_inputs

pytestmark = pytest.mark.gpu
THREADS = min(16, os.cpu_count() or 1)


def _nets(specs):
    return np.concatenate([np.frombuffer(bytes(O.net(s)), W.NET_DT) for s in specs])


def _tables(clf, seed):
    rng = np.random.default_rng(seed)
    tcp_r, udp_r = W.gen_sg_rules(1500, seed, p_range=0.4)
    etcp, eudp = acl_edge_rules()
    tcp, udp = np.concatenate([tcp_r, etcp]), np.concatenate([udp_r, eudp])
    a, na, ka = W.as_ctypes(tcp, V._lib.VcAclRule)
    b, nb, kb = W.as_ctypes(udp, V._lib.VcAclRule)
    V.check(V.lib().vc_compile_acl(clf.h, a, na, b, nb, 0))
    net, plen = W.gen_v4_prefixes(20000, seed + 1)
    nets4 = W.v4_nets(net, plen)
    rng.shuffle(nets4)                          # arbitrary list order = priority
    hi, lo, p6 = W.gen_v6_prefixes(5000, seed + 2)
    nets6 = np.concatenate([
        W.v6_nets(hi, lo, p6),
        _nets(["::ffff:0.0.0.0/96", "::ffff:10.0.0.0/104", "::/96", "::ffff:8.8.8.0/120",
               "::/0", "2001:db8::/32"])])
    rng.shuffle(nets6)
    ra, rn, rk = W.as_ctypes(nets4, V._lib.VcNet)
    rb, rbn, rbk = W.as_ctypes(nets6, V._lib.VcNet)
    clf.compile_routes_raw(ra, rn, rb, rbn)
    groups, ghosts = W.gen_groups(3000, seed + 3)
    clf.compile_upstream(groups)
    names = W.gen_hostnames(ghosts, 5000, seed + 4)
    pool = clf.hint_search(names)
    return dict(tcp=tcp, udp=udp, net=net, plen=plen, nets4=nets4, nets6=nets6, hi=hi, lo=lo,
                p6=p6, pool=pool, groups=groups, names=names)


def _packets(t, n, seed):
    """n packets, half IPv6; the IPv6 half mixes native destinations with
    IPv4-mapped / IPv4-compatible forms of addresses inside the v4 routes."""
    rng = np.random.default_rng(seed)
    fam = np.where(rng.random(n) < 0.5, 4, 6).astype(np.uint8)
    proto, src4, dport = W.gen_acl_queries(t["tcp"], t["udp"], n, seed + 1)
    dst4 = W.v4_lookups(t["net"], t["plen"], n, seed + 2)
    src6, p6, port6 = v6_edge_inputs(rng, n)
    dst6 = W.v6_lookups(t["hi"], t["lo"], t["p6"], n, seed + 3)
    k = rng.integers(0, 4, n)
    v4b = W.v4_to_bytes(dst4)
    dst6[k == 1, :10] = 0
    dst6[k == 1, 10:12] = 0xFF
    dst6[k == 1, 12:] = v4b[k == 1]
    dst6[k == 2, :12] = 0
    dst6[k == 2, 12:] = v4b[k == 2]
    six = fam == 6
    proto = np.where(six, p6, proto).astype(np.uint8)
    dport = np.where(six, port6, dport).astype(np.uint16)
    hid = rng.integers(0, len(t["pool"]), n).astype(np.uint32)
    hid[::89] = 0xFFFFFFFF
    return dict(family=fam, proto=proto, src4=src4, dst4=dst4, src6=src6, dst6=dst6,
                dport=dport, host_id=hid)


def _oracle(t, p):
    fam = p["family"]
    n = len(fam)
    acl = np.empty(n, np.int32)
    allow = np.empty(n, np.uint8)
    route = np.empty(n, np.int32)
    for f, sel in ((4, fam != 6), (6, fam == 6)):
        if f == 4:
            a, v = O.sg_batch_v4_np(t["tcp"], t["udp"], False, p["proto"][sel], p["src4"][sel],
                                    p["dport"][sel], nthreads=THREADS)
            r = O.rt_batch_v4_np(t["nets4"], p["dst4"][sel], nthreads=THREADS)
        else:
            a, v = O.sg_batch_v6_np(t["tcp"], t["udp"], False, p["proto"][sel], p["src6"][sel],
                                    p["dport"][sel], nthreads=THREADS)
            r = O.rt_batch_v6_np(t["nets6"], p["dst6"][sel], nthreads=THREADS)
        acl[sel], allow[sel], route[sel] = a, v, r
    h = p["host_id"]
    grp = np.where(h < len(t["pool"]), t["pool"][np.minimum(h, len(t["pool"]) - 1)], -1)
    return acl, route, grp.astype(np.int32), allow


def _dev(p, offset=0):
    import torch
    out = {}
    for k, v in p.items():
        raw = torch.from_numpy(np.ascontiguousarray(v)).cuda()
        if offset and k not in ("src6", "dst6"):
            # shift by one element (the 16-byte v6 arrays must stay aligned)
            buf = torch.empty(len(v) + 1, dtype=raw.dtype, device="cuda")
            buf[1:] = raw
            raw = buf[1:]
        out[k] = raw
    return out


def _call(clf, d, pool, want_allow=True, family=True, hosts=True):
    return clf.pipeline(d["proto"], d["src4"], d["dst4"], d["dport"],
                        d["host_id"] if hosts else None, pool if hosts else None,
                        family=d["family"] if family else None,
                        src6=d["src6"] if family else None, dst6=d["dst6"] if family else None,
                        want_allow=want_allow)


@pytest.fixture(scope="module")
def setup():
    clf = V.Classifier(0)
    t = _tables(clf, 301)
    yield clf, t
    clf.close()


@pytest.mark.parametrize("offset", [0, 1])
def test_mixed_pipeline_vs_oracle(setup, offset):
    import torch
    clf, t = setup
    n = 200_003
    p = _packets(t, n, 7 + offset)
    want = _oracle(t, p)
    d = _dev(p, offset)
    pool = torch.from_numpy(t["pool"]).cuda()
    clf.counters_enable(True)
    clf.counters_reset()
    got = _call(clf, d, pool)
    torch.cuda.synchronize()
    clf.counters_enable(False)
    got = [x.cpu().numpy() for x in got]
    for g, w, name in zip(got, want, ("acl", "route", "group", "allow")):
        np.testing.assert_array_equal(g, w, err_msg=name)
    acl, route, grp, _ = want
    fam, proto = p["family"], p["proto"]
    nt, nu = len(t["tcp"]), len(t["udp"])
    is_t = proto == 6
    exp = np.zeros(nt + nu + 2, np.uint64)
    np.add.at(exp, np.where(acl >= 0, np.where(is_t, acl, nt + acl), nt + nu + (~is_t)), 1)
    np.testing.assert_array_equal(clf.counters_read(V.COUNTERS_ACL), exp)
    n4, n6 = len(t["nets4"]), len(t["nets6"])
    six = fam == 6
    rb = np.where(route >= 0, np.where(six, n4 + route, route), n4 + n6 + six)
    exp = np.bincount(rb, minlength=n4 + n6 + 2).astype(np.uint64)
    np.testing.assert_array_equal(clf.counters_read(V.COUNTERS_ROUTE), exp)
    ng = len(t["groups"])
    exp = np.bincount(np.where(grp >= 0, grp, ng), minlength=ng + 1).astype(np.uint64)
    np.testing.assert_array_equal(clf.counters_read(V.COUNTERS_GROUP), exp)
    # the mapped/compat v6 packets really exercised the v6 lists
    assert (route[six] >= 0).mean() > 0.3 and (route[~six] >= 0).mean() > 0.8


def test_pipeline_without_family_or_hosts(setup):
    """family NULL = every packet IPv4 (the v4 lists); host_id NULL = no
    hostname stage (group -1, group counters untouched)."""
    import torch
    clf, t = setup
    p = _packets(t, 50_001, 19)
    p4 = dict(p, family=np.full(len(p["family"]), 4, np.uint8))
    want = _oracle(t, p4)
    d = _dev(p)
    pool = torch.from_numpy(t["pool"]).cuda()
    clf.counters_enable(True)
    clf.counters_reset()
    acl, route, grp, allow = _call(clf, d, pool, family=False, hosts=False)
    torch.cuda.synchronize()
    clf.counters_enable(False)
    np.testing.assert_array_equal(acl.cpu().numpy(), want[0])
    np.testing.assert_array_equal(route.cpu().numpy(), want[1])
    np.testing.assert_array_equal(allow.cpu().numpy(), want[3])
    assert bool((grp == -1).all())
    assert int(clf.counters_read(V.COUNTERS_GROUP).sum()) == 0
    acl2, route2, grp2, _ = _call(clf, d, pool, family=False, hosts=True)
    np.testing.assert_array_equal(acl2.cpu().numpy(), want[0])
    np.testing.assert_array_equal(route2.cpu().numpy(), want[1])
    np.testing.assert_array_equal(grp2.cpu().numpy(), want[2])


def host_entry_point_equals_device(clf, t, registered):
    """vc_pipeline over host arrays: pageable (chunked staging, 3 chunks) or
    registered (zero-copy) give the device entry point's outputs."""
    import torch
    n = (9 << 20) + 5
    p = _packets(t, n, 23)
    pool = np.array(t["pool"], np.int32)          # an array of its own (it may be registered)
    d = _dev(p)
    ref = [x.cpu().numpy() for x in _call(clf, d, torch.from_numpy(pool).cuda())]
    outs = (np.empty(n, np.int32), np.empty(n, np.int32), np.empty(n, np.int32),
            np.empty(n, np.uint8))
    bufs = list(p.values()) + [pool] + list(outs)
    if registered:
        for x in bufs:
            V.check(V.lib().vc_host_register(x.ctypes.data, x.nbytes))
    try:
        got = clf.pipeline(p["proto"], p["src4"], p["dst4"], p["dport"], p["host_id"], pool,
                           family=p["family"], src6=p["src6"], dst6=p["dst6"], outs=outs)
    finally:
        if registered:
            for x in bufs:
                V.check(V.lib().vc_host_unregister(x.ctypes.data))
    for g, r in zip(got, ref):
        np.testing.assert_array_equal(g, r)


def test_host_entry_point_equals_device(setup):
    host_entry_point_equals_device(*setup, registered=False)


def test_bad_arguments(setup):
    clf, t = setup
    p = _packets(t, 8, 29)
    with pytest.raises(V.IllegalArgumentException):
        clf.pipeline(p["proto"], p["src4"], p["dst4"], p["dport"], family=p["family"])
    with pytest.raises(V.IllegalArgumentException):
        clf.pipeline(p["proto"], None, p["dst4"], p["dport"])


def _compact(d):
    six = d["family"] == 6
    return d["src6"][six].contiguous(), d["dst6"][six].contiguous()


@pytest.mark.parametrize("n,frac", [(1, 1.0), (3, 0.5), (4, 0.5), (5, 1.0), (257, 0.5),
                                    (4099, 0.0), (4099, 1.0), (200_003, 0.5), (1 << 20, 0.15)])
def test_compact6_rows_vs_oracle(setup, n, frac):
    """vc_pipeline_c6_dev: src6 / dst6 with one row per IPv6 packet (packet
    order) give every output the oracle gives the sparse batch, and the same
    hit counters -- at sizes with partial groups of four, no IPv6 packet,
    only IPv6 packets, and several workgroups' wave shares."""
    import torch
    clf, t = setup
    p = _packets(t, n, 41 + n)
    rng = np.random.default_rng(n)
    p["family"] = np.where(rng.random(n) < frac, 6, 4).astype(np.uint8)
    want = _oracle(t, p)
    d = _dev(p)
    pool = torch.from_numpy(t["pool"]).cuda()
    s6, d6 = _compact(d)
    clf.counters_enable(True)
    clf.counters_reset()
    got = clf.pipeline(d["proto"], d["src4"], d["dst4"], d["dport"], d["host_id"], pool,
                       family=d["family"], src6=s6, dst6=d6, want_allow=True, compact6=True)
    torch.cuda.synchronize()
    clf.counters_enable(False)
    cnt = [clf.counters_read(k) for k in (V.COUNTERS_ACL, V.COUNTERS_ROUTE, V.COUNTERS_GROUP)]
    for g, w, name in zip(got, want, ("acl", "route", "group", "allow")):
        np.testing.assert_array_equal(g.cpu().numpy(), w, err_msg=name)
    clf.counters_reset()
    clf.counters_enable(True)
    _call(clf, d, pool)                              # the sparse form, same counters
    torch.cuda.synchronize()
    clf.counters_enable(False)
    for k, c in zip((V.COUNTERS_ACL, V.COUNTERS_ROUTE, V.COUNTERS_GROUP), cnt):
        np.testing.assert_array_equal(clf.counters_read(k), c)


def test_compact6_short_rows_and_alignment(setup):
    """Fewer rows than IPv6 packets never reads outside the rows (the packets
    past them get unspecified results; the ones before are exact), no rows at
    all reads nothing; misaligned fields are refused."""
    import torch
    clf, t = setup
    n = 50_001
    p = _packets(t, n, 53)
    want = _oracle(t, p)
    d = _dev(p)
    pool = torch.from_numpy(t["pool"]).cuda()
    s6, d6 = _compact(d)
    k = len(s6) // 2
    got = clf.pipeline(d["proto"], d["src4"], d["dst4"], d["dport"], d["host_id"], pool,
                       family=d["family"], src6=s6[:k], dst6=d6[:k], compact6=True)
    torch.cuda.synchronize()
    first = np.nonzero(p["family"] == 6)[0][k - 1] + 1     # packets before the k-th IPv6 one
    for g, w in zip(got[:3], want[:3]):
        np.testing.assert_array_equal(g.cpu().numpy()[:first], w[:first])
    e6 = s6[:0]
    got = clf.pipeline(d["proto"], d["src4"], d["dst4"], d["dport"], d["host_id"], pool,
                       family=d["family"], src6=e6, dst6=e6, compact6=True)
    torch.cuda.synchronize()
    v4 = p["family"] == 4
    np.testing.assert_array_equal(got[1].cpu().numpy()[v4], want[1][v4])
    dm = _dev(p, offset=1)
    with pytest.raises(V.IllegalArgumentException):
        clf.pipeline(dm["proto"], dm["src4"], dm["dst4"], dm["dport"], dm["host_id"], pool,
                     family=dm["family"], src6=s6, dst6=d6, compact6=True)


@pytest.mark.parametrize("registered", [False, True])
def test_compact6_host_entry(setup, registered):
    """vc_pipeline_c6 over host arrays, pageable (chunked staging: each
    4M-packet chunk's rows found by counting its IPv6 packets; the second
    chunk has none) or registered (zero-copy, the rows read coalesced), gives
    the device entry point's outputs for the sparse batch; a row count that
    disagrees with the family array is refused on the staged path."""
    import torch
    clf, t = setup
    n = (9 << 20) + 5
    p = _packets(t, n, 61)
    rng = np.random.default_rng(61)
    p["family"] = np.where(rng.random(n) < 0.15, 6, 4).astype(np.uint8)
    p["family"][4 << 20:8 << 20] = 4
    pool = np.array(t["pool"], np.int32)
    ref = [x.cpu().numpy() for x in _call(clf, _dev(p), torch.from_numpy(pool).cuda())]
    six = p["family"] == 6
    s6, d6 = np.ascontiguousarray(p["src6"][six]), np.ascontiguousarray(p["dst6"][six])
    outs = (np.empty(n, np.int32), np.empty(n, np.int32), np.empty(n, np.int32),
            np.empty(n, np.uint8))
    bufs = [p[k] for k in ("family", "proto", "src4", "dst4", "dport", "host_id")] + [
        s6, d6, pool] + list(outs)
    if registered:
        for x in bufs:
            V.check(V.lib().vc_host_register(x.ctypes.data, x.nbytes))
    try:
        got = clf.pipeline(p["proto"], p["src4"], p["dst4"], p["dport"], p["host_id"], pool,
                           family=p["family"], src6=s6, dst6=d6, outs=outs, compact6=True)
    finally:
        if registered:
            for x in bufs:
                V.check(V.lib().vc_host_unregister(x.ctypes.data))
    for g, r, name in zip(got, ref, ("acl", "route", "group", "allow")):
        np.testing.assert_array_equal(g, r, err_msg=name)
    # a row count that disagrees with the family array is refused before any
    # output is written, on the staged and the zero-copy path alike
    for k in (len(s6) - 1, len(s6) + 1):
        rows = np.zeros((k, 16), np.uint8)
        mark = [np.full(n, -7, np.int32) for _ in range(3)] + [np.full(n, 9, np.uint8)]
        regs = [rows] + [p[k2] for k2 in ("family", "proto", "src4", "dst4", "dport",
                                           "host_id")] + [pool] + mark
        if registered:
            for x in regs:
                V.check(V.lib().vc_host_register(x.ctypes.data, x.nbytes))
        try:
            with pytest.raises(V.IllegalArgumentException):
                clf.pipeline(p["proto"], p["src4"], p["dst4"], p["dport"], p["host_id"], pool,
                             family=p["family"], src6=rows, dst6=rows, outs=tuple(mark),
                             compact6=True)
        finally:
            if registered:
                for x in regs:
                    V.check(V.lib().vc_host_unregister(x.ctypes.data))
        assert all((m == m.flat[0]).all() for m in mark), "outputs written before the refusal"


def test_compact6_host_entry_small(setup):
    """vc_pipeline_c6 at sizes below one chunk: no IPv6 packet (no rows),
    only IPv6 packets, a partial group of four."""
    clf, t = setup
    for n, frac in ((1, 0.0), (1, 1.0), (7, 0.5), (4099, 0.0), (4099, 1.0)):
        p = _packets(t, n, 67 + n)
        rng = np.random.default_rng(n)
        p["family"] = np.where(rng.random(n) < frac, 6, 4).astype(np.uint8)
        want = _oracle(t, p)
        six = p["family"] == 6
        s6, d6 = np.ascontiguousarray(p["src6"][six]), np.ascontiguousarray(p["dst6"][six])
        got = clf.pipeline(p["proto"], p["src4"], p["dst4"], p["dport"], p["host_id"],
                           t["pool"], family=p["family"], src6=s6, dst6=d6, want_allow=True,
                           compact6=True)
        for g, w, name in zip(got, want, ("acl", "route", "group", "allow")):
            np.testing.assert_array_equal(g, w, err_msg="%s n=%d frac=%s" % (name, n, frac))

"""GPU tier: the headline C5 configuration exactly as bench.py runs it.

The tables are built by bench.c5_tables (10k ACL rules, 980,848 + 200,000
routes shortest-first, 100k groups, a 16M-name pool) and the packets by
bench.gen_packets (the sharded global batch's generator).  The fused
pipeline runs with the in-kernel hit counters on, over 16M device-resident
packets, once from aligned arrays (the vector kernel) and once offset by
one packet (the one-packet-per-lane kernel).  Checks: oracle samples of the
ACL (SecurityGroup.java:30-45), route (RouteTable.java:44-59) and pool
group (Upstream.java:187-198) results; whole-batch properties; and counters
equal to exact histograms of the outputs.

Every output of every batch is compared exactly: tests/exact.py restates
SecurityGroup.allow, RouteTable.lookup and Upstream.searchForGroup with
per-prefix-length sorted keys and a hint-host dict (validated against the
oracle in tests/test_exact_cpu.py), fast enough for all 16M packets and the
whole 16M-name pool.  Oracle samples stay beside them as a second witness.

Also here: DNS at C4 scale (100k groups + 50k hosts), counters fed values
outside the counter space, and the bench's N > 1 schedule (HitCounterBucket
fill from the library's device counters on the counting stream + an RCCL
all-reduce) run as a world-size-1 process group on one GPU.
"""
import os
import socket

import numpy as np
import pytest

import bench as B
import oracle_ffi as O
import vproxy_amd as V
from exact import AclChecker, DnsChecker, HintChecker, RouteChecker
from vproxy_amd import workloads as W

pytestmark = pytest.mark.gpu
THREADS = min(16, os.cpu_count() or 1)


@pytest.fixture(scope="module")
def c5():
    import torch
    clf = V.Classifier(0)
    dev = torch.device("cuda", 0)
    t = B.c5_tables(clf, dev, 16 << 20)
    t.acl_chk = AclChecker(t.tcp, t.udp, False, dev)
    t.rt4_chk = RouteChecker(t.v4_list, 4, dev)
    t.rt6_chk = RouteChecker(t.v6_list, 6, dev)
    # the pool is 16M draws (t.pidx) from 1M distinct names: classify those
    # with the dict checker once, then index
    t.name_want = torch.from_numpy(HintChecker(t.groups).batch(t.nblob, t.noff)).to(dev)
    t.pool_want = t.name_want[torch.from_numpy(t.pidx).to(dev)]
    yield clf, t, dev
    clf.close()


def _rule_arrays(rules, dev):
    import torch
    ip, mk = W.rule_v4_fields(rules)
    T = lambda x: torch.from_numpy(np.asarray(x).astype(np.int64)).to(dev)
    return T(ip), T(mk), T(rules["min_port"]), T(rules["max_port"]), T(rules["allow"])


def _check_batch(clf, t, dev, pkts, outs, pool, check_counters=True):
    """Oracle samples + whole-batch properties + exact counters of one
    pipeline call whose outputs are `outs`."""
    import torch
    proto, src, dst, dport, hid = pkts
    acl, route, grp, allow = outs
    n = len(src)
    u32 = lambda x: x.to(torch.int64) & 0xFFFFFFFF
    # group = pool[host_id] and the pool = searchForGroup of each name, whole batch
    assert torch.equal(grp, pool[hid.long()])
    assert torch.equal(pool, t.pool_want)
    # every ACL index / verdict and every route index, whole batch
    want_acl, want_allow = t.acl_chk.v4(proto, src, dport)
    assert torch.equal(acl, want_acl), int((acl != want_acl).sum())
    assert torch.equal(allow, want_allow)
    want_route = t.rt4_chk(dst)
    assert torch.equal(route, want_route), int((route != want_route).sum())
    # whole-batch ACL properties: the index names a rule of the packet's
    # protocol that contains src and whose port range holds dport; allow is
    # that rule's bit (defaultAllow = false otherwise)
    s64, d64, p64 = u32(src), u32(dst), dport.to(torch.int64) & 0xFFFF
    is_tcp = proto == 6
    for lst, sel in ((t.tcp, is_tcp), (t.udp, ~is_tcp)):
        ip, mk, lo, hi, al = _rule_arrays(lst, dev)
        a = acl[sel].long()
        assert bool((a < len(lst)).all())
        h = a >= 0
        r = a[h]
        assert bool(((s64[sel][h] & mk[r]) == ip[r]).all())
        pp = p64[sel][h]
        assert bool(((pp >= lo[r]) & (pp <= hi[r])).all())
        assert bool((allow[sel][h].long() == al[r]).all())
        assert bool((allow[sel][~h] == 0).all())
    # route: the rule's prefix contains dst; 90 % of dsts were drawn inside one
    rip = torch.from_numpy(t.v4_list["ip"][:, :4].copy().view(">u4").reshape(-1)
                           .astype(np.int64)).to(dev)
    rmk = torch.from_numpy(t.v4_list["mask"][:, :4].copy().view(">u4").reshape(-1)
                           .astype(np.int64)).to(dev)
    rr = route.long()
    h = rr >= 0
    assert bool(((d64[h] & rmk[rr[h]]) == rip[rr[h]]).all())
    assert float(h.float().mean()) > 0.85
    # oracle samples
    rng = np.random.default_rng(n)
    s = rng.integers(0, n, 20000)
    hs = lambda x: x.cpu().numpy()[s]
    want, wv = O.sg_batch_v4_np(t.tcp, t.udp, False, hs(proto), hs(src).view(np.uint32),
                                hs(dport).view(np.uint16), nthreads=THREADS)
    np.testing.assert_array_equal(hs(acl), want)
    np.testing.assert_array_equal(hs(allow), wv)
    s = s[:3000]
    np.testing.assert_array_equal(route.cpu().numpy()[s],
                                  O.rt_batch_v4_np(t.v4_list, dst.cpu().numpy()[s].view(np.uint32),
                                                   nthreads=THREADS))
    if not check_counters:
        return
    nt, nu = len(t.tcp), len(t.udp)
    a = acl.long()
    bins = torch.where(a >= 0, torch.where(is_tcp, a, nt + a),
                       torch.where(is_tcp, nt + nu, nt + nu + 1))
    exp = torch.bincount(bins, minlength=nt + nu + 2).cpu().numpy().astype(np.uint64)
    np.testing.assert_array_equal(clf.counters_read(V.COUNTERS_ACL), exp)
    nn = t.n4 + t.n6
    exp = torch.bincount(torch.where(rr >= 0, rr, nn), minlength=nn + 2).cpu().numpy()
    np.testing.assert_array_equal(clf.counters_read(V.COUNTERS_ROUTE), exp.astype(np.uint64))
    ng = len(t.groups)
    g = grp.long()
    exp = torch.bincount(torch.where(g >= 0, g, ng), minlength=ng + 1).cpu().numpy()
    np.testing.assert_array_equal(clf.counters_read(V.COUNTERS_GROUP), exp.astype(np.uint64))


def test_c5_bench_tables_and_pool(c5):
    """The bench's tables are the C5 sizes, and the classified pool equals
    searchForGroup for all 16M names (dict checker) and the oracle on a
    sample; the device pool blob holds exactly the drawn names' lengths."""
    import torch
    clf, t, dev = c5
    assert len(t.tcp) + len(t.udp) == 10000
    assert t.n4 == 980848 and t.n6 == 200000
    assert len(t.groups) == 100000 and t.pool_n == 16 << 20
    # the compiled snapshots' digests equal the host-only builds (what the
    # replica check of bench.py / dist.check_replicated compares across ranks)
    assert clf.table_digest(V.COUNTERS_ACL) == V.digest_acl(t.tcp, t.udp, False)
    assert clf.table_digest(V.COUNTERS_ROUTE) == V.digest_routes(t.v4_list.copy(), t.v6_list.copy())
    assert clf.table_digest(V.COUNTERS_GROUP) == V.digest_upstream(t.groups)
    pool = clf.hint_search((t.pool_blob, t.pool_off, None))
    torch.cuda.synchronize()
    lens = torch.from_numpy(np.diff(t.noff.astype(np.int64))[t.pidx]).to(dev)
    assert torch.equal(torch.diff(t.pool_off.long()), lens)
    assert torch.equal(pool, t.pool_want), int((pool != t.pool_want).sum())
    s = np.random.default_rng(9).integers(0, t.pool_n, 1500)
    names = [bytes(t.nblob[t.noff[i]:t.noff[i + 1]]) for i in t.pidx[s]]
    blob, off = W.pack(names)
    want = O.hint_batch_np(O.Groups(t.groups), blob, off, None, nthreads=THREADS)
    np.testing.assert_array_equal(pool.cpu().numpy()[s], want)
    assert (pool >= 0).float().mean() > 0.5


@pytest.mark.parametrize("offset", [0, 1])
def test_c5_pipeline_fused_counters(c5, offset):
    """16M packets of the bench's global batch through the fused pipeline
    with counters on: aligned (vector kernel) and offset by one (scalar)."""
    import torch
    clf, t, dev = c5
    pool = clf.hint_search((t.pool_blob, t.pool_off, None))
    n = 16 << 20
    pk = B.gen_packets(0, n + 1, t, t.pool_n, dev=dev)
    pk = tuple(x[offset:offset + n] for x in pk)
    if offset:
        assert pk[1].data_ptr() % 16 != 0
    torch.cuda.synchronize()
    clf.counters_enable(True)
    clf.counters_reset()
    outs = clf.pipeline_v4(*pk, pool, want_allow=True)
    torch.cuda.synchronize()
    clf.counters_enable(False)
    _check_batch(clf, t, dev, pk, outs, pool)


def test_c5_pipeline_count_stream(c5):
    """The counter finish on a separate stream (the bench schedule) gives
    the same counters."""
    import torch
    clf, t, dev = c5
    pool = clf.hint_search((t.pool_blob, t.pool_off, None))
    n = 8 << 20
    pk = B.gen_packets(5 << 20, n, t, t.pool_n, dev=dev)
    s_cnt = torch.cuda.Stream()
    torch.cuda.synchronize()
    clf.counters_enable(True)
    clf.counters_reset()
    outs = clf.pipeline_v4(*pk, pool, want_allow=True, count_stream=s_cnt)
    torch.cuda.synchronize()
    clf.counters_enable(False)
    _check_batch(clf, t, dev, pk, outs, pool)


def test_c5_timed_launch_exact(c5):
    """The launch the headline times, at its size: bench.main's C5 schedule
    (make_c5_steps with the default arguments: 125M packets per GPU, 3
    batches in flight, fused counters with the finish on the counting
    stream, the pool pass in order on the pipeline stream) run for 3 warmup
    + 2 timed steps over rank 0's shard.  Every ACL, route and group output
    of every in-flight buffer equal to the exact checkers
    (SecurityGroup.java:30-45, RouteTable.java:44-59, Upstream.java:187-198),
    every pool buffer equal to searchForGroup of all 16M names, and the
    counters equal to 5 x the per-step histograms."""
    import torch
    clf, t, dev = c5
    args = B.build_parser().parse_args([])
    assert args.packets == 125_000_000 and args.inflight == 3 and args.counters == "fused"
    lo, hi = B.shard(args.packets, 0, 1)
    pk = B.gen_packets(lo, hi - lo, t, t.pool_n, dev=dev)
    clf.counters_reset()
    steps = B.make_c5_steps(clf, t, pk, dev, args, bucket=False)
    nw, nk = 3, 2
    steps.run(0, nw, False)
    torch.cuda.synchronize()
    steps.reset_events()
    steps.run(nw, nk, True)
    torch.cuda.synchronize()
    assert steps.span("pipe") > 0
    last = (nw + nk - 1) % steps.nbuf
    acl, route, grp, _ = steps.outsb[last]
    assert acl.shape[0] == 125_000_000
    for pool in steps.pools:
        assert torch.equal(pool, t.pool_want)
    proto, src, dst, dport, hid = pk
    assert torch.equal(grp, t.pool_want[hid.long()])
    want_acl, _ = t.acl_chk.v4(proto, src, dport)
    assert torch.equal(acl, want_acl), int((acl != want_acl).sum())
    del want_acl
    want_route = t.rt4_chk(dst)
    assert torch.equal(route, want_route), int((route != want_route).sum())
    del want_route
    for b in range(steps.nbuf):                   # every buffer holds a full step
        if b != last:
            for x, y in zip(steps.outsb[b][:3], steps.outsb[last][:3]):
                assert torch.equal(x, y)
    steps_run = nw + nk
    nt, nu = len(t.tcp), len(t.udp)
    a = acl.long()
    is_tcp = proto == 6
    bins = torch.where(a >= 0, torch.where(is_tcp, a, nt + a),
                       torch.where(is_tcp, nt + nu, nt + nu + 1))
    exp = steps_run * torch.bincount(bins, minlength=nt + nu + 2)
    del a, bins
    np.testing.assert_array_equal(clf.counters_read(V.COUNTERS_ACL),
                                  exp.cpu().numpy().astype(np.uint64))
    nn = t.n4 + t.n6
    r = route.long()
    exp = steps_run * torch.bincount(torch.where(r >= 0, r, nn), minlength=nn + 2)
    del r
    np.testing.assert_array_equal(clf.counters_read(V.COUNTERS_ROUTE),
                                  exp.cpu().numpy().astype(np.uint64))
    ng = len(t.groups)
    g = grp.long()
    exp = steps_run * torch.bincount(torch.where(g >= 0, g, ng), minlength=ng + 1)
    np.testing.assert_array_equal(clf.counters_read(V.COUNTERS_GROUP),
                                  exp.cpu().numpy().astype(np.uint64))
    del steps, pk
    torch.cuda.empty_cache()


def test_mix_bench_batch_vs_oracle(c5):
    """The `mix` sub-bench exactly as bench.py runs it: 125M packets of
    bench.gen_mixed (15 % IPv6: IPv4-mapped and 2001:db8:: sources, 90 % of
    destinations inside a rulesV6 prefix) through vc_pipeline_dev on the C5
    tables, counter finish on a second stream.  Every ACL / verdict / route
    output equal to the exact checkers per family (the `instanceof IPv4`
    dispatch, RouteTable.java:44-58), oracle samples per family, group =
    pool[host_id] over the whole batch, exact route counters."""
    import torch
    clf, t, dev = c5
    pool = clf.hint_search((t.pool_blob, t.pool_off, None))
    n = B.build_parser().parse_args([]).packets          # the bench's 125M
    fam, proto, src, dst, src6, dst6, dport, hid = B.gen_mixed(0, n, t, t.pool_n, dev=dev)
    s_cnt = torch.cuda.Stream()
    torch.cuda.synchronize()
    clf.counters_enable(True)
    clf.counters_reset()
    acl, route, grp, allow = clf.pipeline(proto, src, dst, dport, hid, pool, family=fam,
                                          src6=src6, dst6=dst6, want_allow=True,
                                          count_stream=s_cnt)
    torch.cuda.synchronize()
    clf.counters_enable(False)
    assert torch.equal(grp, pool[hid.long()])
    assert torch.equal(pool, t.pool_want)
    # every packet, both families: the v4 rules see IPv6 sources through
    # Network.maskMatch's cross-family cases (exact.AclChecker.v6)
    is6 = fam == 6
    a4, w4 = t.acl_chk.v4(proto, src, dport)
    a6, w6 = t.acl_chk.v6(proto, src6, dport)
    assert torch.equal(acl, torch.where(is6, a6, a4)), int((acl != torch.where(is6, a6, a4)).sum())
    assert torch.equal(allow, torch.where(is6, w6, w4))
    want_route = torch.where(is6, t.rt6_chk(dst6), t.rt4_chk(dst))
    assert torch.equal(route, want_route), int((route != want_route).sum())
    six = (fam == 6).cpu().numpy()
    assert 0.13 < six.mean() < 0.17
    rng = np.random.default_rng(77)
    h = lambda x: x.cpu().numpy()
    acl_h, route_h, allow_h = h(acl), h(route), h(allow)
    proto_h, dport_h = h(proto), h(dport).view(np.uint16)
    for is6, k in ((False, 8000), (True, 3000)):
        s = rng.choice(np.nonzero(six == is6)[0], k)              # with replacement: O(k)
        if is6:
            want, wv = O.sg_batch_v6_np(t.tcp, t.udp, False, proto_h[s], h(src6)[s], dport_h[s],
                                        nthreads=THREADS)
            wr = O.rt_batch_v6_np(t.v6_list, h(dst6)[s][:1500], nthreads=THREADS)
        else:
            want, wv = O.sg_batch_v4_np(t.tcp, t.udp, False, proto_h[s], h(src)[s].view(np.uint32),
                                        dport_h[s], nthreads=THREADS)
            wr = O.rt_batch_v4_np(t.v4_list, h(dst)[s][:1500].view(np.uint32), nthreads=THREADS)
        np.testing.assert_array_equal(acl_h[s], want)
        np.testing.assert_array_equal(allow_h[s], wv)
        np.testing.assert_array_equal(route_h[s][:1500], wr)
    assert (route_h[six] >= 0).mean() > 0.8 and (acl_h[six] >= 0).mean() > 0.05
    nn = t.n4 + t.n6
    rr = route.long()
    bins = torch.where(rr >= 0, torch.where(fam == 6, t.n4 + rr, rr),
                       torch.where(fam == 6, nn + 1, nn))
    exp = torch.bincount(bins, minlength=nn + 2).cpu().numpy().astype(np.uint64)
    np.testing.assert_array_equal(clf.counters_read(V.COUNTERS_ROUTE), exp)
    del bins, rr
    # the `mix --compact6` form of the same batch (vc_pipeline_c6_dev): the
    # same outputs with the IPv6 addresses as one row per IPv6 packet
    six = fam == 6
    s6, d6 = src6[six].contiguous(), dst6[six].contiguous()
    c = clf.pipeline(proto, src, dst, dport, hid, pool, family=fam, src6=s6, dst6=d6,
                     want_allow=True, compact6=True)
    torch.cuda.synchronize()
    for x, y, name in zip(c, (acl, route, grp, allow), ("acl", "route", "group", "allow")):
        assert torch.equal(x, y), name


def test_c3_bench_batch():
    """The `c3` sub-bench exactly as bench.py builds it (bench.c3_workload:
    980,848 + 200,000 prefixes shortest-first, 256M lookups, 85 % IPv4):
    every one of the 217.6M IPv4 and 38.4M IPv6 results equal to
    exact.RouteChecker (RouteTable.java:44-59), the IPv6 ones through the
    wide root."""
    import torch
    clf = V.Classifier(0)
    try:
        dev = torch.device("cuda", 0)
        c = B.c3_workload(clf, dev)
        o4 = clf.route_v4(c.q4)
        o6 = clf.route_v6(c.q6)
        torch.cuda.synchronize()
        a4, k4 = c.rt.rules_raw(4)
        a6, k6 = c.rt.rules_raw(6)
        v4 = np.frombuffer(bytes(a4)[:k4 * 40], W.NET_DT)
        v6 = np.frombuffer(bytes(a6)[:k6 * 40], W.NET_DT)
        w4 = RouteChecker(v4, 4, dev)(c.q4)
        assert torch.equal(o4, w4), int((o4 != w4).sum())
        del w4
        w6 = RouteChecker(v6, 6, dev)(c.q6)
        assert torch.equal(o6, w6), int((o6 != w6).sum())
        assert len(c.q4) + len(c.q6) == 256 << 20
        assert float((o6 >= 0).float().mean()) > 0.85
    finally:
        clf.close()


def test_generator_device_equals_host(c5):
    """bench.gen_packets is index-addressable and device-independent."""
    import torch
    clf, t, dev = c5
    a = B.gen_packets(123456, 100000, t, t.pool_n, dev=dev)
    b = B.gen_packets(123456, 100000, t, t.pool_n, dev="cpu")
    for x, y in zip(a, b):
        assert torch.equal(x.cpu(), y)


def _dns_checker(text, groups):
    oh = O.Hosts(O.hosts_parse(text)[0])
    og = O.Groups(groups)
    return DnsChecker(text, groups), oh, og


def test_dns_c4_scale():
    """DNSServer classification at C4 scale: 100k groups + 50k hosts-file
    names (the bench's DNS workload, with hosts keys in both forms and IPv4
    literals mixed in): every one of the 1M results equal to DnsChecker
    (DNSServer.java:116-166 over Resolver.java:130-141's dual-key map), an
    oracle sample beside it, and exact group counters."""
    import torch
    clf = V.Classifier(0)
    try:
        groups, text, names, _ = B.c4_workload(True, 0)
        clf.compile_upstream(groups)
        clf.compile_hosts_text(text)
        names[::50] = [b"h%d.hosts.local." % i for i in range(0, len(names[::50]))]
        names[7::97] = [b"h%d.hosts.local" % i for i in range(0, len(names[7::97]))]
        names[3::211] = [b"1.2.3.%d." % (i & 255) for i in range(len(names[3::211]))]
        blob, off = W.pack(names)
        bd = torch.from_numpy(blob).cuda()
        od = torch.from_numpy(off.astype(np.int32)).cuda()
        clf.counters_enable(True)
        clf.counters_reset()
        kind, val = clf.dns_classify((bd, od))
        torch.cuda.synchronize()
        clf.counters_enable(False)
        kind, val = kind.cpu().numpy(), val.cpu().numpy()
        chk, oh, og = _dns_checker(text, groups)
        wk, wv = chk.batch(blob, off)
        np.testing.assert_array_equal(kind, wk)
        np.testing.assert_array_equal(val, wv)
        s = np.random.default_rng(4).integers(0, len(names), 300)
        want = [O.dns_classify(oh, og, names[i]) for i in s]
        assert [(int(kind[i]), int(val[i])) for i in s] == want
        # the "*" group (W.gen_groups) takes every name the hosts map does not
        assert {int(k) for k in np.unique(kind)} == {V.DNS_HOSTS, V.DNS_GROUP}
        assert (kind == V.DNS_HOSTS).sum() == sum(1 for q in names if q.endswith(
            (b".hosts.local", b".hosts.local.")))
        g = val[kind == V.DNS_GROUP]
        exp = np.bincount(g, minlength=len(groups) + 1).astype(np.uint64)
        np.testing.assert_array_equal(clf.counters_read(V.COUNTERS_GROUP), exp)
    finally:
        clf.close()


def test_dns_bench_batch():
    """The `dns` sub-bench's batch exactly as bench.py builds it
    (bench.c4_workload: 16M seeded draws from 1M DNS-flavoured names, 100k
    groups, 50k hosts lines) through vc_dns_classify_dev: every one of the
    16M (kind, value) pairs equal to DnsChecker."""
    import torch
    clf = V.Classifier(0)
    try:
        n = 16 << 20
        groups, text, names, pidx = B.c4_workload(True, n)
        clf.compile_upstream(groups)
        clf.compile_hosts_text(text)
        nblob, noff = W.pack(names)
        blob, off, _ = B.gather_strings_dev(nblob, noff, pidx, "cuda")
        kind, val = clf.dns_classify((blob, off))
        torch.cuda.synchronize()
        wk, wv = _dns_checker(text, groups)[0].batch(nblob, noff)
        pi = torch.from_numpy(pidx).cuda()
        wk = torch.from_numpy(wk).cuda()[pi]
        wv = torch.from_numpy(wv).cuda()[pi]
        assert kind.shape[0] == n
        assert torch.equal(kind, wk), int((kind != wk).sum())
        assert torch.equal(val, wv), int((val != wv).sum())
    finally:
        clf.close()


def test_dnsd_bench_workload():
    """The `dnsd` sub-bench exactly as bench.py builds it (bench.dnsd_tables /
    dnsd_batch: 10k-rule SecurityGroup, 100k groups, 50k hosts, its 16M
    datagrams from random IPv4 senders).  Every datagram: the UDP rule and
    verdict of the sender (exact.AclChecker, SecurityGroup.java:30-45 with
    DNSServer.java:469's source port), the status, the question count, and
    the answered question's type, kind and value (DnsChecker over the
    templates' qnames, DNSServer.java:116-166).  An oracle sample of the
    whole drain loop (vo_dnsd_batch) beside it."""
    import torch
    clf = V.Classifier(0)
    try:
        t = B.dnsd_tables(clf)
        n = 16 << 20                                   # the bench's batch
        blob, off, nbytes, r4, rport, pidx = B.dnsd_batch(t, n, "cuda")
        res = clf.dns_datagrams((blob, off), r4, rport)
        torch.cuda.synchronize()
        dev = torch.device("cuda", 0)
        # every datagram against the exact checkers
        proto = torch.full((n,), 17, dtype=torch.uint8, device=dev)
        want_acl, want_allow = AclChecker(t.tcp, t.udp, True, dev).v4(proto, r4, rport)
        assert torch.equal(res["acl"], want_acl), int((res["acl"] != want_acl).sum())
        qb, qo = W.pack(t.qnames)
        qk, qv = _dns_checker(t.hosts, t.groups)[0].batch(qb, qo)
        pi = torch.from_numpy(pidx).to(dev)
        qk = torch.from_numpy(qk).to(dev)[pi]
        qv = torch.from_numpy(qv).to(dev)[pi]
        qt = torch.from_numpy(t.qtypes.astype(np.int64)).to(dev)[pi]
        ok = want_allow == 1
        full = lambda v: torch.full((n,), v, dtype=torch.uint8, device=dev)
        want_status = torch.where(~ok, full(V.DNSD_REJECTED),
                                  torch.where(qk == V.DNS_RECURSIVE, full(V.DNSD_RECURSIVE),
                                              full(V.DNSD_ANSWER)))
        assert torch.equal(res["status"], want_status), int((res["status"] != want_status).sum())
        assert torch.equal(res["nq"], ok.to(torch.uint8))
        assert torch.equal(res["qtype"][:, 0][ok].long() & 0xFFFF, qt[ok])
        assert torch.equal(res["kind"][:, 0][ok], qk[ok])
        assert torch.equal(res["value"][:, 0][ok], qv[ok])
        assert 0 < int((~ok).sum()) < n
        # oracle sample of the drain loop
        res = {k: v.cpu().numpy() for k, v in res.items()}
        res["qtype"] = res["qtype"].view(np.uint16)
        h4 = r4.cpu().numpy().view(np.uint32)
        hp = rport.cpu().numpy().view(np.uint16)
        og = O.Groups(t.groups)
        oh = O.Hosts(O.hosts_parse(t.hosts)[0])
        s = np.sort(np.random.default_rng(5).choice(n, 1500, replace=False))
        sb, so = W.pack([bytes(t.dblob[t.doff[j]:t.doff[j + 1]]) for j in pidx[s]])
        want = O.dnsd_batch_np(t.tcp, t.udp, True, oh, og, sb, so, None, h4[s], None, hp[s],
                               nthreads=16)
        for k in ("status", "acl", "nq"):
            np.testing.assert_array_equal(res[k][s], want[k], err_msg=k)
        live = want["nq"] > 0                          # per-question fields for q < nq
        assert live.mean() > 0.99
        for k in ("qtype", "kind", "value"):
            np.testing.assert_array_equal(res[k][s, 0][live].astype(want[k].dtype),
                                          want[k][live, 0], err_msg=k)
    finally:
        clf.close()


def test_counters_values_outside_the_space():
    """A counter space above 65,536 bins (the bucketed path) fed values at or
    past its size -- e.g. a hostname pool classified against an older, larger
    Upstream -- counts only the in-range values and never faults; the fused
    pipeline agrees."""
    import torch
    clf = V.Classifier(0)
    try:
        ng = 70_000
        groups = [({}, {"host": "g%d.example" % i}) for i in range(ng)]
        clf.compile_upstream(groups)
        g = torch.Generator(device="cuda")
        g.manual_seed(3)
        n = (4 << 20) + 3
        out = torch.randint(-1, 3 * ng, (n,), generator=g, device="cuda", dtype=torch.int32)
        out[::1000] = 2**31 - 1
        clf.counters_enable(True)
        clf.counters_reset()
        clf.counters_add(V.COUNTERS_GROUP, out)
        torch.cuda.synchronize()
        o = out.long()
        keep = (o >= 0) & (o < ng)
        exp = torch.bincount(o[keep], minlength=ng + 1)
        exp[ng] = int((o < 0).sum())
        np.testing.assert_array_equal(clf.counters_read(V.COUNTERS_GROUP),
                                      exp.cpu().numpy().astype(np.uint64))
        # the pipeline's in-kernel group buckets, pool values past n_groups
        tcp, udp = W.gen_sg_rules(100, 1)
        a, na, ka = W.as_ctypes(tcp, V._lib.VcAclRule)
        b, nb, kb = W.as_ctypes(udp, V._lib.VcAclRule)
        V.check(V.lib().vc_compile_acl(clf.h, a, na, b, nb, 0))
        net, plen = W.gen_v4_prefixes(200_000, 2)
        nets = W.v4_nets(net, plen)
        ra, rn, rk = W.as_ctypes(nets, V._lib.VcNet)
        clf.compile_routes_raw(ra, rn, (V._lib.VcNet * 1)(), 0)
        pool = torch.randint(-1, 2 * ng, (1 << 20,), generator=g, device="cuda",
                             dtype=torch.int32)
        m = 8 << 20
        T = lambda x: torch.from_numpy(x).cuda()
        proto, src, port = W.gen_acl_queries(tcp, udp, m, 5)
        dst = W.v4_lookups(net, plen, m, 6)
        hid = torch.randint(0, 1 << 20, (m,), generator=g, device="cuda", dtype=torch.int32)
        clf.counters_reset()
        clf.counters_enable(True)
        acl, route, grp, _ = clf.pipeline_v4(T(proto), T(src), T(dst), T(port), hid, pool)
        torch.cuda.synchronize()
        clf.counters_enable(False)
        assert torch.equal(grp, pool[hid.long()])
        o = grp.long()
        keep = (o >= 0) & (o < ng)
        exp = torch.bincount(o[keep], minlength=ng + 1)
        exp[ng] = int((o < 0).sum())
        np.testing.assert_array_equal(clf.counters_read(V.COUNTERS_GROUP),
                                      exp.cpu().numpy().astype(np.uint64))
        r = route.long()
        exp = torch.bincount(torch.where(r >= 0, r, len(nets)), minlength=len(nets) + 2)
        np.testing.assert_array_equal(clf.counters_read(V.COUNTERS_ROUTE),
                                      exp.cpu().numpy().astype(np.uint64))
    finally:
        clf.close()


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


@pytest.mark.parametrize("serial,finish", [(False, "stream"), (False, "inline"), (True, "inline")])
def test_bench_schedule_with_rccl_bucket(serial, finish):
    """bench.C5Steps with the counter bucket on: HitCounterBucket.fill copies
    the library's device counters (vc_counters_device) device-to-device on
    the counting stream, then one RCCL all-reduce (world size 1 on this
    box); the elapsed-time MAX all-reduce of bench.main.  After W + K steps
    over the same packets the bucket equals vc_counters_read and (W + K) x
    the histograms of one step's outputs."""
    import torch
    import torch.distributed as dist
    dev = torch.device("cuda", 0)
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(_free_port())
    dist.init_process_group("nccl", rank=0, world_size=1, device_id=dev)
    clf = V.Classifier(0)
    try:
        t = B.c5_tables(clf, dev, 1 << 20, acl_rules=2000, v4=150_000, v6=20_000,
                        groups=70_000)
        lo, hi = B.shard(4_000_003, 0, 1)
        pk = B.gen_packets(lo, hi - lo, t, t.pool_n, dev=dev)
        steps = B.C5Steps(clf, t, pk, dev, bucket=True, serial=serial, finish=finish)
        clf.counters_reset()
        steps.run(0, 1, False)
        torch.cuda.synchronize()
        steps.reset_events()
        steps.run(1, 2, True)
        torch.cuda.synchronize()
        el = B.max_over_ranks(1.5, dev)
        assert el == 1.5
        views = [v.cpu().numpy().view(np.uint64) for v in steps.bucket.views]
        for k, v in zip((V.COUNTERS_ACL, V.COUNTERS_ROUTE, V.COUNTERS_GROUP), views):
            np.testing.assert_array_equal(v, clf.counters_read(k))
        acl, route, grp, _ = steps.outsb[0]
        nt, nu = len(t.tcp), len(t.udp)
        is_tcp = pk[0] == 6
        a = acl.long()
        bins = torch.where(a >= 0, torch.where(is_tcp, a, nt + a),
                           torch.where(is_tcp, nt + nu, nt + nu + 1))
        exp = 3 * torch.bincount(bins, minlength=nt + nu + 2)
        np.testing.assert_array_equal(views[0], exp.cpu().numpy().astype(np.uint64))
        r = route.long()
        nn = t.n4 + t.n6
        exp = 3 * torch.bincount(torch.where(r >= 0, r, nn), minlength=nn + 2)
        np.testing.assert_array_equal(views[1], exp.cpu().numpy().astype(np.uint64))
        g = grp.long()
        ng = len(t.groups)
        exp = 3 * torch.bincount(torch.where(g >= 0, g, ng), minlength=ng + 1)
        np.testing.assert_array_equal(views[2], exp.cpu().numpy().astype(np.uint64))
        assert steps.span("pipe") > 0
    finally:
        clf.close()
        dist.destroy_process_group()

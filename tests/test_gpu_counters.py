"""GPU tier: the hit-counter passes (device/counters.hip) on synthetic output
arrays, checked exactly against numpy histograms.

Covers the small-space path (ACL, 32K-bin LDS histograms) and the
large-space path (routes, groups: bucket partition + per-segment LDS
histograms), a hot bin holding 30 % of the items, nulls, n not a multiple
of 4, unaligned array starts (the scalar kernels) and the DNS kind filter.
"""
import numpy as np
import pytest

import vproxy_amd as V
from vproxy_amd import workloads as W

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def clf():
    c = V.Classifier(0)
    yield c
    c.close()


def _compile(clf):
    tcp, udp = W.gen_sg_rules(4000, 124)
    a, na, ka = W.as_ctypes(tcp, V._lib.VcAclRule)
    b, nb, kb = W.as_ctypes(udp, V._lib.VcAclRule)
    V.check(V.lib().vc_compile_acl(clf.h, a, na, b, nb, 0))
    net, plen = W.gen_v4_prefixes(300000, 125)
    nets = W.v4_nets(net, plen)
    r, nr, kr = W.as_ctypes(nets, V._lib.VcNet)
    clf.compile_routes_raw(r, nr, (V._lib.VcNet * 1)(), 0)
    groups, _ = W.gen_groups(100000, 126)
    clf.compile_upstream(groups)
    return len(tcp), len(udp), nr, len(groups)


@pytest.mark.parametrize("n,off", [(3_000_001, 0), (1_000_003, 1), (4099, 3), (5, 0)])
def test_counter_passes_synthetic(clf, n, off):
    import torch
    nt, nu, n4, ng = _compile(clf)
    rng = np.random.default_rng(n)
    T = lambda x: torch.from_numpy(x).cuda()
    clf.counters_enable(False)
    clf.counters_reset()
    m = n + off
    proto = np.where(rng.random(m) < 0.5, 6, 17).astype(np.uint8)
    acl = np.where(proto == 6, rng.integers(0, nt, m), rng.integers(0, nu, m))
    acl = np.where(rng.random(m) < 0.3, 7, acl)                 # hot rule
    acl = np.where(rng.random(m) < 0.2, -1, acl).astype(np.int32)
    route = rng.integers(0, n4, m)
    route = np.where(rng.random(m) < 0.3, n4 - 1, route)        # hot route
    route = np.where(rng.random(m) < 0.1, -1, route).astype(np.int32)
    grp = rng.integers(0, ng, m)
    grp = np.where(rng.random(m) < 0.3, 5, grp)                 # hot group
    grp = np.where(rng.random(m) < 0.1, -1, grp).astype(np.int32)
    da, dp, dr, dg = T(acl), T(proto), T(route), T(grp)
    clf.counters_add(V.COUNTERS_ACL, da[off:], aux=dp[off:])
    clf.counters_add(V.COUNTERS_ROUTE, dr[off:], family=4)
    clf.counters_add(V.COUNTERS_GROUP, dg[off:])
    torch.cuda.synchronize()
    acl, proto, route, grp = acl[off:], proto[off:], route[off:], grp[off:]
    is_t = proto == 6
    exp = np.bincount(np.where(acl >= 0, np.where(is_t, acl, nt + acl), nt + nu + (~is_t)),
                      minlength=nt + nu + 2)
    np.testing.assert_array_equal(clf.counters_read(V.COUNTERS_ACL), exp.astype(np.uint64))
    exp = np.bincount(np.where(route >= 0, route, n4), minlength=n4 + 2)
    np.testing.assert_array_equal(clf.counters_read(V.COUNTERS_ROUTE), exp.astype(np.uint64))
    exp = np.bincount(np.where(grp >= 0, grp, ng), minlength=ng + 1)
    np.testing.assert_array_equal(clf.counters_read(V.COUNTERS_GROUP), exp.astype(np.uint64))


def test_counter_dns_kinds(clf):
    """DNS outputs: only items whose kind is VC_DNS_GROUP count."""
    import torch
    nt, nu, n4, ng = _compile(clf)
    rng = np.random.default_rng(7)
    clf.counters_reset()
    n = 777_777
    kind = rng.integers(1, 6, n).astype(np.uint8)
    val = rng.integers(0, ng, n).astype(np.int32)
    clf.counters_add(V.COUNTERS_GROUP, torch.from_numpy(val).cuda(),
                     aux=torch.from_numpy(kind).cuda())
    torch.cuda.synchronize()
    exp = np.bincount(val[kind == 2], minlength=ng + 1)
    np.testing.assert_array_equal(clf.counters_read(V.COUNTERS_GROUP), exp.astype(np.uint64))


@pytest.mark.parametrize("n,off", [(2_000_003, 0), (700_001, 1)])
def test_pipeline_counts_in_kernel(clf, n, off):
    """Counters enabled on the pipeline: the kernel histograms the ACL in
    LDS and counts route/group buckets itself (large spaces: 300k routes,
    100k groups), the library finishes them; exact vs numpy histograms of
    the outputs, aligned (16-byte loads) and unaligned (scalar) inputs,
    n % 4 != 0; outputs vs the oracle on a sample."""
    import torch
    import oracle_ffi as O
    nt, nu, n4, ng = _compile(clf)
    tcp, udp = W.gen_sg_rules(4000, 124)
    net, plen = W.gen_v4_prefixes(300000, 125)
    groups, ghosts = W.gen_groups(100000, 126)
    names = W.gen_hostnames(ghosts, 200000, 127)
    pool = clf.hint_search(names)
    m = n + off
    proto, src, port = W.gen_acl_queries(tcp, udp, m, 128)
    dst = W.v4_lookups(net, plen, m, 129)
    hid = np.random.default_rng(130).integers(0, len(names), m).astype(np.uint32)
    hid[::53] = 0xFFFFFFFF
    T = lambda x: torch.from_numpy(x).cuda()
    dev = [T(x)[off:] for x in (proto, src, dst, port, hid)]
    clf.counters_enable(True)
    clf.counters_reset()
    acl, route, grp, _ = clf.pipeline_v4(*dev, T(pool))
    torch.cuda.synchronize()
    clf.counters_enable(False)
    acl, route, grp = (x.cpu().numpy() for x in (acl, route, grp))
    proto, src, dst, port, hid = (x[off:] for x in (proto, src, dst, port, hid))
    is_t = proto == 6
    exp = np.bincount(np.where(acl >= 0, np.where(is_t, acl, nt + acl), nt + nu + (~is_t)),
                      minlength=nt + nu + 2)
    np.testing.assert_array_equal(clf.counters_read(V.COUNTERS_ACL), exp.astype(np.uint64))
    exp = np.bincount(np.where(route >= 0, route, n4), minlength=n4 + 2)
    np.testing.assert_array_equal(clf.counters_read(V.COUNTERS_ROUTE), exp.astype(np.uint64))
    exp = np.bincount(np.where(grp >= 0, grp, ng), minlength=ng + 1)
    np.testing.assert_array_equal(clf.counters_read(V.COUNTERS_GROUP), exp.astype(np.uint64))
    np.testing.assert_array_equal(grp, np.where(hid == 0xFFFFFFFF, -1,
                                                pool[np.minimum(hid, len(pool) - 1)]))
    s = np.random.default_rng(131).integers(0, n, 3000)
    want, _ = O.sg_batch_v4_np(tcp, udp, False, proto[s], src[s], port[s])
    np.testing.assert_array_equal(acl[s], want)
    np.testing.assert_array_equal(route[s], O.rt_batch_v4_np(W.v4_nets(net, plen), dst[s]))


def test_counters_prometheus(clf):
    """vc_counters_prometheus renders the device counters exactly as
    vc_prometheus_hits renders the same counters read back to the host."""
    import torch
    from vproxy_amd import prometheus as P
    nt, nu, n4, ng = _compile(clf)
    rng = np.random.default_rng(11)
    clf.counters_reset()
    val = rng.integers(-1, ng, 100_000).astype(np.int32)
    clf.counters_add(V.COUNTERS_GROUP, torch.from_numpy(val).cuda())
    torch.cuda.synchronize()
    text = clf.counters_prometheus("zone=eu")
    want = P.hits_text(acl=clf.counters_read(V.COUNTERS_ACL), n_tcp=nt, n_udp=nu,
                       route=clf.counters_read(V.COUNTERS_ROUTE), n4=n4, n6=0,
                       group=clf.counters_read(V.COUNTERS_GROUP), n_groups=ng,
                       extra_labels="zone=eu")
    assert text == want
    assert ('upstream_server_group_hit_count{group="none",zone="eu"} %d\n'
            % int((val < 0).sum())) in text

"""GPU tier: IPv4 SecurityGroup images too large to stage whole in LDS.

Above 30K boundary words (both protocol lists together) the kernels stage
every (1 << shift)-th boundary as a fence and finish the interval search in
one block of boundaries in global memory (classify.hip acl_v4_one).  These
tables (20k and 80k rules: ~40K and ~160K boundary words, fence shifts 1 and
3) run through vc_acl_classify_v4 and through both pipeline kernels against
the oracle's first-match scans of SecurityGroup.allow
(core/src/main/java/vproxy/component/secure/SecurityGroup.java:30-45).
"""
import os

import numpy as np
import pytest

import oracle_ffi as O
import vproxy_amd as V
from vproxy_amd import workloads as W

from test_gpu_pipeline import _call, _dev, _oracle, _packets

pytestmark = pytest.mark.gpu
THREADS = min(16, os.cpu_count() or 1)


def _compile(clf, n_rules, seed):
    tcp, udp = W.gen_sg_rules(n_rules, seed, p_range=0.3)
    a, na, ka = W.as_ctypes(tcp, V._lib.VcAclRule)
    b, nb, kb = W.as_ctypes(udp, V._lib.VcAclRule)
    V.check(V.lib().vc_compile_acl(clf.h, a, na, b, nb, 0))
    return tcp, udp


@pytest.fixture(scope="module")
def clf():
    c = V.Classifier(0)
    yield c
    c.close()


@pytest.mark.parametrize("n_rules", [20000, 80000])
def test_acl_v4_fenced_vs_oracle(clf, n_rules):
    import torch
    tcp, udp = _compile(clf, n_rules, 61)
    proto, src, port = W.gen_acl_queries(tcp, udp, 60_001, 62)
    want, wv = O.sg_batch_v4_np(tcp, udp, False, proto, src, port, nthreads=THREADS)
    got, allow = clf.acl_v4(proto, src, port)                  # host entry
    np.testing.assert_array_equal(got, want)
    np.testing.assert_array_equal(allow, wv)
    d = [torch.from_numpy(x).cuda() for x in (proto, src, port)]
    got, allow = clf.acl_v4(*d)                                # device, vector kernel
    torch.cuda.synchronize()
    np.testing.assert_array_equal(got.cpu().numpy(), want)
    np.testing.assert_array_equal(allow.cpu().numpy(), wv)
    # unaligned device inputs: the one-item-per-lane kernel
    d1 = []
    for x in (proto, src, port):
        t = torch.from_numpy(np.concatenate([x[:1], x])).cuda()
        d1.append(t[1:])
    got, allow = clf.acl_v4(*d1)
    torch.cuda.synchronize()
    np.testing.assert_array_equal(got.cpu().numpy(), want)
    np.testing.assert_array_equal(allow.cpu().numpy(), wv)
    assert (want >= 0).mean() > 0.3


@pytest.mark.parametrize("mixed", [False, True])
def test_pipelines_with_fenced_acl(clf, mixed):
    """Both pipeline kernels (the tuned IPv4 one and the mixed-family one)
    with an 80k-rule ACL: the fences share the workgroup's LDS with the
    in-kernel hit counts and, in the mixed kernel, the IPv6 fences."""
    import torch
    tcp, udp = _compile(clf, 80000, 63)
    rng = np.random.default_rng(64)
    net, plen = W.gen_v4_prefixes(20000, 65)
    nets4 = W.v4_nets(net, plen)
    rng.shuffle(nets4)
    hi, lo, p6 = W.gen_v6_prefixes(5000, 66)
    nets6 = W.v6_nets(hi, lo, p6)
    ra, rn, rk = W.as_ctypes(nets4, V._lib.VcNet)
    rb, rbn, rbk = W.as_ctypes(nets6, V._lib.VcNet)
    clf.compile_routes_raw(ra, rn, rb, rbn)
    groups, ghosts = W.gen_groups(2000, 67)
    clf.compile_upstream(groups)
    pool = clf.hint_search(W.gen_hostnames(ghosts, 3000, 68))
    t = dict(tcp=tcp, udp=udp, net=net, plen=plen, nets4=nets4, nets6=nets6, hi=hi, lo=lo,
             p6=p6, pool=pool, groups=groups)
    p = _packets(t, 40_003, 69)
    if not mixed:
        p = dict(p, family=np.full(len(p["family"]), 4, np.uint8))
    want = _oracle(t, p)
    d = _dev(p)
    pool_d = torch.from_numpy(pool).cuda()
    clf.counters_enable(True)
    clf.counters_reset()
    got = _call(clf, d, pool_d, family=mixed)
    torch.cuda.synchronize()
    clf.counters_enable(False)
    for g, w, name in zip(got, want, ("acl", "route", "group", "allow")):
        np.testing.assert_array_equal(g.cpu().numpy(), w, err_msg=name)
    acl = want[0]
    nt, nu = len(tcp), len(udp)
    is_t = p["proto"] == 6
    exp = np.zeros(nt + nu + 2, np.uint64)
    np.add.at(exp, np.where(acl >= 0, np.where(is_t, acl, nt + acl), nt + nu + (~is_t)), 1)
    np.testing.assert_array_equal(clf.counters_read(V.COUNTERS_ACL), exp)

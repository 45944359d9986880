"""GPU tier: the plain (host-buffer) entry points run batches in 4M-item
chunks on two streams (capi.cpp host_chunks).  Batches spanning several
chunks, with a ragged last chunk, must give exactly the device entry
points' results (themselves checked against the oracle elsewhere), from
pageable and from page-locked (vc_host_register) buffers."""
import ctypes as C

import numpy as np
import pytest

import vproxy_amd as V
from vproxy_amd import workloads as W

pytestmark = pytest.mark.gpu
N = 9_437_187          # 2 full chunks + a ragged third


@pytest.fixture(scope="module")
def clf():
    c = V.Classifier(0)
    yield c
    c.close()


@pytest.mark.parametrize("pinned", [False, True])
def test_acl_route_source_chunks(clf, pinned):
    import torch
    tcp, udp = W.gen_sg_rules(3000, 61)
    a, na, ka = W.as_ctypes(tcp, V._lib.VcAclRule)
    b, nb, kb = W.as_ctypes(udp, V._lib.VcAclRule)
    V.check(V.lib().vc_compile_acl(clf.h, a, na, b, nb, 0))
    net, plen = W.gen_v4_prefixes(50000, 62)
    r, nr, kr = W.as_ctypes(W.v4_nets(net, plen), V._lib.VcNet)
    clf.compile_routes_raw(r, nr, (V._lib.VcNet * 1)(), 0)
    rng = np.random.default_rng(63)
    groups = [[(bytes(rng.integers(0, 256, 4).astype(np.uint8)), 80, 1, True)
               for _ in range(int(rng.integers(1, 9)))] for _ in range(500)]
    clf.compile_servers(groups)
    proto, src, port = W.gen_acl_queries(tcp, udp, N, 64)
    dst = W.v4_lookups(net, plen, N, 65)
    grp = rng.integers(0, len(groups), N).astype(np.int32)
    reg = []
    if pinned:
        for x in (proto, src, port, dst, grp):
            V.check(V.lib().vc_host_register(C.c_void_p(x.ctypes.data), x.nbytes))
            reg.append(x)
    try:
        idx, allow = clf.acl_v4(proto, src, port)
        rt = clf.route_v4(dst)
        sv = clf.source_select(grp, src)
    finally:
        for x in reg:
            V.check(V.lib().vc_host_unregister(C.c_void_p(x.ctypes.data)))
    T = lambda x: torch.from_numpy(x).cuda()
    didx, dallow = clf.acl_v4(T(proto), T(src), T(port), want_allow=True)
    drt = clf.route_v4(T(dst))
    dsv = clf.source_select(T(grp), T(src.view(np.int32)))
    torch.cuda.synchronize()
    np.testing.assert_array_equal(idx, didx.cpu().numpy())
    np.testing.assert_array_equal(allow, dallow.cpu().numpy())
    np.testing.assert_array_equal(rt, drt.cpu().numpy())
    np.testing.assert_array_equal(sv, dsv.cpu().numpy())

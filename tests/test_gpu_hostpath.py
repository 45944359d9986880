"""GPU tier: the plain (host-buffer) entry points run batches in 4M-item
chunks on the two lanes of a stager (capi.cpp host_chunks: caller arrays
are copied into a page-locked bounce buffer, DMA'd, classified, and copied
back).  Batches spanning several chunks, with a ragged last chunk, are
checked against the oracle on a sample of every chunk and must equal the
device entry points' results everywhere.  Registered (zero-copy) buffers
are covered by test_gpu_zz_registered.py, which runs last."""
import numpy as np
import pytest

import oracle_ffi as O
import vproxy_amd as V
from vproxy_amd import workloads as W

pytestmark = pytest.mark.gpu
N = 9_437_187          # 2 full chunks + a ragged third
CHUNK = 4 << 20


@pytest.fixture(scope="module")
def clf():
    c = V.Classifier(0)
    yield c
    c.close()


def chunk_sample(n, k, seed):
    """k indices per chunk plus both ends of every chunk"""
    rng = np.random.default_rng(seed)
    idx = [rng.integers(0, n, k)]
    for lo in range(0, n, CHUNK):
        hi = min(n, lo + CHUNK)
        idx.append(np.arange(lo, min(hi, lo + 64)))
        idx.append(np.arange(max(lo, hi - 64), hi))
    return np.unique(np.concatenate(idx))


def tables(clf, seed=61):
    tcp, udp = W.gen_sg_rules(3000, seed)
    a, na, ka = W.as_ctypes(tcp, V._lib.VcAclRule)
    b, nb, kb = W.as_ctypes(udp, V._lib.VcAclRule)
    V.check(V.lib().vc_compile_acl(clf.h, a, na, b, nb, 0))
    net, plen = W.gen_v4_prefixes(50000, seed + 1)
    nets = W.v4_nets(net, plen)
    r, nr, kr = W.as_ctypes(nets, V._lib.VcNet)
    clf.compile_routes_raw(r, nr, (V._lib.VcNet * 1)(), 0)
    rng = np.random.default_rng(seed + 2)
    groups = [[(bytes(rng.integers(0, 256, 4).astype(np.uint8)), 80, 1, True)
               for _ in range(int(rng.integers(1, 9)))] for _ in range(500)]
    clf.compile_servers(groups)
    proto, src, port = W.gen_acl_queries(tcp, udp, N, seed + 3)
    dst = W.v4_lookups(net, plen, N, seed + 4)
    grp = rng.integers(0, len(groups), N).astype(np.int32)
    return dict(tcp=tcp, udp=udp, nets=nets, groups=groups, proto=proto, src=src, port=port,
                dst=dst, grp=grp)


def check_vs_oracle(t, idx, allow, rt, sv, seed):
    s = chunk_sample(N, 20000, seed)
    want_idx, want_allow = O.sg_batch_v4_np(t["tcp"], t["udp"], False, t["proto"][s],
                                            t["src"][s], t["port"][s])
    np.testing.assert_array_equal(idx[s], want_idx)
    np.testing.assert_array_equal(allow[s], want_allow)
    np.testing.assert_array_equal(rt[s], O.rt_batch_v4_np(t["nets"], t["dst"][s]))
    np.testing.assert_array_equal(sv[s], O.source_batch_np(t["groups"], V.SOURCE_ALL,
                                                           t["grp"][s], t["src"][s]))


def test_acl_route_source_chunks(clf):
    import torch
    t = tables(clf)
    idx, allow = clf.acl_v4(t["proto"], t["src"], t["port"])
    rt = clf.route_v4(t["dst"])
    sv = clf.source_select(t["grp"], t["src"])
    check_vs_oracle(t, idx, allow, rt, sv, 66)
    T = lambda x: torch.from_numpy(x).cuda()
    didx, dallow = clf.acl_v4(T(t["proto"]), T(t["src"]), T(t["port"]), want_allow=True)
    drt = clf.route_v4(T(t["dst"]))
    dsv = clf.source_select(T(t["grp"]), T(t["src"].view(np.int32)))
    torch.cuda.synchronize()
    np.testing.assert_array_equal(idx, didx.cpu().numpy())
    np.testing.assert_array_equal(allow, dallow.cpu().numpy())
    np.testing.assert_array_equal(rt, drt.cpu().numpy())
    np.testing.assert_array_equal(sv, dsv.cpu().numpy())

"""GPU tier: batch-size edges of the compute entry points.

- Every compute entry point, host and device form, with n = 0: VC_OK and
  nothing written (sentinel output words unchanged); with n < 0: VC_EINVAL.
- The string kernels (hint, DNS, SNI) share one chunk schedule (chunks.h
  ChunksT): below a resident grid every wave takes one tail ticket; past it a
  static block per wave plus tail tickets; at the bench sizes big tickets
  too (those run whole in test_gpu_c5 / test_gpu_certs).  Sizes around the
  chunk and pair edges (1 .. 129) and across the first two regimes
  (4097 .. 2M) are checked whole against the exact checkers (tests/exact.py,
  oracle-validated), the small ones also against the oracle and through the
  host entry point.
"""
import ctypes as C

import numpy as np
import pytest

import bench as B
import oracle_ffi as O
import vproxy_amd as V
from exact import CertChecker, DnsChecker, HintChecker
from vproxy_amd import workloads as W
from vproxy_amd._lib import VC_EINVAL, VC_OK

pytestmark = pytest.mark.gpu
SIZES = (1, 2, 3, 63, 64, 65, 127, 128, 129, 4097, 100_003, 800_001, 2_000_003)
SMALL = 4097
SENT = 0x5A5A5A5A


@pytest.fixture(scope="module")
def clf():
    c = V.Classifier(0)
    yield c
    c.close()


def _sizes_check(clf, names, want_all, run_dev, run_host, oracle, label):
    """want_all[i]: the checker's answer for names[i]; the batch of size n is
    names[pidx[:n]] in a device blob"""
    import torch
    pidx = np.random.default_rng(len(names)).integers(0, len(names), max(SIZES))
    nblob, noff = W.pack(names)
    for n in SIZES:
        blob, off, _ = B.gather_strings_dev(nblob, noff, pidx[:n], "cuda")
        got = run_dev(blob, off, n)
        torch.cuda.synchronize()
        got = [g.cpu().numpy() for g in got]
        want = [w[pidx[:n]] for w in want_all]
        for g, w in zip(got, want):
            np.testing.assert_array_equal(g, w, err_msg="%s n=%d" % (label, n))
        if n <= SMALL:
            sel = [names[i] for i in pidx[:n]]
            host = run_host(sel)
            for h, w in zip(host, want):
                np.testing.assert_array_equal(h, w, err_msg="%s host n=%d" % (label, n))
            s = np.arange(n) if n <= 129 else np.random.default_rng(n).integers(0, n, 129)
            o = oracle([sel[i] for i in s])
            for k, w in enumerate(o):
                np.testing.assert_array_equal(w, [x[s] for x in want][k],
                                              err_msg="%s oracle n=%d" % (label, n))


def test_hint_ragged_sizes(clf):
    groups, _, names, _ = B.c4_workload(False, 0)
    clf.compile_upstream(groups)
    chk = HintChecker(groups)
    nblob, noff = W.pack(names)
    want = chk.batch(nblob, noff)
    og = O.Groups(groups)

    def oracle(sel):
        b, o = W.pack(sel)
        return [O.hint_batch_np(og, b, o, None, nthreads=16)]

    _sizes_check(clf, names, [want],
                 lambda b, o, n: [clf.hint_search((b, o, None))],
                 lambda sel: [clf.hint_search(sel)], oracle, "hint")


def test_dns_ragged_sizes(clf):
    groups, text, names, _ = B.c4_workload(True, 0)
    clf.compile_upstream(groups)
    clf.compile_hosts_text(text)
    oh = O.Hosts(O.hosts_parse(text)[0])
    og = O.Groups(groups)
    chk = DnsChecker(text, groups)
    nblob, noff = W.pack(names)
    wk, wv = chk.batch(nblob, noff)

    def oracle(sel):
        b, o = W.pack(sel)
        return list(O.dns_batch_np(oh, og, b, o, nthreads=16))

    _sizes_check(clf, names, [wk, wv],
                 lambda b, o, n: list(clf.dns_classify((b, o))),
                 lambda sel: list(clf.dns_classify(sel)), oracle, "dns")


def test_sni_ragged_sizes(clf):
    holders, names, _ = B.sni_workload(0)
    clf.compile_certs(holders)
    nblob, noff = W.pack(names)
    want = CertChecker(holders).batch(nblob, noff)
    certs = O.Certs(holders)

    def oracle(sel):
        b, o = W.pack(sel)
        return [O.cert_batch_np(certs, b, o, nthreads=16)]

    _sizes_check(clf, names, [want],
                 lambda b, o, n: [clf.cert_choose((b, o, None))],
                 lambda sel: [clf.cert_choose(sel)], oracle, "sni")


# ---------------------------------------------------------------------------
# n = 0 and n < 0 through the C ABI
# ---------------------------------------------------------------------------
def _tables(clf):
    """Small tables of every kind, so no entry point refuses for lack of one."""
    tcp, udp = W.gen_sg_rules(50, 3)
    a, na, ka = W.as_ctypes(tcp, V._lib.VcAclRule)
    b, nb, kb = W.as_ctypes(udp, V._lib.VcAclRule)
    V.check(V.lib().vc_compile_acl(clf.h, a, na, b, nb, 0))
    clf.compile_routes(["10.0.0.0/8", "10.1.0.0/16"], ["fd00::/8"])
    groups, ghosts = W.gen_groups(100, 4)
    clf.compile_upstream(groups)
    clf.compile_hosts([("a.example.", 7)])
    clf.compile_servers([[(b"\x01\x02\x03\x04", 80, 1, True)]])
    clf.compile_certs([["a.com"], ["*.b.com"]])
    clf.compile_mirror([{"origin": "o", "mirror": 0}])


class _Buf:
    """A device and a host buffer of sentinel words, passed for every array."""

    def __init__(self):
        import torch
        self.d = torch.full((4096,), SENT, dtype=torch.int32, device="cuda")
        self.h = np.full(4096, SENT, np.int32)
        self.dp = C.c_void_p(self.d.data_ptr())
        self.hp = C.c_void_p(self.h.ctypes.data)

    def untouched(self):
        import torch
        torch.cuda.synchronize()
        return bool((self.d == SENT).all()) and bool((self.h == SENT).all())


def _calls(L, h, p, stream):
    """(name, call(n)) for every compute entry point; every array argument is
    the sentinel buffer p (host or device), structs point into it too."""
    s = stream
    pkt = V._lib.VcPackets(*([p.value] * 8))
    po = V._lib.VcPipelineOut(*([p.value] * 4))
    pk = V._lib.VcPktOut(**{f: p.value for f, _ in V._lib.VcPktOut._fields_})
    dn = V._lib.VcDnsdOut(**{f: p.value for f, _ in V._lib.VcDnsdOut._fields_})
    it = V._lib.VcMirrorItems(**{f: p.value for f, _ in V._lib.VcMirrorItems._fields_})
    host = [
        ("vc_acl_classify_v4", lambda n: L.vc_acl_classify_v4(h, p, p, p, n, p, p)),
        ("vc_acl_classify_v6", lambda n: L.vc_acl_classify_v6(h, p, p, p, n, p, p)),
        ("vc_route_lookup_v4", lambda n: L.vc_route_lookup_v4(h, p, n, p)),
        ("vc_route_lookup_v6", lambda n: L.vc_route_lookup_v6(h, p, n, p)),
        ("vc_hint_search", lambda n: L.vc_hint_search(h, p, p, None, p, None, None, None, n, p)),
        ("vc_dns_classify", lambda n: L.vc_dns_classify(h, p, p, n, p, p)),
        ("vc_dns_datagrams", lambda n: L.vc_dns_datagrams(h, p, p, n, p, p, None, p,
                                                          C.byref(dn))),
        ("vc_cert_choose", lambda n: L.vc_cert_choose(h, p, p, None, n, p)),
        ("vc_source_select_v4", lambda n: L.vc_source_select_v4(h, p, p, n, 0, p)),
        ("vc_source_select_v6", lambda n: L.vc_source_select_v6(h, p, p, n, 0, p)),
        ("vc_parse_packets", lambda n: L.vc_parse_packets(h, p, p, n, 0, C.byref(pk))),
        ("vc_mirror_match", lambda n: L.vc_mirror_match(h, 0, C.byref(it), n, p)),
        ("vc_mirror_switch", lambda n: L.vc_mirror_switch(h, 0, p, p, n, 0, p)),
        ("vc_pipeline", lambda n: L.vc_pipeline(h, C.byref(pkt), n, p, 1, C.byref(po))),
        ("vc_pipeline_c6", lambda n: L.vc_pipeline_c6(h, C.byref(pkt), n, 0, p, 1,
                                                      C.byref(po))),
        ("vc_switch_classify", lambda n: L.vc_switch_classify(h, p, p, n, 0, p, p, None, 4789,
                                                              C.byref(pk), p, p, p)),
    ]
    dev = [
        ("vc_acl_classify_v4_dev", lambda n: L.vc_acl_classify_v4_dev(h, p, p, p, n, p, p, s)),
        ("vc_acl_classify_v6_dev", lambda n: L.vc_acl_classify_v6_dev(h, p, p, p, n, p, p, s)),
        ("vc_route_lookup_v4_dev", lambda n: L.vc_route_lookup_v4_dev(h, p, n, p, s)),
        ("vc_route_lookup_v6_dev", lambda n: L.vc_route_lookup_v6_dev(h, p, n, p, s)),
        ("vc_hint_search_dev", lambda n: L.vc_hint_search_dev(h, p, p, None, p, None, None, None,
                                                              n, p, s)),
        ("vc_dns_classify_dev", lambda n: L.vc_dns_classify_dev(h, p, p, n, p, p, s)),
        ("vc_dns_datagrams_dev", lambda n: L.vc_dns_datagrams_dev(h, p, p, n, p, p, None, p,
                                                                  C.byref(dn), s)),
        ("vc_cert_choose_dev", lambda n: L.vc_cert_choose_dev(h, p, p, None, n, p, s)),
        ("vc_source_select_v4_dev", lambda n: L.vc_source_select_v4_dev(h, p, p, n, 0, p, s)),
        ("vc_source_select_v6_dev", lambda n: L.vc_source_select_v6_dev(h, p, p, n, 0, p, s)),
        ("vc_parse_packets_dev", lambda n: L.vc_parse_packets_dev(h, p, p, n, 0, C.byref(pk), s)),
        ("vc_mirror_match_dev", lambda n: L.vc_mirror_match_dev(h, 0, C.byref(it), n, p, s)),
        ("vc_mirror_switch_dev", lambda n: L.vc_mirror_switch_dev(h, 0, p, p, n, 0, p, s)),
        ("vc_pipeline_dev", lambda n: L.vc_pipeline_dev(h, C.byref(pkt), n, p, 1, C.byref(po),
                                                        s, None, None)),
        ("vc_pipeline_v4_dev", lambda n: L.vc_pipeline_v4_dev(h, p, p, p, p, p, p, 1, n, p, p, p,
                                                              p, s)),
        ("vc_pipeline_c6_dev", lambda n: L.vc_pipeline_c6_dev(h, C.byref(pkt), n, 0, p, 1,
                                                              C.byref(po), s, None, None)),
        ("vc_switch_classify_dev", lambda n: L.vc_switch_classify_dev(
            h, p, p, n, 0, p, p, None, 4789, C.byref(pk), p, p, p, s)),
    ]
    return host, dev


def test_empty_and_negative_batches(clf):
    import torch
    _tables(clf)
    L = V.lib()
    buf = _Buf()
    stream = C.c_void_p(torch.cuda.current_stream().cuda_stream)
    host, _ = _calls(L, clf.h, buf.hp, stream)
    _, dev = _calls(L, clf.h, buf.dp, stream)
    assert len(host) + len(dev) == 33
    for name, call in host + dev:
        assert call(0) == VC_OK, (name, L.vc_last_error())
        assert buf.untouched(), name
        assert call(-1) == VC_EINVAL, name
        assert buf.untouched(), name
    # the context still classifies after all of them
    q = np.array([0x0A010203, 0x0B000001], np.uint32)
    np.testing.assert_array_equal(clf.route_v4(q), [0, -1])   # list order: the /8 first

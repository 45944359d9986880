"""GPU tier: vc_dns_datagrams[_dev] -- DNSServer's drain loop per datagram
(core/src/main/java/vproxy/dns/DNSServer.java:457-500) in one kernel:

    securityGroup.allow(Protocol.UDP, remote.getAddress(), remote.getPort())
    `read == 0`
    Formatter.parsePackets (base/.../dns/Formatter.java:162-372, rdata/*.java)
    isResponse / opcode / handleRequest's question classification
        (DNSServer.java:116-166)

against the hand-derived KATs (tests/golden/kats.json, TestResolver.packet's
packet among them) and the oracle's restatement (vo_dnsd_batch) over random
and mutated datagrams from IPv4 and IPv6 senders.
"""
import random

import numpy as np
import pytest

import dnswire as DW
import oracle_ffi as O
import vproxy_amd as V
from vproxy_amd import workloads as W

from cases import rule_row
from test_dnsd_cpu import check_against_kats, kat_inputs, kats, udp_rules

pytestmark = pytest.mark.gpu


def _compile_acl(clf, tcp, udp, dflt):
    a, na, ka = W.as_ctypes(tcp, V._lib.VcAclRule)
    b, nb, kb = W.as_ctypes(udp, V._lib.VcAclRule)
    V.check(V.lib().vc_compile_acl(clf.h, a, na, b, nb, 1 if dflt else 0))


def _same(got, want, nq_from="want"):
    """status / acl / nq equal everywhere; qtype / kind / value for q < nq"""
    for k in ("status", "acl", "nq"):
        np.testing.assert_array_equal(np.asarray(got[k]), want[k], err_msg=k)
    live = np.arange(V.DNSD_MAXQ)[None, :] < want["nq"][:, None]
    for k in ("qtype", "kind", "value"):
        g = np.asarray(got[k]).astype(want[k].dtype)
        np.testing.assert_array_equal(np.where(live, g, 0), want[k], err_msg=k)


def _cpu(res):
    return {k: v.cpu().numpy() for k, v in res.items()}


def test_dns_datagram_kats():
    import torch
    k = kats()
    clf = V.Classifier(0)
    try:
        _compile_acl(clf, np.zeros(0, W.RULE_DT), udp_rules(k["udp_rules"]), k["default_allow"])
        clf.compile_upstream(k["groups"])
        clf.compile_hosts([tuple(x) for x in k["hosts"]])
        cases, blob, off, fam, r4, r6, port = kat_inputs(k)
        res = clf.dns_datagrams((blob, off), r4, port, remote6=r6, remote_family=fam)
        check_against_kats(res, cases)
        T = lambda x: torch.from_numpy(np.ascontiguousarray(x)).cuda()
        dres = _cpu(clf.dns_datagrams((T(blob), T(off.view(np.int32))), T(r4.view(np.int32)),
                                      T(port.view(np.int16)), remote6=T(r6),
                                      remote_family=T(fam)))
        dres["qtype"] = dres["qtype"].view(np.uint16)
        check_against_kats(dres, cases)
    finally:
        clf.close()


def _remotes(rng, n):
    fam = np.where(rng.random(n) < 0.75, 4, 6).astype(np.uint8)
    base = rng.choice(np.array([0x0A000000, 0x0A010000, 0xC0A80000, 0x08080000], np.uint64), n)
    r4 = (base | rng.integers(0, 1 << 16, n).astype(np.uint64)).astype(np.uint32)
    r6 = np.zeros((n, 16), np.uint8)
    k = rng.integers(0, 2, n)
    r6[k == 0, 10:12] = 0xFF                         # ::ffff:a.b.c.d
    r6[k == 0, 12:] = W.v4_to_bytes(r4)[k == 0]
    r6[k == 1, :4] = [0x20, 0x01, 0x0D, 0xB8]
    r6[:, 14:] = rng.integers(0, 256, (n, 2))
    port = np.where(rng.random(n) < 0.9, 53, rng.integers(0, 65536, n)).astype(np.uint16)
    return fam, r4, r6, port


@pytest.mark.parametrize("shift", [0, 1])
def test_dns_datagrams_vs_oracle(shift):
    """Random queries over group / hosts / literal / internal / unknown names
    (1-5 questions, compression pointers, OPT and answer records), a quarter
    of them mutated (flipped byte, truncated, extended); shift 1 puts the
    blob at an odd address (the unstaged kernel)."""
    import torch
    rng = np.random.default_rng(23)
    prng = random.Random(29)
    clf = V.Classifier(0)
    try:
        udp = np.concatenate([rule_row(*r) for r in (
            ("10.0.0.0/8", 0, 65535, False), ("8.8.0.0/16", 53, 53, True),
            ("0.0.0.0/0", 1000, 2000, False), ("::ffff:192.168.0.0/112", 0, 65535, False),
            ("2001:db8::/32", 0, 52, False))])
        tcp = np.concatenate([rule_row("0.0.0.0/0", 0, 65535, False)])
        _compile_acl(clf, tcp, udp, True)
        groups, ghosts = W.gen_groups(3000, 41)
        clf.compile_upstream(groups)
        hosts = [(h + ".", i) for i, h in enumerate(ghosts[:40])] + [("localhost.", 900)]
        clf.compile_hosts(hosts)
        names = W.gen_hostnames(ghosts, 4000, 42, dns=True)
        names += [b"1.2.3.4.", b"::1.", b"x.vproxy.local.", b"nope.org.", b"caf\xe9.com.",
                  b"localhost.", b"."]
        dg = [DW.random_datagram(prng, names) for _ in range(60013)]
        dg += [DW.reference_packet(True), DW.reference_packet(False), b""]
        n = len(dg)
        fam, r4, r6, port = _remotes(rng, n)
        blob, off = W.pack(dg)
        want = O.dnsd_batch_np(tcp, udp, True, hosts, groups, blob, off, fam, r4, r6, port,
                               nthreads=16)
        st = want["status"]
        for s in range(7):
            assert (st == s).sum() > 0, s          # every outcome occurs
        # device entry point (blob shifted by `shift` bytes)
        T = lambda x: torch.from_numpy(np.ascontiguousarray(x)).cuda()
        dblob = torch.zeros(len(blob) + 16, dtype=torch.uint8, device="cuda")
        dblob[shift:shift + len(blob)] = T(blob)
        clf.counters_enable(True)
        clf.counters_reset()
        res = _cpu(clf.dns_datagrams((dblob[shift:], T(off.view(np.int32))),
                                     T(r4.view(np.int32)), T(port.view(np.int16)),
                                     remote6=T(r6), remote_family=T(fam)))
        torch.cuda.synchronize()
        clf.counters_enable(False)
        res["qtype"] = res["qtype"].view(np.uint16)
        _same(res, want)
        # the unevaluated question slots read kind 0
        live = np.arange(V.DNSD_MAXQ)[None, :] < want["nq"][:, None]
        assert not res["kind"][~live].any()
        # hit counters: the UDP rule of every datagram ([tcp][udp][tcp dflt][udp dflt])
        # and the group of every question classified VC_DNS_GROUP
        nt, nu = len(tcp), len(udp)
        acl_bins = np.where(want["acl"] >= 0, nt + want["acl"], nt + nu + 1)
        np.testing.assert_array_equal(clf.counters_read(V.COUNTERS_ACL),
                                      np.bincount(acl_bins, minlength=nt + nu + 2))
        g = want["value"][live & (want["kind"] == V.DNS_GROUP)]
        np.testing.assert_array_equal(clf.counters_read(V.COUNTERS_GROUP),
                                      np.bincount(g, minlength=len(groups) + 1))
        # the host entry point gives the same
        _same(clf.dns_datagrams((blob, off), r4, port, remote6=r6, remote_family=fam), want)
    finally:
        clf.close()


def test_dns_datagrams_bad_arguments():
    import ctypes as C
    clf = V.Classifier(0)
    try:
        one = C.c_void_p(1)
        o = V._lib.VcDnsdOut()                          # no status / kind / value arrays
        rc = V.lib().vc_dns_datagrams_dev(clf.h, one, one, 1, None, one, None, one,
                                          C.byref(o), None)
        assert rc != 0                                  # EINVAL, nothing launched
        rc = V.lib().vc_dns_datagrams(clf.h, None, None, 1, None, None, None, None, C.byref(o))
        assert rc != 0
    finally:
        clf.close()


def test_dns_datagrams_deferred_over_slot_reuse():
    """The drain-loop kernel leaves datagrams with a question it does not
    finish inline (a possible IP literal, bytes >= 0x80, a name the host scan
    does not cover) to a second kernel, counted in the launch's ticket slot,
    which that kernel resets.  Over 4200 launches (every slot reused) of
    batches with and without such datagrams, on two streams, every result
    equals the oracle's."""
    import torch
    prng = random.Random(31)
    rng = np.random.default_rng(37)
    clf = V.Classifier(0)
    try:
        udp = np.concatenate([rule_row(*r) for r in (
            ("10.0.0.0/8", 0, 65535, False), ("0.0.0.0/0", 0, 65535, True))])
        tcp = np.zeros(0, W.RULE_DT)
        _compile_acl(clf, tcp, udp, True)
        groups, ghosts = W.gen_groups(1000, 43)
        clf.compile_upstream(groups)
        hosts = [(h + ".", i) for i, h in enumerate(ghosts[:20])]
        clf.compile_hosts(hosts)
        plain = W.gen_hostnames(ghosts, 2000, 44, dns=True)
        odd = plain + [b"1.2.3.4.", b"::1.", b"fe80::1.", b"dead.beef.", b"caf\xe9.com.",
                       b"a.b.c.d.e.f.g.h.i.j.k."] * 40
        T = lambda x: torch.from_numpy(np.ascontiguousarray(x)).cuda()
        sets = []
        for names in (plain, odd):
            dg = [DW.random_datagram(prng, names) for _ in range(3000)]
            fam, r4, r6, port = _remotes(rng, len(dg))
            blob, off = W.pack(dg)
            want = O.dnsd_batch_np(tcp, udp, True, hosts, groups, blob, off, fam, r4, r6, port,
                                   nthreads=16)
            dev = ((T(blob), T(off.view(np.int32))), T(r4.view(np.int32)),
                   T(port.view(np.int16)), T(r6), T(fam))
            sets.append((want, dev))
        sizes = [1, 65, 1025, 3000]
        streams = [torch.cuda.Stream(), torch.cuda.Stream()]
        keep = []
        for k in range(4200):
            n = sizes[k % len(sizes)]
            which = (k // len(sizes)) % 2
            want, ((b, o), r4d, pd, r6d, fd) = sets[which]
            with torch.cuda.stream(streams[k % 2]):
                res = clf.dns_datagrams((b, o[:n + 1]), r4d[:n], pd[:n], remote6=r6d[:n],
                                        remote_family=fd[:n])
            if k % 300 < 8 or k >= 4192:
                keep.append((n, which, res))
        torch.cuda.synchronize()
        for n, which, res in keep:
            got = _cpu(res)
            got["qtype"] = got["qtype"].view(np.uint16)
            want = {kk: v[:n] for kk, v in sets[which][0].items()}
            _same(got, want)
    finally:
        clf.close()


def test_dns_datagram_qname_lengths():
    """Decoded qnames of 1 .. 140 chars, around the deferring kernel's
    96-char buffers (longer names go to dnsd_defer_kernel, whose buffers
    hold 128) and the contract's 128 (longer: VC_DNSD_HOST, the Java path):
    hint-host, hosts-file and unknown names of every length, one and two
    questions, through the staged and unstaged kernels, equal to the oracle."""
    import torch
    rng = np.random.default_rng(31)
    clf = V.Classifier(0)
    try:
        tcp = np.concatenate([rule_row("0.0.0.0/0", 0, 65535, False)])
        udp = np.concatenate([rule_row("0.0.0.0/0", 0, 65535, True)])
        _compile_acl(clf, tcp, udp, True)

        def label_name(total):
            """a dotted name of exactly `total` chars, trailing dot included
            (30-char labels)"""
            c = list("".join(rng.choice(list("abcdefghij"), total - 1)))
            for p in range(30, total - 2, 31):
                c[p] = "."
            return "".join(c) + "."
        names = [label_name(L) for L in range(2, 141)]
        assert all(len(n) == L for n, L in zip(names, range(2, 141)))
        groups = [({}, {"host": n.rstrip(".")}) for n in names[::3]]
        hosts = [(n, 100 + i) for i, n in enumerate(names[1::3])]
        clf.compile_upstream(groups)
        clf.compile_hosts(hosts)
        dg = []
        for n in names:
            dg.append(DW.query([(n, DW.A)]))
            dg.append(DW.query([("x.org.", DW.A), (n, DW.AAAA)]))
        N = len(dg)
        fam = np.full(N, 4, np.uint8)
        r4 = np.full(N, 0x08080808, np.uint32)
        r6 = np.zeros((N, 16), np.uint8)
        port = np.full(N, 53, np.uint16)
        blob, off = W.pack(dg)
        want = O.dnsd_batch_np(tcp, udp, True, hosts, groups, blob, off, fam, r4, r6, port)
        lens = np.array([len(n) - 1 for n in names])
        assert (lens > 96).sum() > 20 and (lens > 128).sum() > 5
        T = lambda x: torch.from_numpy(np.ascontiguousarray(x)).cuda()
        for shift in (0, 1):
            dblob = torch.zeros(len(blob) + 16, dtype=torch.uint8, device="cuda")
            dblob[shift:shift + len(blob)] = T(blob)
            res = _cpu(clf.dns_datagrams((dblob[shift:], T(off.view(np.int32))),
                                         T(r4.view(np.int32)), T(port.view(np.int16)),
                                         remote6=T(r6), remote_family=T(fam)))
            res["qtype"] = res["qtype"].view(np.uint16)
            _same(res, want)
        st = want["status"]
        assert (st == V.DNSD_HOST).sum() > 0 and (st == V.DNSD_ANSWER).sum() > 0
    finally:
        clf.close()

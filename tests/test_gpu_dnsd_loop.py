"""GPU tier: DNSServer's drain loop (DNSServer.java:457-500) batched through
vc_dns_datagrams by the batcher of jni/DnsDrainBatcher.java, replayed in C
(tests/native/dnsd_loop.c).  Over a queue of random, mutated, empty,
response and rejected datagrams, at batch sizes from 1 to the whole queue,
its action trace equals the reference loop's (dnsd_loop.reference_trace
over the oracle's per-datagram outcome): REJECTED / RESPONSE skipped,
EMPTY / MALFORMED end the readable event at that datagram with the rest
handled by the next, HOST handed to the Java body, ANSWER with every
question's kind and value; and a device failure part-way sends the rest of
the queue down the Java path."""
import random

import numpy as np
import pytest

import dnsd_loop as L
import dnswire as DW
import oracle_ffi as O
import vproxy_amd as V
from vproxy_amd import workloads as W

from cases import rule_row

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def setup():
    rng = np.random.default_rng(31)
    prng = random.Random(37)
    clf = V.Classifier(0)
    udp = np.concatenate([rule_row(*r) for r in (
        ("10.0.0.0/8", 0, 65535, False), ("8.8.0.0/16", 53, 53, True),
        ("0.0.0.0/0", 1000, 2000, False))])
    tcp = np.concatenate([rule_row("0.0.0.0/0", 0, 65535, False)])
    a, na, ka = W.as_ctypes(tcp, V._lib.VcAclRule)
    b, nb, kb = W.as_ctypes(udp, V._lib.VcAclRule)
    V.check(V.lib().vc_compile_acl(clf.h, a, na, b, nb, 1))
    groups, ghosts = W.gen_groups(500, 43)
    clf.compile_upstream(groups)
    hosts = [(h + ".", i) for i, h in enumerate(ghosts[:20])]
    clf.compile_hosts(hosts)
    names = W.gen_hostnames(ghosts, 500, 44, dns=True) + [b"1.2.3.4.", b"x.vproxy.local.",
                                                          b"nope.org."]
    dg = [DW.random_datagram(prng, names) for _ in range(3000)]
    for i in range(0, 3000, 97):
        dg[i] = b""                                   # read == 0
    dg += [DW.reference_packet(True), DW.reference_packet(False)]
    n = len(dg)
    fam = np.full(n, 4, np.uint8)
    r4 = rng.choice(np.array([0x0A000001, 0x08080808, 0xC0A80001], np.uint32), n)
    r6 = np.zeros((n, 16), np.uint8)
    port = np.where(rng.random(n) < 0.9, 53, 1500).astype(np.uint16)
    blob, off = W.pack(dg)
    want = O.dnsd_batch_np(tcp, udp, True, hosts, groups, blob, off, fam, r4, r6, port,
                           nthreads=16)
    for s in range(7):
        assert (want["status"] == s).sum() > 0, s
    yield clf, (blob, off, fam, r4, r6, port), want
    clf.close()


@pytest.mark.parametrize("batch", [1, 7, 64, 1000, 5000])
def test_trace_equals_reference_loop(setup, batch):
    clf, q, want = setup
    got = L.trace(clf.h, *q, batch=batch)
    ref = L.reference_trace(want)
    assert got == ref, next(i for i, (a, b) in enumerate(zip(got, ref)) if a != b)


def test_device_failure_midway_takes_the_java_path(setup):
    clf, q, want = setup
    got = L.trace(clf.h, *q, batch=256, inject=[0, 0, L.EDEVICE])
    ref = L.reference_trace(want)
    # the first two batches as the reference (up to where batch 3 starts), then Java
    cut = got.index("D")
    assert got[:cut] == ref[:cut]
    rest = got[cut + 1:]
    assert rest[0::2] == ["J"] * (len(rest) // 2)
    assert int(rest[-1]) == len(want["status"]) - 1

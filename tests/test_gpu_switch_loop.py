"""GPU tier: the vswitch's UDP drain loop (Switch.java:744-776 with
handleNetworkAndGetVXLanPacket :643-731) batched through vc_switch_classify
by the batcher of jni/SwitchDrainBatcher.java, replayed in C
(tests/native/switch_loop.c).  Over a queue of the parse-chain frames of
tests/cases.py (every layer, malformed and truncated shapes, parser
exceptions), user-iface datagrams (the test's stand-in for
VProxyEncryptedPacket.from succeeding), empty reads and IPv4 / IPv6 senders,
at batch sizes from 1 to the whole queue, the action trace equals the
reference loop's (switch_loop.reference_trace over the oracle's allow,
parse status and inner route per datagram): decrypted -> handleEncrypted,
denied -> dropped, parse error -> dropped, parser exception -> the Java
body, parsed -> handleBare with the route; and a device failure part-way
sends the rest of the bare datagrams down the Java path."""
import numpy as np
import pytest

import oracle_ffi as O
import switch_loop as L
import vproxy_amd as V
from vproxy_amd import workloads as W

from cases import gen_frames
from test_gpu_switch import BIND_PORT, _nets, _remotes, _rules

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def setup():
    rng = np.random.default_rng(91)
    clf = V.Classifier(0)
    tcp, udp = _rules(rng)
    a, na, ka = W.as_ctypes(tcp, V._lib.VcAclRule)
    b, nb, kb = W.as_ctypes(udp, V._lib.VcAclRule)
    V.check(V.lib().vc_compile_acl(clf.h, a, na, b, nb, 0))
    nets4, nets6 = _nets(rng, 2000, 1000)
    ra, rn, rk = W.as_ctypes(nets4, V._lib.VcNet)
    rb, rbn, rbk = W.as_ctypes(nets6, V._lib.VcNet)
    clf.compile_routes_raw(ra, rn, rb, rbn)
    frames = gen_frames(rng, 6000)
    for i in range(0, len(frames), 409):
        frames[i] = b""                               # a 0-byte read ends the event
    n = len(frames)
    fam, r4, r6 = _remotes(rng, n)
    decrypt = (rng.random(n) < 0.1).astype(np.uint8)
    blob, off = W.pack(frames)
    # the oracle's outcome per datagram
    proto = np.full(n, 17, np.uint8)
    ports = np.full(n, BIND_PORT, np.uint16)
    _, a4 = O.sg_batch_v4_np(tcp, udp, False, proto, r4, ports)
    _, a6 = O.sg_batch_v6_np(tcp, udp, False, proto, np.ascontiguousarray(r6), ports)
    allow = np.where(fam == 6, a6, a4)
    status = np.zeros(n, np.int32)
    route = np.full(n, -1, np.int32)
    for i, f in enumerate(frames):
        if not f:
            continue
        p = O.parse_packet(f, V.LAYER_VXLAN)
        status[i] = p["status"]
        if not allow[i] or p["status"] != 0 or p["l3"] not in (4, 6):
            continue
        dst = bytes.fromhex(p["dst"])
        if p["l3"] == 4:
            route[i] = O.rt_batch_v4_np(nets4, np.frombuffer(dst, ">u4").astype(np.uint32))[0]
        else:
            route[i] = O.rt_batch_v6_np(nets6, np.frombuffer(dst, np.uint8).reshape(1, 16))[0]
    lens = np.diff(off.astype(np.int64))
    want = L.reference_trace(lens, decrypt, allow, status, route)
    acts = set(want[0::1])
    for a_ in ("E", "S", "X", "J", "B", "|"):
        assert a_ in acts, a_
    yield clf, (blob, off, decrypt, fam, r4, r6), want
    clf.close()


@pytest.mark.parametrize("batch", [1, 7, 64, 1000, 8000])
def test_trace_equals_reference_loop(setup, batch):
    clf, q, want = setup
    got = L.trace(clf.h, *q, BIND_PORT, batch=batch)
    assert got == want, next(i for i, (a, b) in enumerate(zip(got, want)) if a != b)


def test_device_failure_midway_takes_the_java_path(setup):
    clf, q, want = setup
    got = L.trace(clf.h, *q, BIND_PORT, batch=256, inject=[0, 0, L.EDEVICE])
    cut = got.index("D")
    assert got[:cut] == want[:cut]
    # after it: decrypted datagrams still go to handleEncrypted, bare ones to Java
    rest = [x for x in got[cut + 1:] if x != "|"]
    acts = rest[0::2]
    assert set(acts) <= {"E", "J"} and "J" in acts
    decrypt = q[2]
    for a_, i in zip(acts, rest[1::2]):
        assert (a_ == "E") == bool(decrypt[int(i)])

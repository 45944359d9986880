"""GPU tier: the plain C99 consumer (tests/native/abi_c.c) on the MI355X.

The binary runs the JNI shim's call sequence through the C ABI (control-
plane mirrors, registered and pageable host batches, the mixed-family host
pipeline, counters and the Prometheus size-query protocol) and dumps its
rules, inputs and outputs.  Here the same work goes through the ctypes path
and the oracle; everything must agree bit for bit, and the Prometheus text
must be identical.
"""
import subprocess

import numpy as np
import pytest

import oracle_ffi as O
import vproxy_amd as V
from vproxy_amd import workloads as W
from test_abi_c import build_abi_c

pytestmark = pytest.mark.gpu


def _read(path):
    raw = open(path, "rb").read()
    assert raw[:8] == b"VCABI1\0\0"
    pos = 8
    n = int(np.frombuffer(raw, np.int64, 1, pos)[0])
    pos += 8
    rsz, nsz, n_tcp, n_udp, n4, n6 = np.frombuffer(raw, np.int32, 6, pos)
    pos += 24
    assert rsz == W.RULE_DT.itemsize and nsz == W.NET_DT.itemsize

    def take(dt, count, shape=None):
        nonlocal pos
        a = np.frombuffer(raw, dt, count, pos).copy()
        pos += a.nbytes
        return a.reshape(shape) if shape else a

    d = {"n": n}
    d["tcp"], d["udp"] = take(W.RULE_DT, n_tcp), take(W.RULE_DT, n_udp)
    d["v4"], d["v6"] = take(W.NET_DT, n4), take(W.NET_DT, n6)
    d["proto"], d["src4"] = take(np.uint8, n), take(np.uint32, n)
    d["port"], d["dst4"] = take(np.uint16, n), take(np.uint32, n)
    d["family"] = take(np.uint8, n)
    d["src6"], d["dst6"] = take(np.uint8, n * 16, (n, 16)), take(np.uint8, n * 16, (n, 16))
    d["idx"], d["allow"], d["route"] = take(np.int32, n), take(np.uint8, n), take(np.int32, n)
    d["p_acl"], d["p_route"], d["p_allow"] = take(np.int32, n), take(np.int32, n), take(np.uint8, n)
    nc = int(take(np.int64, 1)[0])
    d["acl_cnt"] = take(np.uint64, nc)
    ln = int(take(np.int64, 1)[0])
    d["prom"] = raw[pos:pos + ln].decode()
    assert pos + ln == len(raw)
    return d


def test_abi_c_sequence_matches_ctypes_and_oracle(tmp_path):
    out = tmp_path / "abi.bin"
    r = subprocess.run([build_abi_c(), str(out)], capture_output=True, text=True, timeout=180)
    assert r.returncode == 0, r.stdout + r.stderr
    d = _read(out)
    # oracle: SecurityGroup.allow and RouteTable.lookup on the dumped lists
    want, wv = O.sg_batch_v4_np(d["tcp"], d["udp"], False, d["proto"], d["src4"], d["port"],
                                nthreads=8)
    np.testing.assert_array_equal(d["idx"], want)
    np.testing.assert_array_equal(d["allow"], wv)
    np.testing.assert_array_equal(d["route"], O.rt_batch_v4_np(d["v4"], d["dst4"], nthreads=8))
    six = d["family"] == 6
    w6, wv6 = O.sg_batch_v6_np(d["tcp"], d["udp"], False, d["proto"][six], d["src6"][six],
                               d["port"][six], nthreads=8)
    np.testing.assert_array_equal(d["p_acl"][six], w6)
    np.testing.assert_array_equal(d["p_allow"][six], wv6)
    np.testing.assert_array_equal(d["p_route"][six],
                                  O.rt_batch_v6_np(d["v6"], d["dst6"][six], nthreads=8))
    np.testing.assert_array_equal(d["p_acl"][~six], d["idx"][~six])
    # the same sequence through ctypes: identical outputs, counters and text
    clf = V.Classifier(0)
    try:
        a, na, ka = W.as_ctypes(d["tcp"], V._lib.VcAclRule)
        b, nb, kb = W.as_ctypes(d["udp"], V._lib.VcAclRule)
        V.check(V.lib().vc_compile_acl(clf.h, a, na, b, nb, 0))
        ra, rn, rk = W.as_ctypes(d["v4"], V._lib.VcNet)
        rb, rbn, rbk = W.as_ctypes(d["v6"], V._lib.VcNet)
        clf.compile_routes_raw(ra, rn, rb, rbn)
        clf.counters_enable(True)
        for _ in range(2):
            idx, allow = clf.acl_v4(d["proto"], d["src4"], d["port"])
            route = clf.route_v4(d["dst4"])
        np.testing.assert_array_equal(idx, d["idx"])
        np.testing.assert_array_equal(allow, d["allow"])
        np.testing.assert_array_equal(route, d["route"])
        pa, pr, pg, pal = clf.pipeline(d["proto"], d["src4"], d["dst4"], d["port"],
                                       family=d["family"], src6=d["src6"], dst6=d["dst6"],
                                       want_allow=True)
        np.testing.assert_array_equal(pa, d["p_acl"])
        np.testing.assert_array_equal(pr, d["p_route"])
        np.testing.assert_array_equal(pal, d["p_allow"])
        assert np.all(pg == -1)
        np.testing.assert_array_equal(clf.counters_read(V.COUNTERS_ACL), d["acl_cnt"])
        assert clf.counters_prometheus("host=gpu0") == d["prom"]
    finally:
        clf.close()


def test_jni_shim_on_gpu():
    """The JNI shim under a fake JNIEnv (tests/native/jni_harness.c) against
    the C ABI called directly: ACL, routes, per-VNI routes and two
    compileUpstream calls from one groups buffer, HTTP request heads and
    source hashing give identical results."""
    import os
    native = os.path.join(os.path.dirname(os.path.abspath(__file__)), "native")
    exe = os.path.join(native, "build", "jni_harness")
    if not os.path.exists(exe):
        subprocess.check_call(["make", "-s", "-C", native, "build/jni_harness"])
    r = subprocess.run([exe, "gpu"], capture_output=True, text=True, timeout=120)
    assert r.returncode == 0 and "JNI OK" in r.stdout, r.stdout + r.stderr

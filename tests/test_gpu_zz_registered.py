"""GPU tier, run last: zero-copy over page-locked caller buffers
(vc_host_register / vc_host_unregister, capi.cpp `mapped`), and a
regression test for the host-buffer path after registrations.

Round 2's driver run stopped at an illegal-address error raised by the
staging copy of vc_parse_packets (a pageable H2D hipMemcpyAsync into a
stream-ordered pool allocation), in a process that had registered and
unregistered large NumPy arrays earlier.  The host entry points no longer
DMA from caller memory or allocate from a stream-ordered pool (capi.cpp
Stager: library-owned device arenas and page-locked bounce buffers); this
module keeps the registered-buffer tests after every other GPU module and
checks that calls on freshly allocated pageable arrays, some of them in
address ranges that were registered moments before, stay correct."""
import gc

import numpy as np
import pytest

import oracle_ffi as O
import vproxy_amd as V
from cases import gen_frames
from test_gpu_hostpath import N, check_vs_oracle, tables
from test_gpu_pipeline import host_entry_point_equals_device, setup  # noqa: F401 (fixture)

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def clf():
    c = V.Classifier(0)
    yield c
    c.close()


def _register(arrs):
    for x in arrs:
        V.check(V.lib().vc_host_register(x.ctypes.data, x.nbytes))


def _unregister(arrs):
    for x in arrs:
        V.check(V.lib().vc_host_unregister(x.ctypes.data))


def test_registered_zero_copy(clf):
    t = tables(clf, 71)
    outs = dict(idx=np.empty(N, np.int32), allow=np.empty(N, np.uint8),
                rt=np.empty(N, np.int32), sv=np.empty(N, np.int32))
    ins = [t[k] for k in ("proto", "src", "port", "dst", "grp")]
    _register(ins)
    try:
        idx, allow = clf.acl_v4(t["proto"], t["src"], t["port"])
        rt = clf.route_v4(t["dst"])
        sv = clf.source_select(t["grp"], t["src"])
    finally:
        _unregister(ins)
    check_vs_oracle(t, idx, allow, rt, sv, 72)
    del outs


def test_pipeline_registered(setup):  # noqa: F811
    host_entry_point_equals_device(*setup, registered=True)


def test_pageable_after_unregister(clf):
    """Register, use and unregister large arrays, free them, then classify
    and parse from new pageable arrays of the same sizes (which the
    allocator may place in the released ranges): every result checked
    against the oracle."""
    for rnd in range(3):
        t = tables(clf, 80 + rnd)
        ins = [t[k] for k in ("proto", "src", "port", "dst", "grp")]
        _register(ins)
        try:
            clf.acl_v4(t["proto"], t["src"], t["port"])
            clf.route_v4(t["dst"])
        finally:
            _unregister(ins)
        del ins, t
        gc.collect()
        t = tables(clf, 90 + rnd)                     # fresh pageable arrays
        idx, allow = clf.acl_v4(t["proto"], t["src"], t["port"])
        rt = clf.route_v4(t["dst"])
        sv = clf.source_select(t["grp"], t["src"])
        check_vs_oracle(t, idx, allow, rt, sv, 100 + rnd)
        frames = gen_frames(np.random.default_rng(110 + rnd), 20000)
        res = clf.parse_packets(frames, 0)
        for i in range(0, len(frames), 97):
            w = O.parse_packet(frames[i], 0)
            assert int(res["status"][i]) == w["status"] and int(res["l3"][i]) == w["l3"], i
        ok = (res["status"] == 0) & (res["l3"] == 4) & (res["l4"] == 6)
        got, gv = clf.acl_v4(res["proto"][ok], res["src4"][ok], res["dport"][ok])
        want, wv = O.sg_batch_v4_np(t["tcp"], t["udp"], False, res["proto"][ok],
                                    res["src4"][ok], res["dport"][ok])
        np.testing.assert_array_equal(got, want)
        np.testing.assert_array_equal(gv, wv)

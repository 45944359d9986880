"""GPU tier: snapshot pins (include/vclassify.h "Snapshot pins").

A pin keeps the snapshots that were current when it was taken; bound to a
thread it is what that thread's calls classify against, while other threads
and unbound calls see every later compile -- the copy-on-write behaviour of
SecurityGroup.java:56-103 / Upstream.java:146-157, where a reader holding
the old list keeps reading it.  Generations grow by one per publish.
"""
import threading

import numpy as np
import pytest

import vproxy_amd as V
from vproxy_amd import _lib as L

pytestmark = pytest.mark.gpu


def _acl(clf, allow_first):
    clf.compile_acl([("10.0.0.0/8", 0, 65535, allow_first), ("0.0.0.0/0", 80, 80, True)],
                    [("0.0.0.0/0", 0, 65535, False)], False)


def test_pin_keeps_its_snapshot():
    clf = V.Classifier(0)
    try:
        with pytest.raises(V.StateError):
            with clf.pin():                       # nothing compiled: pinned empty
                clf.acl_v4(np.array([6], np.uint8), np.array([0x0A000001], np.uint32),
                           np.array([80], np.uint16))
        _acl(clf, True)
        g1 = clf.generation(L.SNAP_ACL)
        p = clf.pin()
        assert p.generation(L.SNAP_ACL) == g1 > 0
        assert p.generation(L.SNAP_ROUTE) == 0          # no routes compiled
        clf.compile_routes(["10.0.0.0/8"])
        _acl(clf, False)
        g2 = clf.generation(L.SNAP_ACL)
        assert g2 > clf.generation(L.SNAP_ROUTE) > g1
        proto = np.array([6, 6, 17], np.uint8)
        src = np.array([0x0A000001, 0x0B000001, 0x0A000001], np.uint32)
        port = np.array([22, 80, 53], np.uint16)
        idx_new, allow_new = clf.acl_v4(proto, src, port)
        with p:
            idx_old, allow_old = clf.acl_v4(proto, src, port)
            # the pin holds no route snapshot: routes are VC_ESTATE through it
            with pytest.raises(V.StateError):
                clf.route_v4(np.array([0x0A000001], np.uint32))
            seen = {}
            t = threading.Thread(target=lambda: seen.update(
                r=clf.acl_v4(proto, src, port)))          # another thread is not bound
            t.start()
            t.join()
        assert list(idx_old) == list(idx_new) == [0, 1, 0]
        assert list(allow_old) == [1, 1, 0] and list(allow_new) == [0, 1, 0]
        assert list(seen["r"][1]) == [0, 1, 0]
        # a pin of only the route kind leaves the ACL current
        q = clf.pin(1 << L.SNAP_ROUTE)
        _acl(clf, True)
        with q:
            assert list(clf.acl_v4(proto, src, port)[1]) == [1, 1, 0]
            assert list(clf.route_v4(np.array([0x0A000001, 0x0B000001], np.uint32))) == [0, -1]
        with pytest.raises(V.IllegalArgumentException):
            q.generation(L.SNAP_ACL)                      # not pinned
        p.release()
        q.release()
        # bound pins are gone with their release; unbound calls see the current tables
        assert list(clf.acl_v4(proto, src, port)[1]) == [1, 1, 0]
    finally:
        clf.close()


def test_pin_of_another_context_is_refused():
    a, b = V.Classifier(0), V.Classifier(0)
    try:
        _acl(a, True)
        p = a.pin()
        with pytest.raises(V.IllegalArgumentException):
            V.check(V.lib().vc_pin_bind(b.h, p.h))
        p.release()
    finally:
        a.close()
        b.close()


def test_pinned_snapshots_are_freed_after_release():
    """A pin keeps its snapshot's device tables alive across recompiles,
    and they go once it is released: after nine recompiles of a 200k-rule
    route table (each image tens of MB) under a pin held all along, the
    device memory in use comes back to about one table image above the
    start once the pin is released and the next compile frees the
    graveyard (capi.cpp: a replaced snapshot's buffers are freed by the
    control thread, never by the thread that drops the last pin)."""
    import torch
    from vproxy_amd import workloads as W
    net, plen = W.gen_v4_prefixes(200_000, 5)
    a = [W.v4_nets(net, plen), W.v4_nets(net[::-1].copy(), plen[::-1].copy())]
    arrs = [W.as_ctypes(x, V._lib.VcNet) for x in a]
    clf = V.Classifier(0)
    try:
        torch.cuda.synchronize()
        free0 = torch.cuda.mem_get_info()[0]
        clf.compile_routes_raw(arrs[0][0], arrs[0][1], None, 0)
        q = np.random.default_rng(6).integers(0, 2**32, 100000, dtype=np.uint64).astype(np.uint32)
        want = clf.route_v4(q)
        p = clf.pin(1 << L.SNAP_ROUTE)
        for k in range(9):                                     # the last one: table 1
            clf.compile_routes_raw(arrs[(k + 1) % 2][0], arrs[(k + 1) % 2][1], None, 0)
        with p:
            np.testing.assert_array_equal(clf.route_v4(q), want)     # the pinned table
        assert (clf.route_v4(q) != want).mean() > 0.5               # the current one differs
        torch.cuda.synchronize()
        held = free0 - torch.cuda.mem_get_info()[0]
        p.release()
        clf.compile_routes_raw(arrs[0][0], arrs[0][1], None, 0)     # frees the graveyard
        torch.cuda.synchronize()
        after = free0 - torch.cuda.mem_get_info()[0]
        assert held > 0 and after < held, (held, after)
        assert after < 0.75 * held or held - after > (16 << 20), (held, after)
    finally:
        clf.close()


def test_switch_port_image_on_a_pinned_snapshot():
    """The bind-port ACL image (AclPortImage) is built on the first switch
    call with a port for the snapshot the call uses: through a pin of an old
    SecurityGroup, a new port builds that old list's image (and the current
    snapshot gets its own), each call answering by its own list."""
    import torch
    clf = V.Classifier(0)
    try:
        clf.compile_routes(["10.0.0.0/8", "0.0.0.0/0"])
        clf.compile_acl([], [("10.0.0.0/8", 4789, 4789, True), ("0.0.0.0/0", 0, 65535, False)],
                        False)
        p = clf.pin()
        clf.compile_acl([], [("10.0.0.0/8", 53, 53, True), ("0.0.0.0/0", 4789, 4789, True)],
                        False)
        # one IPv4/UDP VXLAN datagram, senders 10.0.0.1 and 11.0.0.1
        inner = bytes([0x45, 0, 0, 28, 0, 0, 0, 0, 64, 17, 0, 0, 10, 0, 0, 2, 10, 0, 0, 3]) + \
            bytes([0, 1, 0, 2, 0, 8, 0, 0])
        frame = bytes([8, 0, 0, 0, 0, 0, 1, 0]) + bytes(12) + b"\x08\x00" + inner
        blob = torch.tensor(list(frame * 2), dtype=torch.uint8, device="cuda")
        off = torch.tensor([0, len(frame), 2 * len(frame)], dtype=torch.int32, device="cuda")
        r4 = torch.tensor([0x0A000001, 0x0B000001], dtype=torch.int32, device="cuda")

        def verdicts(port):
            _, acl, allow, _ = clf.switch_classify((blob, off), r4, port)
            torch.cuda.synchronize()
            return acl.cpu().tolist(), allow.cpu().tolist()
        for port in (4789, 53, 4789):
            with p:                                    # the old list
                assert verdicts(port) == ({4789: ([0, 1], [1, 0]), 53: ([1, 1], [0, 0])}[port])
            # the current list
            assert verdicts(port) == ({4789: ([1, 1], [1, 1]), 53: ([0, -1], [1, 0])}[port])
        p.release()
    finally:
        clf.close()

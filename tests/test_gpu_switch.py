"""GPU tier: vc_switch_classify_dev -- the vswitch's per-datagram chain in
one kernel, against the oracle's restatements of each step:

    bareVXLanAccess.allow(Protocol.UDP, remote, vxlanBindingAddress.port)
        core/src/main/java/vswitch/Switch.java:679 -> SecurityGroup.java:30-45
    VXLanPacket.from / EthernetPacket / Ipv4Packet / Ipv6Packet ...
        Switch.java:681-684 -> base/src/main/java/vpacket/*.java
    RouteTable.lookup(inner dst)
        core/src/main/java/vswitch/stack/L3.java:423-444 -> RouteTable.java:44-59

Frames are the parse-chain cases of tests/cases.py (every layer, malformed
and truncated shapes); senders are IPv4 and IPv6 (incl. IPv4-mapped).
With per-VNI tables (Switch.tables, Switch.java:560-566) the route comes
from the table of the packet's VNI, and an undefined VNI is dropped.
"""
import numpy as np
import pytest

import oracle_ffi as O
import vproxy_amd as V
from vproxy_amd import workloads as W

from cases import gen_frames

pytestmark = pytest.mark.gpu
BIND_PORT = 4789


def _rules(rng):
    udp = [("10.0.0.0/8", 4789, 4789, True), ("10.1.0.0/16", 0, 65535, False),
           ("192.168.0.0/16", 4000, 5000, True), ("::ffff:172.16.0.0/108", 0, 65535, True),
           ("2001:db8::/32", 4789, 4789, False), ("2001:db8:1::/48", 0, 65535, True),
           ("0.0.0.0/0", 1, 100, True)]
    tcp = [("0.0.0.0/0", 0, 65535, True)]
    from cases import rule_row
    return (np.concatenate([rule_row(*r) for r in tcp]),
            np.concatenate([rule_row(*r) for r in udp]))


def _remotes(rng, n):
    fam = np.where(rng.random(n) < 0.7, 4, 6).astype(np.uint8)
    base = rng.choice(np.array([0x0A000000, 0x0A010000, 0xC0A80000, 0xAC100000, 0x08080000],
                               np.uint64), n)
    r4 = (base | rng.integers(0, 1 << 16, n).astype(np.uint64)).astype(np.uint32)
    r6 = np.zeros((n, 16), np.uint8)
    k = rng.integers(0, 3, n)
    r6[k == 0, 10:12] = 0xFF                         # ::ffff:a.b.c.d
    r6[k == 0, 12:] = W.v4_to_bytes(r4)[k == 0]
    r6[k >= 1, :4] = [0x20, 0x01, 0x0D, 0xB8]
    r6[k == 2, 4:6] = [0, 1]
    r6[:, 14:] = rng.integers(0, 256, (n, 2))
    return fam, r4, r6


def _nets(rng, k4, k6):
    """k4 IPv4 and k6 IPv6 distinct random prefixes in a random list order"""
    plen = rng.integers(1, 20, k4)
    net = rng.integers(0, 2**32, k4, dtype=np.uint64).astype(np.uint32) & W._mask32(plen)
    key = (net.astype(np.uint64) << 8) | plen.astype(np.uint64)
    _, first = np.unique(key, return_index=True)
    nets4 = W.v4_nets(net[np.sort(first)], plen[np.sort(first)])
    rng.shuffle(nets4)
    hi = rng.integers(0, 2**64, k6, dtype=np.uint64)
    p6 = rng.integers(1, 24, k6)
    hi &= np.where(p6 >= 64, np.uint64(2**64 - 1),
                   np.uint64(2**64 - 1) << (64 - p6).astype(np.uint64))
    keyh = np.stack([hi.view(np.int64), p6], 1)
    _, f6 = np.unique(keyh, axis=0, return_index=True)
    nets6 = W.v6_nets(hi[np.sort(f6)], np.zeros(len(f6), np.uint64), p6[np.sort(f6)])
    return nets4, nets6


def _want_route(frames, allow, tables, single=None):
    """the oracle's route per datagram: parse, then RouteTable.lookup in the
    table of the packet's VNI (tables: vni -> (nets4, nets6)), or in
    `single` for every VNI; -2 for an allowed, parsed packet whose VNI has
    no table"""
    want = np.full(len(frames), -1, np.int32)
    for i, f in enumerate(frames):
        p = O.parse_packet(f, V.LAYER_VXLAN)
        _want_route.vni[i] = p["vni"]
        if not allow[i] or p["status"] != 0:
            continue
        t = single if single is not None else tables.get(p["vni"])
        if t is None:
            want[i] = V.SWITCH_NO_TABLE
            continue
        if p["l3"] not in (4, 6):
            continue
        dst = bytes.fromhex(p["dst"])
        if p["l3"] == 4:
            want[i] = O.rt_batch_v4_np(t[0], np.frombuffer(dst, ">u4").astype(np.uint32))[0]
        else:
            want[i] = O.rt_batch_v6_np(t[1], np.frombuffer(dst, np.uint8).reshape(1, 16))[0]
    return want


_want_route.vni = {}


def _rt_nets(rt, family):
    arr, n = rt.rules_raw(family)
    return np.frombuffer(bytes(arr)[:n * W.NET_DT.itemsize], W.NET_DT).copy()


@pytest.mark.parametrize("dflt", [False, True])
def test_switch_classify_vs_oracle(dflt):
    import torch
    rng = np.random.default_rng(17)
    clf = V.Classifier(0)
    try:
        tcp, udp = _rules(rng)
        a, na, ka = W.as_ctypes(tcp, V._lib.VcAclRule)
        b, nb, kb = W.as_ctypes(udp, V._lib.VcAclRule)
        V.check(V.lib().vc_compile_acl(clf.h, a, na, b, nb, 1 if dflt else 0))
        nets4, nets6 = _nets(rng, 3000, 2000)
        ra, rn, rk = W.as_ctypes(nets4, V._lib.VcNet)
        rb, rbn, rbk = W.as_ctypes(nets6, V._lib.VcNet)
        clf.compile_routes_raw(ra, rn, rb, rbn)
        frames = gen_frames(rng, 30011)
        n = len(frames)
        fam, r4, r6 = _remotes(rng, n)
        blob, off = W.pack(frames)
        T = lambda x: torch.from_numpy(np.ascontiguousarray(x)).cuda()
        res, acl, allow, route = clf.switch_classify(
            (T(blob), T(off.astype(np.int32))), T(r4.view(np.int32)), BIND_PORT, remote6=T(r6),
            remote_family=T(fam))
        torch.cuda.synchronize()
        acl, allow, route = acl.cpu().numpy(), allow.cpu().numpy(), route.cpu().numpy()
        l3 = res["l3"].cpu().numpy()
        status = res["status"].cpu().numpy()
        # the bare-VXLAN ACL on the sender (UDP list, bind port)
        proto = np.full(n, 17, np.uint8)
        ports = np.full(n, BIND_PORT, np.uint16)
        w4, a4 = O.sg_batch_v4_np(tcp, udp, dflt, proto, r4, ports)
        r6m = np.ascontiguousarray(r6)
        w6, a6 = O.sg_batch_v6_np(tcp, udp, dflt, proto, r6m, ports)
        six = fam == 6
        np.testing.assert_array_equal(acl, np.where(six, w6, w4))
        np.testing.assert_array_equal(allow, np.where(six, a6, a4))
        assert 0.1 < allow.mean() < 0.9
        # the parse, then the inner route for allowed IP packets
        want = np.full(n, -1, np.int32)
        for i, f in enumerate(frames):
            p = O.parse_packet(f, V.LAYER_VXLAN)
            assert (p["status"], p["l3"]) == (int(status[i]), int(l3[i])), i
            if not allow[i] or p["status"] != 0 or p["l3"] not in (4, 6):
                continue
            dst = bytes.fromhex(p["dst"])
            if p["l3"] == 4:
                want[i] = O.rt_batch_v4_np(nets4, np.frombuffer(dst, ">u4").astype(np.uint32))[0]
            else:
                want[i] = O.rt_batch_v6_np(nets6, np.frombuffer(dst, np.uint8).reshape(1, 16))[0]
        np.testing.assert_array_equal(route, want)
        assert (route >= 0).sum() > 1000
        # the host entry point (vc_switch_classify) gives the same results
        import ctypes as C
        P = lambda x: C.c_void_p(x.ctypes.data)
        h_route, h_acl = np.empty(n, np.int32), np.empty(n, np.int32)
        h_allow, h_l3 = np.empty(n, np.uint8), np.empty(n, np.uint8)
        o = V._lib.VcPktOut(l3=h_l3.ctypes.data)
        V.check(V.lib().vc_switch_classify(clf.h, P(blob), P(off), n, 0, P(fam), P(r4), P(r6m),
                                           BIND_PORT, C.byref(o), P(h_acl), P(h_allow),
                                           P(h_route)))
        for g, w in ((h_route, route), (h_acl, acl), (h_allow, allow), (h_l3, l3)):
            np.testing.assert_array_equal(g, w)
    finally:
        clf.close()


def test_switch_per_vni_tables():
    """Three networks with different RouteTables: each packet is routed in
    the table of its VNI (Switch.java:560-566 tables.get(vni), L3.java:444
    ctx.table.routeTable.lookup); a packet of an undefined VNI comes back
    VC_SWITCH_NO_TABLE.  Both the raw CSR entry point and the RouteTable
    mirrors (vc_routetables_compile_vni); removing the per-VNI tables goes
    back to the single table."""
    import torch
    rng = np.random.default_rng(29)
    clf = V.Classifier(0)
    try:
        tcp, udp = _rules(rng)
        a, na, ka = W.as_ctypes(tcp, V._lib.VcAclRule)
        b, nb, kb = W.as_ctypes(udp, V._lib.VcAclRule)
        V.check(V.lib().vc_compile_acl(clf.h, a, na, b, nb, 1))
        single = _nets(rng, 500, 300)
        ra, rn, rk = W.as_ctypes(single[0], V._lib.VcNet)
        rb, rbn, rbk = W.as_ctypes(single[1], V._lib.VcNet)
        clf.compile_routes_raw(ra, rn, rb, rbn)
        vnis = [7, 100, 0xABCDE]
        tables = {v: _nets(rng, 1500 + 700 * k, 900 + 300 * k) for k, v in enumerate(vnis)}
        clf.compile_vni_routes([(v, tables[v][0], tables[v][1]) for v in (100, 0xABCDE, 7)])
        frames = gen_frames(rng, 20011)
        pick = np.array(vnis + [55])
        for i, f in enumerate(frames):                     # rewrite the VXLAN vni
            if len(f) >= 8:
                v = int(rng.choice(pick))
                frames[i] = f[:4] + bytes([(v >> 16) & 255, (v >> 8) & 255, v & 255]) + f[7:]
        n = len(frames)
        fam, r4, r6 = _remotes(rng, n)
        blob, off = W.pack(frames)
        T = lambda x: torch.from_numpy(np.ascontiguousarray(x)).cuda()

        def run():
            res, acl, allow, route = clf.switch_classify(
                (T(blob), T(off.astype(np.int32))), T(r4.view(np.int32)), BIND_PORT,
                remote6=T(r6), remote_family=T(fam))
            torch.cuda.synchronize()
            return allow.cpu().numpy(), route.cpu().numpy()

        allow, route = run()
        assert 0.1 < allow.mean()
        want = _want_route(frames, allow, tables)
        np.testing.assert_array_equal(route, want)
        vni_of = np.array([_want_route.vni[i] for i in range(n)])
        for v in vnis:                                     # every table was used
            assert ((route >= 0) & (vni_of == v)).sum() > 100, v
        assert (route == V.SWITCH_NO_TABLE).sum() > 500
        # the same tables from RouteTable mirrors, each created with its vni
        rts = []
        for v in vnis:
            rt = V.RouteTable("10.0.0.0/8", None, v)
            for k in range(len(tables[v][0])):
                try:
                    rt.add_rule("r%d" % k, O.net_str(V._lib.VcNet.from_buffer_copy(
                        tables[v][0][k].tobytes())))
                except V.VcError:
                    pass
            rts.append(rt)
        clf.compile_route_tables_vni(rts)
        allow2, route2 = run()
        mirror = {v: (_rt_nets(rt, 4), _rt_nets(rt, 6)) for v, rt in zip(vnis, rts)}
        np.testing.assert_array_equal(allow2, allow)
        np.testing.assert_array_equal(route2, _want_route(frames, allow, mirror))
        # no per-VNI tables: every packet uses the single table
        clf.compile_vni_routes([])
        allow3, route3 = run()
        np.testing.assert_array_equal(route3, _want_route(frames, allow, None, single=single))
        with pytest.raises(V.AlreadyExistException):
            clf.compile_vni_routes([(7, tables[7][0], tables[7][1])] * 2)
    finally:
        clf.close()


@pytest.mark.parametrize("env", ["1", "0"])
def test_switch_bind_port_images(env, monkeypatch):
    """The UDP list's IPv4 image at the bind port (images.h AclPortImage: the
    switch kernel's LDS table; built on the first call with a port, kept with
    the snapshot, and built ahead by every later compile): the sender's rule
    and verdict for three ports in turn, on two lists (a recompile between),
    against the oracle's SecurityGroup.allow(UDP, remote, port) scan.
    VC_ACL_PORT=0 at compile keeps the general image (the A/B)."""
    import torch
    monkeypatch.setenv("VC_ACL_PORT", env)
    rng = np.random.default_rng(23)
    clf = V.Classifier(0)
    try:
        nets4, nets6 = _nets(rng, 500, 100)
        ra, rn, rk = W.as_ctypes(nets4, V._lib.VcNet)
        rb, rbn, rbk = W.as_ctypes(nets6, V._lib.VcNet)
        clf.compile_routes_raw(ra, rn, rb, rbn)
        frames = gen_frames(rng, 20000)
        n = len(frames)
        fam, r4, r6 = _remotes(rng, n)
        blob, off = W.pack(frames)
        T = lambda x: torch.from_numpy(np.ascontiguousarray(x)).cuda()
        tcp0, udp0 = _rules(rng)
        from cases import rule_row
        lists = [udp0, np.concatenate([udp0[::-1], rule_row("10.0.0.0/9", 53, 53, False)])]
        for udp in lists:
            a, na, ka = W.as_ctypes(tcp0, V._lib.VcAclRule)
            b, nb, kb = W.as_ctypes(udp, V._lib.VcAclRule)
            V.check(V.lib().vc_compile_acl(clf.h, a, na, b, nb, 0))
            for port in (BIND_PORT, 53, 4500, BIND_PORT):
                _, acl, allow, _ = clf.switch_classify(
                    (T(blob), T(off.astype(np.int32))), T(r4.view(np.int32)), port,
                    remote6=T(r6), remote_family=T(fam))
                torch.cuda.synchronize()
                proto = np.full(n, 17, np.uint8)
                ports = np.full(n, port, np.uint16)
                w4, a4 = O.sg_batch_v4_np(tcp0, udp, False, proto, r4, ports)
                w6, a6 = O.sg_batch_v6_np(tcp0, udp, False, proto, np.ascontiguousarray(r6), ports)
                six = fam == 6
                np.testing.assert_array_equal(acl.cpu().numpy(), np.where(six, w6, w4), err_msg=str(port))
                np.testing.assert_array_equal(allow.cpu().numpy(), np.where(six, a6, a4))
    finally:
        clf.close()

"""CPU tier: the product's C++ host logic (IP/Network parsing, SecurityGroup
and RouteTable mirrors) against the oracle and the reference's vectors."""
import json
import os

import numpy as np
import pytest

import oracle_ffi as O
import vproxy_amd as V
from vproxy_amd import workloads as W

G = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


def load(name):
    with open(os.path.join(G, name)) as f:
        return json.load(f)


def test_ip_parser_golden():
    d = load("ip_parser.json")
    for v in d["v4_ok"]:
        assert list(V.parse_ip(v["s"])) == v["bytes"]
    for s in d["v4_fail"] + d["bogus"]:
        assert V.parse_ip(s) is None, s
    for v in d["v6_ok"]:
        assert list(V.parse_ip(v["s"])) == v["bytes"], v


def test_ip_parser_fuzz_vs_oracle():
    rng = np.random.default_rng(5)
    alpha = list("0123456789abcdefABCDEF:.[]xg")
    extra = ["::x:1.2.3.4", "::hello:1.2.3.4", "1:2:3:4:5:6:7:1.2.3.4", "::1:2:3:4:5:6:7:1.2.3.4"]
    for s in extra + ["".join(rng.choice(alpha, int(rng.integers(1, 22)))) for _ in range(5000)]:
        assert V.parse_ip(s) == O.parse_ip(s), s


def test_netmask_golden_via_product():
    d = load("netmask.json")
    for v in d["valid_network"]:
        s = "%s/%d" % (v["addr"], v["mask"])
        ok = True
        try:
            V.Network(s)
        except V.IllegalArgumentException:
            ok = False
        assert ok == v["expect"], v
    for v in d["mask_match"] + load("kats.json")["mask_match"]:
        ip_s, m = v["net"].rsplit("/", 1)
        n = V.Network(ip=ip_s, prefix=int(m)) if v["expect"] or True else None
        assert n.contains(v["input"]) == v["expect"], v


def test_network_parse_vs_oracle():
    specs = ["10.0.0.0/8", "10.0.0.1/8", "0.0.0.0/0", "1.2.3.4/32", "1.2.3.4/33", "::/0",
             "::/129", "2001:db8::/32", "[2001:db8::]/32", "1.2.3.0/+24", "1.2.3.0/-1",
             "1.2.3.0/", "/24", "1.2.3.0//24", "1.2.3.0/24/1", "::ffff:0:0/96", "1.2.3.0/024",
             "1.2.3.0/2147483648", "a/1"]
    for s in specs:
        try:
            O.net(s)
            want = True
        except ValueError:
            want = False
        try:
            V.Network(s)
            got = True
        except V.IllegalArgumentException:
            got = False
        assert got == want, s


def _random_nets(rng, n, v6_frac=0.3):
    out = []
    for _ in range(n):
        if rng.random() < v6_frac:
            m = int(rng.integers(0, 129))
            b = bytearray(rng.integers(0, 256, 16, dtype=np.int64).astype(np.uint8).tobytes())
            b[0] = 0x20
            full = int.from_bytes(b, "big") & (((1 << 128) - 1) ^ ((1 << (128 - m)) - 1))
            import ipaddress
            out.append("%s/%d" % (ipaddress.IPv6Address(full), m))
        else:
            m = int(rng.integers(0, 33))
            a = int(rng.integers(0, 2**32)) & ((0xFFFFFFFF << (32 - m)) & 0xFFFFFFFF)
            out.append("%d.%d.%d.%d/%d" % (a >> 24, (a >> 16) & 255, (a >> 8) & 255, a & 255, m))
    return out


def test_route_table_heuristic_vs_oracle():
    rng = np.random.default_rng(9)
    for trial in range(5):
        nets = _random_nets(rng, 250)
        ot = O.RouteTable()
        pt = V.RouteTable()
        for i, s in enumerate(nets):
            ok = ot.add(s)
            if ok:
                pt.add_rule("r%d" % i, s)
            else:
                with pytest.raises(V.AlreadyExistException):
                    pt.add_rule("r%d" % i, s)
        assert [str(x) for x in pt.get_rules()] == ot.rules()


def test_route_table_bulk_shortest_first_vs_oracle():
    """vc_routetable_add_rules' O(n log n) path == the exact heuristic."""
    net, plen = W.gen_v4_prefixes(3000, 12)
    hi, lo, p6 = W.gen_v6_prefixes(800, 13)
    v4 = W.v4_nets(net, plen)
    v6 = W.v6_nets(hi, lo, p6)
    ot = O.RouteTable()
    O.rt_add_np(ot, v4)
    O.rt_add_np(ot, v6)
    pt = V.RouteTable()
    allnets = np.concatenate([v4, v6])
    arr, n, keep = W.as_ctypes(allnets, V._lib.VcNet)
    assert pt.add_rules("p", arr, n=n)          # the O(n log n) path ran
    a4, b6 = O.rt_table_np(ot)
    g4, n4 = pt.rules_raw(4)
    g6, n6 = pt.rules_raw(6)
    assert n4 == len(a4) and n6 == len(b6)
    assert bytes(g4)[:n4 * 40] == a4.tobytes()
    assert bytes(g6)[:n6 * 40] == b6.tobytes()


def test_route_table_bulk_fallback_random_order():
    rng = np.random.default_rng(14)
    nets = _random_nets(rng, 200)
    ot = O.RouteTable()
    uniq = []
    for s in nets:
        if ot.add(s):
            uniq.append(s)
    pt = V.RouteTable()
    assert not pt.add_rules("x", uniq)          # random order: per-rule heuristic
    assert [str(x) for x in pt.get_rules()] == ot.rules()


def test_route_table_with_default_and_validation():
    t = V.RouteTable("10.0.0.0/8", "fd00::/8", 1337)
    assert [str(x) for x in t.get_rules()] == ["10.0.0.0/8", "fd00::/8"]
    t.add_rule("a", "10.1.0.0/16", to_vni=2)
    t.add_rule("b", "0.0.0.0/0", to_vni=3)
    t.add_rule("via", "172.16.0.0/12", via="10.0.0.1")
    with pytest.raises(V.XException):
        t.add_rule("via2", "172.17.0.0/16", via="11.0.0.1")      # RouteTable.java:98-100
    with pytest.raises(V.AlreadyExistException):
        t.add_rule("a", "10.2.0.0/16")                           # alias
    with pytest.raises(V.AlreadyExistException):
        t.add_rule("c", "10.1.0.0/16")                           # same network
    with pytest.raises(V.AlreadyExistException):
        t.add_rule("default", "10.9.0.0/16")                     # alias check first (:70-72)
    t.del_rule("default")
    with pytest.raises(V.XException):
        t.add_rule("default", "10.9.0.0/16")                     # RouteTable.java:86-89
    t.del_rule("a")
    with pytest.raises(V.NotFoundException):
        t.del_rule("a")
    t2 = V.RouteTable("10.0.0.0/8", None, 1)
    with pytest.raises(V.XException):
        t2.add_rule("v6via", "192.168.0.0/16", via="::1")        # RouteTable.java:95-97


def test_security_group_mirror():
    sg = V.SecurityGroup("sg", False)
    sg.add_rule("a", "10.0.0.0/8", "TCP", 1, 2, True)
    sg.add_rule("b", "10.0.0.0/8", "UDP", 1, 2, True)       # other protocol: fine
    with pytest.raises(V.AlreadyExistException):
        sg.add_rule("a", "11.0.0.0/8", "UDP", 1, 2, True)    # alias (SecurityGroup.java:57-58)
    with pytest.raises(V.AlreadyExistException):
        sg.add_rule("c", "10.0.0.0/8", "tcp", 1, 2, False)   # same net/proto/ports (:67-74)
    sg.add_rule("d", "10.0.0.0/8", "TCP", 1, 3, False)
    assert [(r.min_port, r.max_port) for r in sg.rules("TCP")] == [(1, 2), (1, 3)]
    sg.remove_rule("a")
    assert [(r.min_port, r.max_port) for r in sg.rules("TCP")] == [(1, 3)]
    with pytest.raises(V.NotFoundException):
        sg.remove_rule("a")
    with pytest.raises(V.IllegalArgumentException):
        sg.add_rule("e", "10.0.0.1/8", "TCP", 1, 2, True)    # invalid network
    with pytest.raises(V.IllegalArgumentException):
        sg.add_rule("e", "10.0.0.0/8", "ICMP", 1, 2, True)   # ProtocolHandle


def test_no_gpu_fails_loudly():
    import torch
    if torch.cuda.is_available():
        pytest.skip("GPU present")
    with pytest.raises(V.DeviceError):
        V.Classifier(0)


def test_ipv6_row_shapes():
    """classifier._rows16: IPv6 address arrays are [m, 16] bytes or flat bytes
    of a length divisible by 16; anything else is refused before a kernel is
    handed a row count its buffer does not hold (vc_pipeline_c6 trusts n6)."""
    import torch
    from vproxy_amd.classifier import _rows16
    assert _rows16(np.zeros((5, 16), np.uint8), "x") == 5
    assert _rows16(np.zeros(48, np.uint8), "x") == 3
    assert _rows16(np.zeros((0, 16), np.uint8), "x") == 0
    assert _rows16(torch.zeros((7, 16), dtype=torch.uint8), "x") == 7
    for bad in (np.zeros(47, np.uint8), np.zeros((5, 8), np.uint8), np.zeros((5, 4), np.int32),
                np.zeros(12, np.uint32), np.zeros((2, 16, 1), np.uint8)):
        with pytest.raises(V.IllegalArgumentException):
            _rows16(bad, "x")


def test_pipeline_argument_errors_before_any_call():
    """Classifier.pipeline refuses inconsistent IPv6 arguments before it
    touches the library (so this runs without a device)."""
    from vproxy_amd.classifier import Classifier
    c = object.__new__(Classifier)          # no context: a library call would fail differently
    n = 8
    z = lambda dt: np.zeros(n, dt)
    base = (z(np.uint8), z(np.uint32), z(np.uint32), z(np.uint16), z(np.uint32),
            np.zeros(4, np.int32))
    rows = np.zeros((n, 16), np.uint8)
    cases = [dict(src6=rows),                                        # dst6 missing
             dict(dst6=rows),                                        # src6 missing
             dict(src6=rows, dst6=rows[:3]),                         # row counts differ
             dict(src6=rows[:3], dst6=rows[:3]),                     # not one row per packet
             dict(src6=np.zeros(40, np.uint8), dst6=np.zeros(40, np.uint8)),   # not 16-byte rows
             dict(src6=np.zeros((n + 1, 16), np.uint8), dst6=np.zeros((n + 1, 16), np.uint8),
                  compact6=True),                                    # more rows than packets
             dict(family=z(np.uint8), compact6=True)]                # compact without rows
    for kw in cases:
        with pytest.raises(V.IllegalArgumentException):
            c.pipeline(*base, **kw)

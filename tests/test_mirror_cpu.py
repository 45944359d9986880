"""CPU tier: traffic-mirror filters.

The oracle (vo_mirror_match / vo_mirror_switch: FilterConfig.java:27-94,
Mirror.java:73-139) against hand-derived vectors -- no reference test
covers vmirror, so these pin it (parity pinned by hand-derived vectors) --
then the kernels' own item loading and filter code run on the host
(tests/native/imgcheck.hip) against the oracle on random filter sets, for
MirrorData items and for switchPacket frames."""
import numpy as np
import pytest

import imgcheck_ffi as I
import oracle_ffi as O
import vproxy_amd as V
from cases import gen_mirror_case, mirror_columns, mirror_frames, mirror_v6_frames
from vproxy_amd.mirror import MirrorFilters, items_struct, parse_mac

A, B, C_, D = ("0a:00:27:00:00:%02x" % i for i in range(4))


def _one(filters, origin="switch", mac_src=A, mac_dst=B, ip_src=None, ip_dst=None,
         transport=None, ps=0, pd=0, app=None):
    ids = {}
    arr = O.mirror_filters(filters, ids)
    iid = lambda s: -1 if s is None else ids.get(s, -2)
    ip = lambda s: None if s is None else O.parse_ip(s)
    return O.mirror_match(arr, len(filters), iid(origin), parse_mac(mac_src), parse_mac(mac_dst),
                          ip(ip_src), ip(ip_dst), iid(transport), ps, pd, iid(app))


def test_oracle_ethernet_level():
    f = [{"origin": "switch", "mirror": 0, "mac": A},
         {"origin": "switch", "mirror": 1, "mac": A, "mac2": C_},
         {"origin": "switch", "mirror": 2},
         {"origin": "tcp-lb", "mirror": 3}]
    assert _one(f, mac_src=A, mac_dst=B) == 0b101          # macX either side; no-mac filter
    assert _one(f, mac_src=C_, mac_dst=A) == 0b111         # the pair, reversed
    assert _one(f, mac_src=D, mac_dst=B) == 0b100
    assert _one(f, origin="tcp-lb") == 0b1000
    assert _one(f, origin="nobody") == 0
    # a null IP selects matchEthernet: the network part is not looked at
    f = [{"origin": "switch", "mirror": 5, "network": "192.168.0.0/16"}]
    assert _one(f, ip_src=None, ip_dst="10.0.0.1") == 1 << 5


def test_oracle_ip_level():
    f = [{"origin": "switch", "mirror": 0, "network": "10.0.0.0/8"},
         {"origin": "switch", "mirror": 1, "network": "10.0.0.0/8", "network2": "192.168.0.0/16"},
         {"origin": "switch", "mirror": 2, "mac": D, "network": "10.0.0.0/8"},
         {"origin": "switch", "mirror": 3, "network": "::ffff:10.0.0.0/104"},
         {"origin": "switch", "mirror": 4, "network": "fd00::/8", "port": [1, 2]}]
    assert _one(f, ip_src="10.1.1.1", ip_dst="8.8.8.8") == 0b01001
    assert _one(f, ip_src="192.168.3.3", ip_dst="10.9.9.9") == 0b01011
    assert _one(f, ip_src="8.8.8.8", ip_dst="8.8.4.4") == 0
    assert _one(f, ip_src="::ffff:10.1.1.1", ip_dst="fd00::1") == 0b11001   # v4 rule, mapped v6
    # transport null -> matchIp: the port range of filter 4 is not checked
    assert _one(f, ip_src="fd00::1", ip_dst="fd00::2", ps=80, pd=80) == 1 << 4


def test_oracle_transport_and_app_level():
    f = [{"origin": "o", "mirror": 0, "transportLayerProtocol": "tcp"},
         {"origin": "o", "mirror": 1, "port": [80, 80]},
         {"origin": "o", "mirror": 2, "port": [80, 80], "port2": [1000, 2000]},
         {"origin": "o", "mirror": 3, "applicationLayerProtocol": "http"},
         {"origin": "o", "mirror": 4, "transportLayerProtocol": "udp", "port": [53, 53]}]
    ip = dict(ip_src="10.0.0.1", ip_dst="10.0.0.2")
    assert _one(f, "o", transport="tcp", ps=1500, pd=80, **ip) == 0b01111
    assert _one(f, "o", transport="tcp", ps=80, pd=80, **ip) == 0b01011
    assert _one(f, "o", transport="quic", ps=9, pd=9, **ip) == 0b01000
    # application level: filters without an app protocol still match
    assert _one(f, "o", transport="tcp", ps=80, pd=1200, app="http", **ip) == 0b01111
    assert _one(f, "o", transport="tcp", ps=80, pd=1200, app="dns", **ip) == 0b00111
    assert _one(f, "o", transport="udp", ps=53, pd=9, app="dns", **ip) == 0b10000


def test_parse_mac_like_java():
    assert parse_mac("0a:00:27:00:00:ff") == bytes([10, 0, 0x27, 0, 0, 255])
    assert parse_mac("+f:-1:00:00:00:00") == bytes([15, 255, 0, 0, 0, 0])   # parseInt(s, 16)
    for bad in ("0a:00:27:00:00:0", "0a-00-27-00-00-00", "0a:00:27:00:00:0g", "0a::27:00:00:000"):
        with pytest.raises(V.IllegalArgumentException):
            parse_mac(bad)


def _device_vs_oracle(filters, items):
    mf = MirrorFilters()
    arr, nf = mf.build(filters)
    ids = {}
    oarr = O.mirror_filters(filters, ids)
    assert ids == mf.ids                                 # same interning order
    cols = mirror_columns(items, lambda s: mf.id_of(s, create=False), V.parse_ip)
    it = items_struct(cols)
    origins = sorted(set(f["origin"] for f in filters)) + ["nobody"]
    for origin in origins:
        got = I.mirror(arr, nf, mf.id_of(origin, create=False), it, len(items))
        oid = ids.get(origin, -2)
        want = [O.mirror_match(oarr, len(filters), oid, parse_mac(i["mac_src"]),
                               parse_mac(i["mac_dst"]),
                               None if i["ip_src"] is None else O.parse_ip(i["ip_src"]),
                               None if i["ip_dst"] is None else O.parse_ip(i["ip_dst"]),
                               ids.get(i["transport"], -2) if i["transport"] else -1,
                               i["port_src"], i["port_dst"],
                               ids.get(i["app"], -2) if i["app"] else -1) for i in items]
        np.testing.assert_array_equal(got, np.array(want, np.uint64), err_msg=origin)


@pytest.mark.parametrize("seed,nf", [(1, 0), (2, 1), (3, 8), (4, 60)])
def test_items_vs_oracle(seed, nf):
    filters, items = gen_mirror_case(np.random.default_rng(seed), nf, 3000)
    _device_vs_oracle(filters, items)


@pytest.mark.parametrize("seed,nf", [(5, 1), (6, 9), (7, 40), (8, 150), (9, 200)])
def test_items_bitsets_vs_oracle(seed, nf):
    """Mirror.mirror over MirrorData items through the per-origin bit-set
    image (mirror_match_sw: nets per family, MAC filters, transport / app
    ids, port ranges of both sides) against the oracle at every level, for
    every origin; origins over 64 filters have no image.  Ports include
    values outside 0-65535 and negative ones (Java ints)."""
    rng = np.random.default_rng(seed)
    filters, items = gen_mirror_case(rng, nf, 4000)
    for f in filters[::7]:
        if "port" in f:
            f["port"] = [-5, f["port"][1]] if rng.random() < 0.5 else [f["port"][0], 70000]
    for i in items[::11]:
        i["port_src"] = int(rng.choice([-1, -70000, 65535, 65536, 2**31 - 1, -2**31]))
    mf = MirrorFilters()
    arr, n = mf.build(filters)
    ids = {}
    oarr = O.mirror_filters(filters, ids)
    cols = mirror_columns(items, lambda s: mf.id_of(s, create=False), V.parse_ip)
    it = items_struct(cols)
    built = 0
    for origin in sorted(set(f["origin"] for f in filters)) + ["nobody"]:
        oid = mf.id_of(origin, create=False)
        got = I.mirror_sw(arr, n, oid, it, len(items))
        count = sum(f["origin"] == origin for f in filters)
        if count == 0 or count > 64:
            assert got is None, (origin, count)
            continue
        built += 1
        want = I.mirror(arr, n, oid, it, len(items))      # per-filter path, == oracle above
        np.testing.assert_array_equal(got, want, err_msg=origin)
        o2 = np.array([O.mirror_match(oarr, len(filters), ids.get(origin, -2),
                                      parse_mac(i["mac_src"]), parse_mac(i["mac_dst"]),
                                      None if i["ip_src"] is None else O.parse_ip(i["ip_src"]),
                                      None if i["ip_dst"] is None else O.parse_ip(i["ip_dst"]),
                                      ids.get(i["transport"], -2) if i["transport"] else -1,
                                      i["port_src"], i["port_dst"],
                                      ids.get(i["app"], -2) if i["app"] else -1)
                       for i in items[:800]], np.uint64)
        np.testing.assert_array_equal(got[:800], o2, err_msg=origin)
    assert built >= 1 or nf > 64 * 3


@pytest.mark.parametrize("layer", [0, 1])
def test_switch_vs_oracle(layer):
    rng = np.random.default_rng(40 + layer)
    filters, _ = gen_mirror_case(rng, 40, 0, origins=("switch", "other"))
    frames = [f if layer == 0 else f[8:] for f in mirror_frames(rng, 4000)]
    mf = MirrorFilters()
    arr, nf = mf.build(filters)
    oarr = O.mirror_filters(filters, {})
    oid = mf.id_of("switch", create=False)
    got = I.mirror_switch(arr, nf, oid, frames, layer)
    want = np.array([O.mirror_switch(oarr, nf, oid, f, layer) for f in frames], np.uint64)
    np.testing.assert_array_equal(got, want)
    assert (want != 0).mean() > 0.2


@pytest.mark.parametrize("seed", range(6))
def test_switch_bitsets_vs_oracle(seed):
    """switchPacket through the per-origin bit-set image (MirrorSwImage:
    interval masks of netX / netY per address family, MAC filters, mirror
    bits) against the oracle, on random filter lists over the mirror
    network pools (IPv4, IPv6, v4-mapped and v4-compatible forms) and
    random, mirror-pool and IPv6 frames, for every origin."""
    rng = np.random.default_rng(70 + seed)
    nf = [3, 17, 40, 64, 90, 130][seed]
    origins = ("switch", "other") if nf < 130 else ("switch", "other", "a", "b")
    filters, _ = gen_mirror_case(rng, nf, 0, origins=origins)
    if nf == 130:                       # one origin over 64 filters: per-filter path
        filters += [{"origin": "big", "mirror": k % 5, "network": "10.%d.0.0/16" % k}
                    for k in range(65)]
        origins += ("big",)
    frames = mirror_frames(rng, 3000) + mirror_v6_frames(rng, 1500)
    mf = MirrorFilters()
    arr, nf = mf.build(filters)
    oarr = O.mirror_filters(filters, {})
    built = 0
    for origin in origins:
        oid = mf.id_of(origin, create=False)
        r = I.mirror_switch_sw(arr, nf, oid, frames, 0)
        count = sum(f["origin"] == origin for f in filters)
        if count == 0 or count > 64:
            assert r is None, (origin, count)
            continue
        assert r is not None, (origin, count)
        built += 1
        got, (nb4, nb6) = r
        want = np.array([O.mirror_switch(oarr, nf, oid, f, 0) for f in frames], np.uint64)
        np.testing.assert_array_equal(got, want, err_msg=origin)
        assert nb4 >= 1 and nb6 >= 1
        if nf >= 17:
            assert (want != 0).mean() > 0.1
    assert built >= 1


def test_switch_bitsets_bench_filters():
    """The mirror sub-bench's 17 filters (bench.MIRROR_FILTERS): the
    bit-set image exists, and equals the oracle on the bench's frame
    templates."""
    import bench as Bn
    from vproxy_amd import workloads as W
    frames = W.gen_vxlan_frames(4000, W.SEED + 12)
    mf = MirrorFilters()
    arr, nf = mf.build(Bn.MIRROR_FILTERS)
    oarr = O.mirror_filters(Bn.MIRROR_FILTERS, {})
    oid = mf.id_of("switch", create=False)
    got, (nb4, nb6) = I.mirror_switch_sw(arr, nf, oid, frames, 0)
    want = np.array([O.mirror_switch(oarr, nf, oid, f, 0) for f in frames], np.uint64)
    np.testing.assert_array_equal(got, want)
    assert nb4 <= 2 * 32 + 1 and nb6 >= 1


def test_bitsets_refuse_a_non_prefix_mask():
    """A network whose mask is not a run of high ones (possible only through
    the C ABI: FilterConfig parses masks from prefix lengths) cannot be an
    interval: its origin has no bit-set image and keeps the per-filter loop,
    whose answer still equals the oracle."""
    filters = [{"origin": "switch", "mirror": 1, "network": "10.0.0.0/8"},
               {"origin": "switch", "mirror": 2, "network": "10.0.0.0/16"},
               {"origin": "other", "mirror": 3, "network": "10.0.0.0/8"}]
    mf = MirrorFilters()
    arr, nf = mf.build(filters)
    arr[1].net_x.mask[1] = 0x0F                 # 255.15.0.0: not a prefix
    oarr = O.mirror_filters(filters, {})
    oarr[1].net_x.mask[1] = 0x0F
    frames = mirror_frames(np.random.default_rng(3), 2000)
    oid = mf.id_of("switch", create=False)
    assert I.mirror_switch_sw(arr, nf, oid, frames, 0) is None
    assert I.mirror_switch_sw(arr, nf, mf.id_of("other", create=False), frames, 0) is not None
    got = I.mirror_switch(arr, nf, oid, frames, 0)
    want = np.array([O.mirror_switch(oarr, nf, oid, f, 0) for f in frames], np.uint64)
    np.testing.assert_array_equal(got, want)
    assert ((want >> 2) & 1).any()              # the odd mask matches some frames

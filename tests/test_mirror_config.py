"""CPU tier: the mirror config loader (vproxy_amd.mirror.load_config, after
Mirror.parseAndLoad, base/src/main/java/vmirror/Mirror.java:345-374,
503-601) over the reference's own config files (tests/golden/kats.json
mirror_configs: doc/mirror-example.json and misc/mirror-switch.json), and
the oracle's filter masks (vo_mirror_match, FilterConfig.java:27-94) against
the hand-derived expectations of those KATs.  The GPU kernels are checked
against the same KATs in tests/test_gpu_mirror.py."""
import copy
import json
import os

import pytest

import oracle_ffi as O
import vproxy_amd as V
from vproxy_amd.mirror import load_config, parse_mac

G = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


def configs():
    return json.load(open(os.path.join(G, "kats.json")))["mirror_configs"]


def stripped(case):
    cfg = copy.deepcopy(case["config"])
    if case["strip_strings"]:
        for m in cfg["mirrors"]:
            for o in m["origins"]:
                o["filters"] = [f for f in o["filters"] if isinstance(f, dict)]
    return cfg


def oracle_masks(filters, origin, items):
    ids = {}
    arr = O.mirror_filters(filters, ids)
    iid = lambda s: -1 if s is None else ids.get(s, -2)
    return [O.mirror_match(arr, len(filters), ids.get(origin, -2), parse_mac(i["mac_src"]),
                           parse_mac(i["mac_dst"]),
                           None if i["ip_src"] is None else O.parse_ip(i["ip_src"]),
                           None if i["ip_dst"] is None else O.parse_ip(i["ip_dst"]),
                           iid(i["transport"]), i["port_src"], i["port_dst"], iid(i["app"]))
            for i in items]


@pytest.mark.parametrize("k", [0, 1])
def test_reference_configs_load(k):
    case = configs()[k]
    s = load_config(stripped(case))
    assert s.enabled is case["enabled"], case["source"]
    assert [list(m) for m in s.mirrors] == case["mirrors"]
    assert len(s.filters) == case["n_filters"]
    assert all(f["mirror"] == 0 for f in s.filters)
    # "enabled": false in both files -> Mirror.isEnabled is false everywhere
    for c in case["cases"]:
        assert not s.is_enabled(c["origin"])


def test_example_verbatim_is_rejected():
    """The example's explanation strings are not filter objects: the Java
    cast at Mirror.java:536 fails, the whole load is a type error."""
    with pytest.raises(V.IllegalArgumentException, match="type error.*filters\\[1\\]"):
        load_config(configs()[0]["config"])


@pytest.mark.parametrize("k", [0, 1])
def test_reference_config_masks_oracle(k):
    case = configs()[k]
    s = load_config(stripped(case))
    for c in case["cases"]:
        got = oracle_masks(s.filters, c["origin"], c["items"])
        assert got == [i["want"] for i in c["items"]], [
            (i["why"], g) for i, g in zip(c["items"], got) if g != i["want"]]


def _edit(fn):
    cfg = stripped(configs()[0])
    fn(cfg)
    return cfg


@pytest.mark.parametrize("kind,edit", [
    ("type error", lambda c: c.update(enabled="yes")),
    ("missing field", lambda c: c.pop("mirrors")),
    ("invalid value", lambda c: c["mirrors"][0].update(mtu=1501)),
    ("invalid value", lambda c: c["mirrors"][0].update(mtu=-1)),
    ("type error", lambda c: c["mirrors"][0].update(mtu="1500")),
    ("missing field", lambda c: c["mirrors"][0].pop("tap")),
    ("missing field", lambda c: c["mirrors"][0]["origins"][0].pop("filters")),
    ("invalid value", lambda c: c["mirrors"][0]["origins"][0]["filters"][0].update(port=[80, 1])),
    ("invalid value", lambda c: c["mirrors"][0]["origins"][0]["filters"][0].update(port2=[9, 3])),
    ("invalid value", lambda c: c["mirrors"][0]["origins"][0]["filters"][0].update(mac="zz")),
    ("invalid value",
     lambda c: c["mirrors"][0]["origins"][0]["filters"][0].update(network="172.16.0.1/24")),
    ("type error", lambda c: c["mirrors"][0]["origins"][0]["filters"][0].update(port=[1, "2"])),
])
def test_config_errors(kind, edit):
    with pytest.raises(V.IllegalArgumentException, match=kind):
        load_config(_edit(edit))


def test_second_values_only_with_first():
    """mac2 / network2 / port2 are read only inside their first value's
    block (Mirror.java:548-592): alone they are ignored."""
    cfg = {"enabled": True, "mirrors": [{"tap": "t", "mtu": 1500, "origins": [
        {"origin": "o", "filters": [{"mac2": "zz", "network2": "bad", "port2": [9, 1]}]}]}]}
    s = load_config(cfg)
    assert s.filters == [{"origin": "o", "mirror": 0}]
    assert s.is_enabled("o") and not s.is_enabled("p")


@pytest.mark.parametrize("filt,kind,field", [
    # two bad fields: the one Mirror.parseAndLoadFilter reads first is reported
    ({"mac": "zz", "port": [1, "2"]}, "invalid value", "mac"),
    ({"port": "80", "mac": "00:00:00:00:00:01", "network": "bad"}, "invalid value", "network"),
    ({"network": 7, "mac2": "x", "transportLayerProtocol": 5}, "type error", "network"),
    ({"transportLayerProtocol": 5, "port": [9, 1]}, "type error", "transportLayerProtocol"),
    ({"port": [80], "applicationLayerProtocol": 3}, "invalid value", "port"),
    ({"port": [1, 2], "port2": [5], "applicationLayerProtocol": 3}, "invalid value", "port2"),
    ({"mac": "00:00:00:00:00:01", "mac2": "bad", "network": "nope"}, "invalid value", "mac2"),
])
def test_first_bad_field_is_reported(filt, kind, field):
    """Mirror.java:545-600 reads mac, mac2, network, network2,
    transportLayerProtocol, port, port2, applicationLayerProtocol in that
    order and throws at the first failure (runSub maps ClassCastException
    to a type error, IllegalArgument- and IndexOutOfBoundsException to an
    invalid value), naming that field."""
    cfg = {"enabled": True, "mirrors": [{"tap": "t", "mtu": 1500, "origins": [
        {"origin": "o", "filters": [filt]}]}]}
    with pytest.raises(V.IllegalArgumentException, match=r"%s .*filters\[0\]\.%s$" % (kind, field)):
        load_config(cfg)

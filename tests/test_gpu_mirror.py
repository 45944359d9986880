"""GPU tier: traffic-mirror filters (device/mirror.hip) through the C ABI
against the oracle (vo_mirror_match / vo_mirror_switch, FilterConfig.java
:27-94, Mirror.java:73-139), bit-exact: MirrorData items at every null
level, host and device entry points, and switchPacket over raw VXLAN and
Ethernet frames."""
import numpy as np
import pytest

import oracle_ffi as O
import vproxy_amd as V
from cases import gen_mirror_case, mirror_columns, mirror_frames, mirror_v6_frames
from vproxy_amd.mirror import parse_mac

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def clf():
    c = V.Classifier(0)
    yield c
    c.close()


@pytest.mark.parametrize("sw", ["2", "1", "0"])   # bit sets from LDS / global / per filter
def test_items_vs_oracle(clf, sw, monkeypatch):
    import torch
    filters, items = gen_mirror_case(np.random.default_rng(7), 50, 20000)
    monkeypatch.setenv("VC_MIRROR_SW", sw)
    mf = clf.compile_mirror(filters)
    ids = {}
    oarr = O.mirror_filters(filters, ids)
    cols = mirror_columns(items, lambda s: mf.id_of(s, create=False), V.parse_ip)
    iid = lambda s: -1 if s is None else ids.get(s, -2)
    for origin in ("switch", "tcp-lb", "socks5", "nobody"):
        got = clf.mirror_match(origin, cols, len(items))
        want = np.array([O.mirror_match(oarr, len(filters), ids.get(origin, -2),
                                        parse_mac(i["mac_src"]), parse_mac(i["mac_dst"]),
                                        None if i["ip_src"] is None else O.parse_ip(i["ip_src"]),
                                        None if i["ip_dst"] is None else O.parse_ip(i["ip_dst"]),
                                        iid(i["transport"]), i["port_src"], i["port_dst"],
                                        iid(i["app"])) for i in items], np.uint64)
        np.testing.assert_array_equal(got, want, err_msg=origin)
        dcols = {k: torch.from_numpy(v).cuda() for k, v in cols.items()}
        dev = clf.mirror_match(origin, dcols, len(items))
        torch.cuda.synchronize()
        np.testing.assert_array_equal(dev.cpu().numpy().view(np.uint64), want)


def test_items_defaults(clf):
    """Absent columns: MirrorData's default MACs, null IPs (ether level)."""
    clf.compile_mirror([{"origin": "o", "mirror": 0, "mac": "00:00:00:00:00:00"},
                        {"origin": "o", "mirror": 1, "mac": "ff:ff:ff:ff:ff:ff",
                         "mac2": "00:00:00:00:00:00"},
                        {"origin": "o", "mirror": 2, "mac": "0a:00:00:00:00:00"}])
    got = clf.mirror_match("o", {}, 5)
    np.testing.assert_array_equal(got, np.full(5, 0b011, np.uint64))


# switchPacket's three kernels, chosen at compile by VC_MIRROR_SW: "2" (the
# default) the per-origin bit-set image with its IPv4 intervals in LDS, "1"
# the same read from the global table, "0" the per-filter kernel
@pytest.mark.parametrize("sw", ["2", "1", "0"])
@pytest.mark.parametrize("layer", [0, 1])
def test_switch_vs_oracle(clf, layer, sw, monkeypatch):
    import torch
    rng = np.random.default_rng(50 + layer)
    filters, _ = gen_mirror_case(rng, 60, 0, origins=("switch", "other"))
    frames = [f if layer == 0 else f[8:] for f in mirror_frames(rng, 30000) + mirror_v6_frames(rng, 8000)]
    monkeypatch.setenv("VC_MIRROR_SW", sw)
    mf = clf.compile_mirror(filters)
    oarr = O.mirror_filters(filters, {})
    oid = mf.id_of("switch", create=False)
    want = np.array([O.mirror_switch(oarr, len(filters), oid, f, layer) for f in frames],
                    np.uint64)
    got = clf.mirror_switch("switch", frames, layer)
    np.testing.assert_array_equal(got, want)
    lens = np.array([len(f) for f in frames], np.int64)
    off = np.zeros(len(frames) + 1, np.int64)
    off[1:] = np.cumsum(lens)
    blob = torch.from_numpy(np.frombuffer(b"".join(frames), np.uint8).copy()).cuda()
    dev = clf.mirror_switch("switch", (blob, torch.from_numpy(off.astype(np.int32)).cuda()), layer)
    torch.cuda.synchronize()
    np.testing.assert_array_equal(dev.cpu().numpy().view(np.uint64), want)
    assert (want != 0).mean() > 0.2


def test_switch_origin_over_64_filters(clf):
    """An origin with 65 filters has no bit-set image (64-bit masks): its
    frames take the per-filter kernel; the other origin's take the image."""
    rng = np.random.default_rng(61)
    filters = [{"origin": "big", "mirror": k % 7, "network": "10.%d.0.0/16" % (k % 3),
                "mac": "0a:00:27:00:00:%02x" % (k % 4)} for k in range(65)]
    filters += gen_mirror_case(rng, 20, 0, origins=("switch",))[0]
    frames = mirror_frames(rng, 20000)
    mf = clf.compile_mirror(filters)
    oarr = O.mirror_filters(filters, {})
    for origin in ("big", "switch"):
        oid = mf.id_of(origin, create=False)
        want = np.array([O.mirror_switch(oarr, len(filters), oid, f, 0) for f in frames],
                        np.uint64)
        np.testing.assert_array_equal(clf.mirror_switch(origin, frames, 0), want, err_msg=origin)
        assert (want != 0).mean() > 0.05


def test_errors(clf):
    for bad in ({"origin": "o", "mirror": 64}, {"origin": "o", "mirror": 0, "port": [5, 4]},
                {"origin": "o", "mirror": 0, "port": [1, 2], "port2": [9, 3]}):
        with pytest.raises(V.IllegalArgumentException):
            clf.compile_mirror([bad])
    clf.compile_mirror([{"origin": "switch", "mirror": 0}])
    with pytest.raises(V.IllegalArgumentException):
        clf.mirror_switch("switch", [b"\0" * 20], layer=4)


@pytest.mark.parametrize("sw", ["2", "1", "0"])
@pytest.mark.parametrize("shift,pad", [(1, 0), (0, 1400)])
def test_switch_unstaged(clf, shift, pad, sw, monkeypatch):
    import torch
    rng = np.random.default_rng(80 + shift)
    filters, _ = gen_mirror_case(rng, 30, 0, origins=("switch",))
    frames = [f + bytes(int(rng.integers(0, pad + 1))) if pad else f
              for f in mirror_frames(rng, 5000)]
    monkeypatch.setenv("VC_MIRROR_SW", sw)
    mf = clf.compile_mirror(filters)
    oarr = O.mirror_filters(filters, {})
    oid = mf.id_of("switch", create=False)
    want = np.array([O.mirror_switch(oarr, len(filters), oid, f, 0) for f in frames], np.uint64)
    lens = np.array([len(f) for f in frames], np.int64)
    off = np.zeros(len(frames) + 1, np.int64)
    off[1:] = np.cumsum(lens)
    b = np.concatenate([np.zeros(shift, np.uint8), np.frombuffer(b"".join(frames), np.uint8)])
    blob = torch.from_numpy(b).cuda()[shift:]
    dev = clf.mirror_switch("switch", (blob, torch.from_numpy(off.astype(np.int32)).cuda()), 0)
    torch.cuda.synchronize()
    np.testing.assert_array_equal(dev.cpu().numpy().view(np.uint64), want)


@pytest.mark.parametrize("k", [0, 1])
def test_reference_configs(clf, k):
    """The reference's mirror config files (kats.json mirror_configs,
    loaded by vproxy_amd.mirror.load_config) compiled for the kernel: the
    hand-derived masks of every item, host and device entry points."""
    import torch
    from test_mirror_config import configs, stripped
    from vproxy_amd.mirror import load_config
    case = configs()[k]
    s = load_config(stripped(case))
    mf = clf.compile_mirror(s.filters)
    for c in case["cases"]:
        items = c["items"]
        want = np.array([i["want"] for i in items], np.uint64)
        cols = mirror_columns(items, lambda x: mf.id_of(x, create=False), V.parse_ip)
        np.testing.assert_array_equal(clf.mirror_match(c["origin"], cols, len(items)), want,
                                      err_msg=case["source"])
        dcols = {key: torch.from_numpy(v).cuda() for key, v in cols.items()}
        dev = clf.mirror_match(c["origin"], dcols, len(items))
        torch.cuda.synchronize()
        np.testing.assert_array_equal(dev.cpu().numpy().view(np.uint64), want)


def test_items_mac_alignment(clf):
    """vc_mirror_match_dev reads the 6-byte MAC columns with 16-bit loads:
    an odd device address is refused (VC_EINVAL), an even one is read."""
    import torch
    clf.compile_mirror([{"origin": "o", "mirror": 3, "mac": "0a:00:27:00:00:01"}])
    raw = torch.zeros(6 * 4 + 2, dtype=torch.uint8, device="cuda")
    raw[2:8] = torch.tensor([10, 0, 0x27, 0, 0, 1], dtype=torch.uint8)
    with pytest.raises(V.IllegalArgumentException):
        clf.mirror_match("o", {"mac_src": raw[1:25]}, 4)
    got = clf.mirror_match("o", {"mac_src": raw[2:26]}, 4)
    torch.cuda.synchronize()
    np.testing.assert_array_equal(got.cpu().numpy().view(np.uint64), [1 << 3, 0, 0, 0])


def test_mirroritems_bench_batch(clf):
    """The `mirroritems` sub-bench's whole batch (bench.mirror_items_workload:
    32M items, 40 filters) through vc_mirror_match_dev, every result equal to
    the oracle's Mirror.mirror (vo_mirror_match_batch)."""
    import ctypes as C
    import os
    import torch
    import bench as B
    from vproxy_amd.mirror import items_struct
    n = 32 << 20
    filters, mf, tcols, dcols, idx = B.mirror_items_workload(n, torch.device("cuda"),
                                                             clf.compile_mirror)
    out = torch.empty(n, dtype=torch.int64, device="cuda")
    oid = mf.id_of("tcp-lb", create=False)
    it = items_struct(dcols)
    V.check(V.lib().vc_mirror_match_dev(clf.h, oid, C.byref(it), n, C.c_void_p(out.data_ptr()),
                                        C.c_void_p(torch.cuda.current_stream().cuda_stream)))
    torch.cuda.synchronize()
    got = out.cpu().numpy().view(np.uint64)
    ids = {}
    oarr = O.mirror_filters(filters, ids)
    # the oracle on the 64K templates, gathered per item (items are copies of them)
    want_t = O.mirror_match_batch_np(oarr, len(filters), ids["tcp-lb"], tcols,
                                     nthreads=min(16, os.cpu_count() or 1))
    np.testing.assert_array_equal(got, want_t[idx.cpu().numpy()])
    assert (got != 0).mean() > 0.2

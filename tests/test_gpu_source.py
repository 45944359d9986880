"""GPU tier: ServerGroup source hashing (device/select.hip) through the C ABI
against the oracle (vo_source_select, ServerGroup.java:464-490), bit-exact:
random groups of mixed IPv4/IPv6 servers with duplicate addresses, zero
weights and unhealthy servers; IPv4 and IPv6 clients; all three views;
health updates; out-of-range and -1 groups."""
import numpy as np
import pytest

import oracle_ffi as O
import vproxy_amd as V

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def clf():
    c = V.Classifier(0)
    yield c
    c.close()


def _groups(rng, ng):
    groups = []
    for _ in range(ng):
        g = []
        for _ in range(int(rng.integers(0, 14))):
            if g and rng.random() < 0.15:
                ip = g[int(rng.integers(0, len(g)))][0]
            else:
                ip = bytes(rng.integers(0, 256, 4 if rng.random() < 0.7 else 16).astype(np.uint8))
            g.append((ip, int(rng.choice([80, 443, 8080])), int(rng.choice([0, 1, 1, 3])),
                      bool(rng.random() < 0.8)))
        groups.append(g)
    return groups


def _want(groups, grp, src, view):
    out = np.empty(len(grp), np.int32)
    for i, g in enumerate(grp):
        if g < 0 or g >= len(groups):
            out[i] = -1
        else:
            out[i] = O.source_select(groups[g], view, bytes(src[i]))
    return out


def test_source_select_vs_oracle(clf):
    import torch
    rng = np.random.default_rng(21)
    groups = _groups(rng, 700)
    clf.compile_servers(groups)
    n = 20000
    grp = rng.integers(-1, len(groups) + 2, n).astype(np.int32)
    src4 = rng.integers(0, 2**32, n, dtype=np.uint64).astype(np.uint32)
    src4_bytes = src4.astype(">u4").view(np.uint8).reshape(-1, 4)
    src6 = rng.integers(0, 256, (n, 16)).astype(np.uint8)
    for view in (V.SOURCE_ALL, V.SOURCE_IPV4, V.SOURCE_IPV6):
        got = clf.source_select(grp, src4, view)
        np.testing.assert_array_equal(got, _want(groups, grp, src4_bytes, view))
        got6 = clf.source_select(grp, src6, view)
        np.testing.assert_array_equal(got6, _want(groups, grp, src6, view))
        dev = clf.source_select(torch.from_numpy(grp).cuda(),
                                torch.from_numpy(src4.view(np.int32)).cuda(), view)
        torch.cuda.synchronize()
        np.testing.assert_array_equal(dev.cpu().numpy(), got)
    # health checks flip: the device table follows vc_servers_set_health
    flat = [sv for g in groups for sv in g]
    healthy = rng.random(len(flat)) < 0.5
    clf.set_server_health(healthy.astype(np.uint8))
    k = 0
    sick = []
    for g in groups:
        sick.append([(a, p, w, bool(healthy[k + j])) for j, (a, p, w, h) in enumerate(g)])
        k += len(g)
    got = clf.source_select(grp, src4, V.SOURCE_ALL)
    np.testing.assert_array_equal(got, _want(sick, grp, src4_bytes, V.SOURCE_ALL))


@pytest.mark.parametrize("shape", ["many_groups", "long_list"])
def test_source_global_lists(clf, shape):
    """The kernels copy a view's lists (offset, count) into LDS when they fit
    (select.hip kSelLdsMax, ServerImage.view_pk); past that -- more groups
    than the LDS copy holds, or a list of 256+ servers the packed form cannot
    count -- they read the global table.  Both equal the oracle."""
    rng = np.random.default_rng(23 if shape == "many_groups" else 24)
    groups = _groups(rng, 12000 if shape == "many_groups" else 300)
    if shape == "long_list":
        groups[7] = [(bytes(rng.integers(0, 256, 4).astype(np.uint8)), 80, 1,
                      bool(rng.random() < 0.7)) for _ in range(300)]
    clf.compile_servers(groups)
    n = 12000
    grp = rng.integers(-1, len(groups) + 2, n).astype(np.int32)
    if shape == "long_list":
        grp[::3] = 7
    src4 = rng.integers(0, 2**32, n, dtype=np.uint64).astype(np.uint32)
    src4_bytes = src4.astype(">u4").view(np.uint8).reshape(-1, 4)
    src6 = rng.integers(0, 256, (n, 16)).astype(np.uint8)
    for view in (V.SOURCE_ALL, V.SOURCE_IPV4, V.SOURCE_IPV6):
        np.testing.assert_array_equal(clf.source_select(grp, src4, view),
                                      _want(groups, grp, src4_bytes, view))
        np.testing.assert_array_equal(clf.source_select(grp, src6, view),
                                      _want(groups, grp, src6, view))


def test_source_sticky_like_tcplb(clf):
    """TestTcpLB.proxySource: every connection from 127.0.0.1 reaches svr0,
    the backend that answers "0" (TestTcpLB.java:383-405; kats.json source)."""
    import json
    import os
    with open(os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden",
                           "kats.json")) as f:
        cases = json.load(f)["source"]
    for case in cases:
        clf.compile_servers([[tuple(s) for s in case["servers"]]])
        for client, view, want in case["queries"]:
            a, b, c, d = (int(x) for x in client.split("."))
            src = np.full(100, (a << 24) | (b << 16) | (c << 8) | d, np.uint32)
            got = clf.source_select(np.zeros(100, np.int32), src, view)
            assert got.tolist() == [want] * 100, case["source"]


def test_source_errors(clf):
    clf.compile_servers([[("10.0.0.1", 80, 1, True)]])
    with pytest.raises(V.IllegalArgumentException):
        clf.set_server_health(np.ones(2, np.uint8))
    with pytest.raises(V.IllegalArgumentException):
        clf.source_select(np.zeros(1, np.int32), np.zeros(1, np.uint32), view=5)


def test_source_bench_batch(clf):
    """The `source` sub-bench's batch exactly as bench.py builds it
    (bench.source_workload: 10k groups, 128M device-generated clients)
    through vc_source_select_v4_dev: every one of the 128M results equal to
    exact.SourceChecker (ServerGroup.java:377-490,620-664), plus an oracle
    sample."""
    import torch
    import bench as B
    from exact import SourceChecker
    dev = torch.device("cuda", 0)
    n = 128 << 20
    groups, grp, src = B.source_workload(n, dev)
    clf.compile_servers(groups)
    got = clf.source_select(grp, src)
    torch.cuda.synchronize()
    want = SourceChecker(groups, dev).v4(grp, src)
    assert torch.equal(got, want), int((got != want).sum())
    s = np.random.default_rng(5).integers(0, n, 20000)
    gh, sh = grp.cpu().numpy()[s], src.cpu().numpy()[s].view(np.uint32)
    np.testing.assert_array_equal(got.cpu().numpy()[s], O.source_batch_np(groups, 0, gh, sh,
                                                                           nthreads=16))
    assert float((got >= 0).float().mean()) > 0.9


@pytest.mark.parametrize("healthy_frac", [0.5, 0.05, 0.0])
def test_source_health_updates_at_scale(clf, healthy_frac):
    """vc_servers_set_health rebuilds the lists' per-position answers
    (compile.cpp source_pick_table): after each update every one of 32M
    results equals exact.SourceChecker over the new health, in all three
    views -- half the servers down, nearly all down (long probe runs), all
    down (null everywhere) -- and the snapshot taken before the update
    still answers with the old health."""
    import torch
    import bench as B
    from exact import SourceChecker
    dev = torch.device("cuda", 0)
    n = 32 << 20
    groups, grp, src = B.source_workload(n, dev)
    clf.compile_servers(groups)
    before = clf.source_select(grp, src)
    rng = np.random.default_rng(int(healthy_frac * 100) + 7)
    flat = [s for g in groups for s in g]
    h = rng.random(len(flat)) < healthy_frac
    clf.set_server_health(h.astype(np.uint8))
    sick, k = [], 0
    for g in groups:
        sick.append([(a, p, w, bool(h[k + j])) for j, (a, p, w, _) in enumerate(g)])
        k += len(g)
    for view in (V.SOURCE_ALL, V.SOURCE_IPV4, V.SOURCE_IPV6):
        got = clf.source_select(grp, src, view=view)
        torch.cuda.synchronize()
        want = SourceChecker(sick, dev, view=view).v4(grp, src)
        assert torch.equal(got, want), (view, int((got != want).sum()))
    if healthy_frac == 0.0:
        assert bool((got == -1).all())
    # the compile's own health, through a fresh compile, is the first answer
    clf.compile_servers(groups)
    again = clf.source_select(grp, src)
    torch.cuda.synchronize()
    assert torch.equal(again, before)

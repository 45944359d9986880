"""GPU tier: the frame sub-benches' batches exactly as bench.py builds them
(bench.frames_workload: 32M seeded draws from 64K seeded VXLAN frames),
checked item by item.  A result depends only on the item's bytes (and, for
the switch, its sender), so the 64K distinct frames are first checked
against the oracle in full; then every one of the 32M results must equal
its frame's checked result:

- parse:  VXLanPacket / EthernetPacket / Ipv4Packet / Ipv6Packet / TcpPacket
  .from (base/src/main/java/vpacket/*.java) -- every output field;
- mirror: Mirror.switchPacket over the bench's 17 filters
  (base/src/main/java/vmirror/Mirror.java:73-139, FilterConfig.java:27-94);
- switch: bareVXLanAccess.allow(UDP, sender, 4789) for all 32M senders
  (the bench's list: C5's plus a last allow rule for the VXLAN port)
  through exact.AclChecker (SecurityGroup.java:30-45), and the inner
  route (RouteTable.java:44-59) of the frame's destination through
  exact.RouteChecker on the C5 tables, -1 when denied or not IP.
"""
import numpy as np
import pytest

import bench as B
import oracle_ffi as O
import vproxy_amd as V
from exact import AclChecker, RouteChecker
from test_gpu_packets import _rows
from vproxy_amd import workloads as W

pytestmark = pytest.mark.gpu
N = 32 << 20


@pytest.fixture(scope="module")
def frames():
    import torch
    fr, pidx = B.frames_workload(N)
    fblob, foff = W.pack(fr)
    dev = torch.device("cuda", 0)
    blob, off, _ = B.gather_strings_dev(fblob, foff, pidx, dev)
    tb = torch.from_numpy(fblob).to(dev)
    to = torch.from_numpy(foff.astype(np.int32)).to(dev)
    return fr, pidx, (tb, to), (blob, off), torch.from_numpy(pidx).to(dev)


def test_parse_bench_batch(frames):
    import torch
    fr, pidx, tmpl, batch, pi = frames
    clf = V.Classifier(0)
    try:
        t = clf.parse_packets(tmpl, V.LAYER_VXLAN)
        torch.cuda.synchronize()
        uns = {np.dtype(np.int16): np.uint16, np.dtype(np.int32): np.uint32}
        th = {k: (lambda a: a.view(uns.get(a.dtype, a.dtype)))(v.cpu().numpy())
              for k, v in t.items()}
        for i, f in enumerate(fr):                  # the 64K frames against the oracle
            assert _rows(th, i) == O.parse_packet(f, V.LAYER_VXLAN), i
        res = clf.parse_packets(batch, V.LAYER_VXLAN)
        torch.cuda.synchronize()
        for k, v in res.items():                    # all 32M: each its frame's result
            assert torch.equal(v, t[k][pi]), k
        assert (th["status"] == 0).mean() > 0.5
    finally:
        clf.close()


def test_mirror_bench_batch(frames):
    import torch
    fr, pidx, tmpl, batch, pi = frames
    clf = V.Classifier(0)
    try:
        clf.compile_mirror(B.MIRROR_FILTERS)
        ids = {}
        oarr = O.mirror_filters(B.MIRROR_FILTERS, ids)
        tb, to = tmpl
        want = O.mirror_switch_batch_np(oarr, len(B.MIRROR_FILTERS), ids["switch"],
                                        tb.cpu().numpy(), to.cpu().numpy(), 0, nthreads=16)
        got = clf.mirror_switch("switch", batch)
        torch.cuda.synchronize()
        w = torch.from_numpy(want.view(np.int64)).cuda()[pi]
        assert torch.equal(got, w), int((got != w).sum())
        assert (want != 0).mean() > 0.05
    finally:
        clf.close()


def test_switch_bench_batch(frames):
    import torch
    fr, pidx, tmpl, batch, pi = frames
    dev = torch.device("cuda", 0)
    clf = V.Classifier(0)
    try:
        t = B.c5_tables(clf, dev, 1 << 20)
        tcp, udp = B.compile_switch_acl(clf, t)
        r4 = B.switch_senders(N, dev)
        res, acl, allow, route = clf.switch_classify(batch, r4, 4789)
        torch.cuda.synchronize()
        # the bare-VXLAN ACL on every sender: UDP list, bind port
        proto = torch.full((N,), 17, dtype=torch.uint8, device=dev)
        port = torch.full((N,), 4789, dtype=torch.int32, device=dev)
        want_acl, want_allow = AclChecker(tcp, udp, False, dev).v4(proto, r4, port)
        assert torch.equal(acl, want_acl), int((acl != want_acl).sum())
        assert torch.equal(allow, want_allow)
        # the inner route of each frame (the oracle-checked parse of its template)
        p = clf.parse_packets(tmpl, V.LAYER_VXLAN)
        torch.cuda.synchronize()
        ok = p["status"] == 0
        r_v4 = RouteChecker(t.v4_list, 4, dev)(p["dst4"])
        r_v6 = RouteChecker(t.v6_list, 6, dev)(p["dst6"])
        l3 = p["l3"].long()
        tr = torch.where(ok & (l3 == 4), r_v4, torch.where(ok & (l3 == 6), r_v6,
                                                           torch.full_like(r_v4, -1)))
        want_route = torch.where(want_allow == 1, tr[pi], torch.full_like(route, -1))
        assert torch.equal(route, want_route), int((route != want_route).sum())
        assert int((tr >= 0).sum()) > len(fr) // 10
        assert 0.5 < float((want_allow == 1).float().mean()) < 1.0
        assert int((route >= 0).sum()) > N // 10
    finally:
        clf.close()


@pytest.mark.parametrize("n", [1, 2, 63, 64, 65, 127, 129, 4097, 100_003, 800_001, 2_000_003])
def test_frames_ragged_sizes(frames, n):
    """The frame kernels' chunk schedule (chunks.h) at the chunk and pair
    edges and across the work-ticket regimes: the first n frames of the
    bench batch through parse and mirror, every result equal to its frame's
    oracle-checked template result."""
    import torch
    fr, pidx, tmpl, batch, pi = frames
    clf = V.Classifier(0)
    try:
        t = clf.parse_packets(tmpl, V.LAYER_VXLAN)
        clf.compile_mirror(B.MIRROR_FILTERS)
        tm = clf.mirror_switch("switch", tmpl)
        torch.cuda.synchronize()
        sub = (batch[0], batch[1][:n + 1])
        res = clf.parse_packets(sub, V.LAYER_VXLAN)
        m = clf.mirror_switch("switch", sub)
        torch.cuda.synchronize()
        for k, v in res.items():
            assert torch.equal(v, t[k][pi[:n]]), (k, n)
        assert torch.equal(m, tm[pi[:n]]), n
        if n <= 129:                                 # and the oracle on each frame
            uns = {np.dtype(np.int16): np.uint16, np.dtype(np.int32): np.uint32}
            rh = {k: (lambda a: a.view(uns.get(a.dtype, a.dtype)))(v.cpu().numpy())
                  for k, v in res.items()}
            for i in range(n):
                assert _rows(rh, i) == O.parse_packet(fr[pidx[i]], V.LAYER_VXLAN), (n, i)
    finally:
        clf.close()

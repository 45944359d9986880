"""N > 1 path on CPU: world-size-2 `gloo` process groups.

The data path has no collective: each rank classifies its own shard of a
seeded global batch.  Here the oracle stands in for the per-rank kernels
(CPU tier, no GPU), and the test checks the host logic bench.py uses on
the GPU box: bench.gen_packets' index-addressable global batch, the shard
split, the single-bucket counter layout and the all-reduce, against the hit
counters of the whole batch on one rank.
"""
import os
import socket
import types

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

import bench as B
import oracle_ffi as O
from vproxy_amd import workloads as W
from vproxy_amd.dist import HitCounterBucket, shard


def test_shard_covers_batch_once():
    for n in (0, 1, 7, 1000, 125_000_001):
        for world in (1, 2, 3, 8):
            parts = [shard(n, r, world) for r in range(world)]
            assert parts[0][0] == 0 and parts[-1][1] == n
            assert all(a[1] == b[0] for a, b in zip(parts, parts[1:]))
            sizes = [hi - lo for lo, hi in parts]
            assert max(sizes) - min(sizes) <= (1 if n else 0)
    with pytest.raises(ValueError):
        shard(10, 2, 2)


def _tables():
    tcp, udp = W.gen_sg_rules(200, 71, p_range=0.4)
    net, plen = W.gen_v4_prefixes(2000, 72)
    nets = W.v4_nets(net, plen)
    return tcp, udp, net, plen, nets


def _counters(tcp, udp, nets, proto, src, port, dst):
    """Library counter layout (include/vclassify.h VC_COUNTERS_*) from the
    oracle's outputs: ACL [tcp][udp][tcp default][udp default], ROUTE
    [v4][v6][v4 null][v6 null] (v4 only here)."""
    acl, _ = O.sg_batch_v4_np(tcp, udp, False, proto, src, port)
    route = O.rt_batch_v4_np(nets, dst)
    nt, nu = len(tcp), len(udp)
    is_t = proto == 6
    ca = np.bincount(np.where(acl >= 0, np.where(is_t, acl, nt + acl), nt + nu + (~is_t)),
                     minlength=nt + nu + 2)
    cr = np.bincount(np.where(route >= 0, route, len(nets)), minlength=len(nets) + 2)
    return [torch.from_numpy(ca.astype(np.int64)), torch.from_numpy(cr.astype(np.int64))]


def _batch(tcp, udp, net, plen, n, lo=0):
    """Items [lo, lo + n) of the seeded global batch (bench.gen_packets)."""
    t = types.SimpleNamespace(tcp=tcp, udp=udp, net=net, plen=plen)
    proto, src, dst, port, _ = (x.numpy() for x in B.gen_packets(lo, n, t, 1000, seed=73))
    return proto, src.view(np.uint32), port.view(np.uint16), dst.view(np.uint32)


def test_global_batch_is_shardable():
    """Rank r's slice generated on its own equals the same slice of the
    whole batch, for every world size (bench.py generates only its shard)."""
    tcp, udp, net, plen, nets = _tables()
    n = 10007
    whole = _batch(tcp, udp, net, plen, n)
    assert (whole[0] == 6).mean() > 0.4 and (whole[0] == 17).mean() > 0.4
    for world in (2, 3, 8):
        for r in range(world):
            lo, hi = shard(n, r, world)
            part = _batch(tcp, udp, net, plen, hi - lo, lo)
            for a, b in zip(part, whole):
                np.testing.assert_array_equal(a, b[lo:hi])


def _worker(rank, world, port, n, q):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        tcp, udp, net, plen, nets = _tables()                 # replicated tables
        lo, hi = shard(n, rank, world)
        proto, src, dport, dst = _batch(tcp, udp, net, plen, hi - lo, lo)   # this rank's shard
        mine = _counters(tcp, udp, nets, proto, src, dport, dst)
        b = HitCounterBucket([t.numel() for t in mine], "cpu")
        for i, t in enumerate(mine):
            b.fill(i, t)
        views = b.reduce()
        q.put((rank, [v.numpy().copy() for v in views], hi - lo))
    finally:
        dist.destroy_process_group()


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


@pytest.mark.parametrize("world", [2])
def test_counter_allreduce_equals_single_rank(world):
    n = 30011                                                  # odd: uneven shards
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, n, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = [q.get(timeout=120) for _ in procs]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    tcp, udp, net, plen, nets = _tables()
    want = [t.numpy() for t in _counters(tcp, udp, nets, *_batch(tcp, udp, net, plen, n))]
    assert sum(r[2] for r in res) == n
    for rank, views, _ in res:
        for got, exp in zip(views, want):
            np.testing.assert_array_equal(got, exp)


@pytest.mark.parametrize("k", [32, 64, 96, 128])
def test_cu_split_balanced_over_xcds(k):
    """bench.cu_split: CU-mask bit i selects a CU of XCD i mod 8 (measured,
    profiles/r03_cu_scaling.jsonl), so both shares must hold the same number
    of CUs on every XCD, a multiple of 4 -- an uneven share runs part of a
    static-slice kernel's workgroups in a second round."""
    pick, rest = B.cu_split(256, k)
    assert sorted(pick + rest) == list(range(256))
    for share in (pick, rest):
        per_xcd = [sum(1 for c in share if c % 8 == x) for x in range(8)]
        assert len(set(per_xcd)) == 1 and per_xcd[0] % 4 == 0, per_xcd


def _c5_digests(perturb):
    """The C5 tables exactly as bench.c5_tables compiles them, built in host
    memory by libvclassify's own compilers (vc_digest_*: no device)."""
    import vproxy_amd as V
    t = B.c5_rule_tables()
    if perturb:                                   # one rule's port range differs
        t.tcp = t.tcp.copy()
        t.tcp["max_port"][17] = (int(t.tcp["max_port"][17]) + 1) % 65536
    rt = V.RouteTable()
    allnets = np.concatenate([W.v4_nets(t.net, t.plen), W.v6_nets(t.hi, t.lo, t.p6)])
    arr, n_all, keep = W.as_ctypes(allnets, V._lib.VcNet)
    rt.add_rules("bgp", arr, n=n_all)
    a4, n4 = rt.rules_raw(4)
    a6, n6 = rt.rules_raw(6)
    v4 = np.frombuffer(bytes(a4)[:n4 * 40], W.NET_DT).copy()
    v6 = np.frombuffer(bytes(a6)[:n6 * 40], W.NET_DT).copy()
    assert n4 == 980848 and n6 == 200000
    return [V.digest_acl(t.tcp, t.udp, False), V.digest_routes(v4, v6),
            V.digest_upstream(t.groups)]


def _replica_worker(rank, world, port, perturb_rank, q):
    from vproxy_amd.dist import check_replicated
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        try:
            d = _c5_digests(rank == perturb_rank)
        except Exception as e:                     # report, do not leave the parent waiting
            q.put((rank, "error", repr(e)))
            raise
        try:
            q.put((rank, "ok", check_replicated(d)))
        except RuntimeError as e:
            q.put((rank, "mismatch", str(e)))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("perturb_rank", [-1, 1])
def test_replicated_c5_images_are_identical(perturb_rank):
    """Replicated tables are what make the summed hit counters meaningful:
    two spawned ranks compile the C5-shaped tables (10k ACL rules, 980,848 +
    200,000 routes, 100k groups) through libvclassify and the digests of
    the compiled images agree (vproxy_amd.dist.check_replicated, which
    bench.py runs before timing at N > 1); one differing rule on one rank is
    caught on every rank."""
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_replica_worker, args=(r, world, port, perturb_rank, q))
             for r in range(world)]
    for p in procs:
        p.start()
    res = sorted(q.get(timeout=240) for _ in procs)
    assert all(r[1] != "error" for r in res), res
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    if perturb_rank < 0:
        assert [r[1] for r in res] == ["ok", "ok"]
        rows = res[0][2]
        assert rows[0] == rows[1] and len(set(rows[0])) == 3
    else:
        assert [r[1] for r in res] == ["mismatch", "mismatch"]
        assert "[1]" in res[0][2]

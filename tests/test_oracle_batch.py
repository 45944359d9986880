"""CPU tier: the oracle's batched, threaded forms (used as GPU-test checkers
and as bench.py's cpu_baseline legs) equal its one-item restatements."""
import numpy as np

import oracle_ffi as O
from vproxy_amd import workloads as W

from cases import gen_frames


def test_dns_batch_equals_single():
    groups, ghosts = W.gen_groups(300, 3, wildcard=False)
    pairs = [("h%d.hosts.local" % i, i) for i in range(50)] + [("h%d.hosts.local." % i, i)
                                                              for i in range(50)]
    names = W.gen_hostnames(ghosts, 2000, 4, dns=True, port_frac=0)
    names += [b"h7.hosts.local.", b"10.1.2.3.", b"::1.", b"x.vproxy.local.", b"caf\xe9.test."]
    blob, off = W.pack(names)
    og, oh = O.Groups(groups), O.Hosts(pairs)
    kind, value = O.dns_batch_np(oh, og, blob, off, nthreads=4)
    for i, q in enumerate(names):
        v = O.C.c_int32()
        k = O.lib().vo_dns_classify(O.C.byref(oh.h), og.arr, og.n, q, len(q), O.C.byref(v))
        assert (kind[i], value[i]) == (k, v.value), q
    assert len(set(kind.tolist())) >= 4


def test_parse_batch_equals_single():
    rng = np.random.default_rng(5)
    frames = gen_frames(rng, 3000)
    blob, off = W.pack(frames)
    out = O.parse_batch_np(blob, off, 0, nthreads=4)
    for i, f in enumerate(frames):
        p = O.parse_packet(f, 0)
        n = 16 if out[i].l3 == 6 else 4
        assert (out[i].status, out[i].l3, bytes(out[i].dst[:n]).hex()) == \
            (p["status"], p["l3"], p["dst"]), i


def test_switch_batch_equals_composition():
    rng = np.random.default_rng(6)
    tcp, udp = W.gen_sg_rules(400, 7, p_range=0.5)
    udp = np.concatenate([udp, W.gen_sg_rules(4, 8)[1]])
    udp["min_port"][::2], udp["max_port"][::2] = 0, 65535     # half cover the bind port
    frames = gen_frames(rng, 4000)
    blob, off = W.pack(frames)
    n = len(frames)
    net, plen = W.gen_v4_prefixes(3000, 9)
    v4 = W.v4_nets(net, plen)
    hi, lo, p6 = W.gen_v6_prefixes(1000, 10)
    v6 = W.v6_nets(hi, lo, p6)
    remote = rng.integers(0, 2**32, n, dtype=np.uint64).astype(np.uint32)
    ip, mk = W.rule_v4_fields(udp)                  # half the senders inside a UDP rule
    r = rng.integers(0, len(udp), n)
    inside = (ip[r] | (remote & ~mk[r])).astype(np.uint32)
    remote[::2] = inside[::2]
    acl, allow, route = O.switch_batch_np(tcp, udp, False, blob, off, remote, 4789, v4, v6,
                                          nthreads=4)
    wa, wv = O.sg_batch_v4_np(tcp, udp, False, np.full(n, 17, np.uint8), remote,
                              np.full(n, 4789, np.uint16))
    np.testing.assert_array_equal(acl, wa)
    np.testing.assert_array_equal(allow, wv)
    assert 0.05 < allow.mean() < 0.95
    pk = O.parse_batch_np(blob, off, 0)
    for i in range(n):
        want = -1
        if wv[i] and pk[i].status == 0 and pk[i].l3 in (4, 6):
            if pk[i].l3 == 4:
                d = np.frombuffer(bytes(pk[i].dst[:4]), ">u4").astype(np.uint32)
                want = O.rt_batch_v4_np(v4, d)[0]
            else:
                want = O.rt_batch_v6_np(v6, np.frombuffer(bytes(pk[i].dst[:16]), np.uint8)
                                        .reshape(1, 16))[0]
        assert route[i] == want, i


def test_cert_and_mirror_and_source_batches():
    rng = np.random.default_rng(12)
    _, hosts = W.gen_groups(400, 13, wildcard=False)
    holders = [[hosts[i], "*." + hosts[i + 1]] for i in range(0, len(hosts), 2)]
    certs = O.Certs(holders)
    snis = [x.split(b":")[0] for x in W.gen_hostnames(hosts, 2000, 14)]
    blob, off = W.pack(snis)
    out = O.cert_batch_np(certs, blob, off, nthreads=4)
    assert [certs.choose(s.decode()) for s in snis] == list(out)
    ids = {}
    filters = [{"origin": "switch", "mirror": i % 8, "network": "%d.0.0.0/8" % (i + 1),
                "network2": "10.0.0.0/8"} for i in range(16)]
    arr = O.mirror_filters(filters, ids)
    frames = gen_frames(rng, 2000)
    fb, fo = W.pack(frames)
    m = O.mirror_switch_batch_np(arr, len(filters), ids["switch"], fb, fo, 0, nthreads=4)
    assert [O.mirror_switch(arr, len(filters), ids["switch"], f, 0) for f in frames] == \
        [int(x) for x in m]
    groups = [[(bytes(rng.integers(0, 256, 4).astype(np.uint8)), 80, int(rng.integers(0, 3)),
                rng.random() < 0.7) for _ in range(int(rng.integers(1, 9)))] for _ in range(300)]
    grp = rng.integers(0, len(groups), 5000).astype(np.int32)
    src = rng.integers(0, 2**32, 5000, dtype=np.uint64).astype(np.uint32)
    out = O.source_batch_np(groups, 0, grp, src, nthreads=4)
    for i in range(len(grp)):
        b = int(src[i]).to_bytes(4, "big")
        assert out[i] == O.source_select(groups[grp[i]], 0, b), i


def test_mirror_match_batch_equals_single():
    """vo_mirror_match_batch (the mirroritems bench's CPU leg) over
    vc_mirror_items-shaped columns equals vo_mirror_match per item."""
    from cases import gen_mirror_case, mirror_columns
    import vproxy_amd as V
    from vproxy_amd.mirror import MirrorFilters, parse_mac
    rng = np.random.default_rng(33)
    filters, items = gen_mirror_case(rng, 30, 3000)
    mf = MirrorFilters()
    mf.build(filters)
    ids = {}
    arr = O.mirror_filters(filters, ids)
    cols = mirror_columns(items, lambda s: mf.id_of(s, create=False), V.parse_ip)
    for origin in ("switch", "tcp-lb"):
        oid = ids.get(origin, -2)
        got = O.mirror_match_batch_np(arr, len(filters), oid, cols, nthreads=4)
        want = [O.mirror_match(arr, len(filters), oid, parse_mac(i["mac_src"]),
                               parse_mac(i["mac_dst"]),
                               None if i["ip_src"] is None else O.parse_ip(i["ip_src"]),
                               None if i["ip_dst"] is None else O.parse_ip(i["ip_dst"]),
                               ids.get(i["transport"], -2) if i["transport"] else -1,
                               i["port_src"], i["port_dst"],
                               ids.get(i["app"], -2) if i["app"] else -1) for i in items]
        assert [int(x) for x in got] == want, origin

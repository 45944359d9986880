"""ServerGroup source hashing (method == source) on the CPU tier: the C
oracle (oracle/vc_oracle.c vo_source_*) against an independent Python
restatement of ServerGroup.java:377-490 / 620-664 and hand-derived vectors.

The reference's only test of this method (TestTcpLB.proxySource,
test/src/test/java/vproxy/test/cases/TestTcpLB.java:383-405) checks that one
client always reaches the same backend; the vectors below pin the hash
itself, the signed-byte sort and the health-probe walk.
"""
import functools
import random

import oracle_ffi as O


def j32(x):
    x &= 0xFFFFFFFF
    return x - (1 << 32) if x >= (1 << 31) else x


def py_hash(bs):
    """SOURCE.hash, ServerGroup.java:387-397"""
    h = 0
    for b in bs:
        sb = b - 256 if b >= 128 else b
        h = j32(sb + (h << 6) + (h << 16) - h)
    h = abs(h) if h != -(1 << 31) else h          # Math.abs(MIN_VALUE) == MIN_VALUE
    return 0 if h < 0 else h


def py_list(servers, view):
    """sourceReset, ServerGroup.java:620-664"""
    ids = [i for i, (ip, port, w, hl) in enumerate(servers)
           if w > 0 and (view == 0 or (view == 4) == (len(ip) == 4))]

    def cmp(a, b):
        ba, bb = servers[a][0], servers[b][0]
        if len(ba) != len(bb):
            return 1 if len(ba) > len(bb) else -1
        for x, y in zip(ba, bb):
            d = (x - 256 if x >= 128 else x) - (y - 256 if y >= 128 else y)
            if d:
                return d
        return servers[a][1] - servers[b][1]
    return sorted(ids, key=functools.cmp_to_key(cmp))      # stable, like List.sort


def py_select(servers, view, src):
    """sourceHashGet, ServerGroup.java:464-490"""
    lst = py_list(servers, view)
    h = py_hash(src)
    for _ in range(len(lst)):
        idx = h % len(lst)
        if servers[lst[idx]][3]:
            return lst[idx]
        h = idx + 1
    return -1


def test_hash_vectors():
    # 127.0.0.1: 127 -> 127; 0 -> 127*64 + 127*65536 - 127 = 8331073;
    # 0 -> 8331073*65599 wrapped; 1 -> ...
    assert py_hash(b"\x7f") == 127
    assert py_hash(b"\x7f\x00") == 8331073
    assert py_hash(bytes([0, 0, 0, 0])) == 0
    assert py_hash(bytes([255])) == 1                       # byte -1 -> abs(-1)
    for bs in (b"\x7f\x00\x00\x01", bytes([10, 0, 0, 200]), bytes([192, 168, 1, 1]),
               bytes(range(16)), bytes([255] * 16), b""):
        assert O.source_hash(bs) == py_hash(bs), bs
    rng = random.Random(5)
    for _ in range(2000):
        bs = bytes(rng.randrange(256) for _ in range(rng.choice((4, 16))))
        assert O.source_hash(bs) == py_hash(bs)


def test_min_value_quirk():
    """Math.abs(Integer.MIN_VALUE) stays negative -> hash 0 (:392-395).
    A 16-byte address whose sdbm is exactly MIN_VALUE, found by meeting in
    the middle (sdbm is h * 65599 + signed byte, and 65599 is invertible
    mod 2^32): 11 zero bytes keep h = 0, 3 bytes forward, 2 bytes back."""
    import numpy as np
    M = 1 << 32
    inv = pow(65599, -1, M)
    sb = np.arange(256, dtype=np.int64)
    sb = np.where(sb >= 128, sb - 256, sb)
    h = np.zeros(1, np.int64)
    for _ in range(3):                                   # forward: all 3-byte prefixes
        h = ((h[:, None] * 65599 + sb[None, :]) % M).reshape(-1)
    target = (-(1 << 31)) % M
    x = ((target - sb) % M) * inv % M                    # state before the last byte
    h3 = ((x[:, None] - sb[None, :]) % M) * inv % M      # state before the last two
    hit = np.isin(h3.reshape(-1), h)
    k = int(np.flatnonzero(hit)[0])
    last, prev = divmod(k, 256)                          # h3[last_idx, prev_idx]
    fwd = int(np.flatnonzero(h == h3.reshape(-1)[k])[0])
    a, rem = divmod(fwd, 65536)
    bb, c = divmod(rem, 256)
    bs = bytes(11) + bytes([a, bb, c, prev, last])
    assert py_hash(bs) == 0 and O.source_hash(bs) == 0
    assert j32(sum((b - 256 if b >= 128 else b) * pow(65599, len(bs) - 1 - i, M)
                   for i, b in enumerate(bs))) == -(1 << 31)


def test_signed_sort_and_probe():
    ip = lambda *b: bytes(b)
    servers = [(ip(10, 0, 0, 1), 80, 1, True), (ip(10, 0, 0, 200), 80, 1, True),
               (ip(10, 0, 0, 1), 79, 1, True), (bytes(16), 80, 1, True),
               (ip(10, 0, 0, 5), 80, 0, True)]                  # weight 0: never listed
    # 200 is byte -56 < 1; IPv4 (4 bytes) before IPv6; port breaks ties
    assert py_list(servers, 0) == [1, 2, 0, 3] == O.source_list(servers, 0)
    assert O.source_list(servers, 4) == [1, 2, 0]
    assert O.source_list(servers, 6) == [3]
    # an unhealthy pick moves to the next server in the sorted list
    src = bytes([1, 2, 3, 4])
    first = py_select(servers, 0, src)
    sick = [(a, p, w, i != first) for i, (a, p, w, h) in enumerate(servers)]
    lst = py_list(servers, 0)
    nxt = lst[(lst.index(first) + 1) % len(lst)]
    assert O.source_select(sick, 0, src) == py_select(sick, 0, src) == nxt
    # no healthy server -> null
    dead = [(a, p, w, False) for a, p, w, h in servers]
    assert O.source_select(dead, 0, src) == -1
    assert O.source_select([], 0, src) == -1


def test_oracle_vs_restatement_random():
    rng = random.Random(11)
    for _ in range(300):
        servers = []
        for _ in range(rng.randrange(0, 12)):
            a = bytes(rng.randrange(256) for _ in range(rng.choice((4, 16))))
            if servers and rng.random() < 0.2:
                a = servers[rng.randrange(len(servers))][0]            # duplicate address
            servers.append((a, rng.choice((80, 443, 8080)), rng.choice((0, 1, 1, 2, 5)),
                            rng.random() < 0.7))
        for view in (0, 4, 6):
            assert O.source_list(servers, view) == py_list(servers, view)
            for _ in range(5):
                src = bytes(rng.randrange(256) for _ in range(rng.choice((4, 16))))
                assert O.source_select(servers, view, src) == py_select(servers, view, src)

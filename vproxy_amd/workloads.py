"""Seeded synthetic workloads for the BASELINE.json configs.

C1  SecurityGroup 64 rules + RouteTable 256 IPv4 CIDRs, 1M 5-tuples
C2  SecurityGroup 10k rules with port ranges, 64M IPv4 5-tuples
C3  RouteTable ~1M IPv4 + 200k IPv6 prefixes (shortest-first), 256M lookups
C4  100k hint-host groups vs 16M hostnames (Host/SNI + DNS flavour)
C5  combined ACL -> route -> host pipeline over packet batches

Rule tables are numpy structured arrays whose layout is the C struct layout
of include/vclassify.h (vc_net, vc_acl_rule), so they pass to the C ABI (and
to the oracle, whose vo_net/vo_sg_rule have the same layout) without copies.
There is no real traffic or dataset here: everything is synthetic.
"""
import ctypes as C

import numpy as np

NET_DT = np.dtype([("ip", np.uint8, 16), ("mask", np.uint8, 16), ("ip_len", np.int32),
                   ("mask_len", np.int32)])
RULE_DT = np.dtype([("net", NET_DT), ("min_port", np.int32), ("max_port", np.int32),
                    ("allow", np.int32)])
assert NET_DT.itemsize == 40 and RULE_DT.itemsize == 52

SEED = 0x5EED


def _mask32(plen):
    plen = np.asarray(plen, dtype=np.int64)
    return ((np.int64(0xFFFFFFFF) << (32 - plen)) & 0xFFFFFFFF).astype(np.uint32)


def v4_nets(addr, plen):
    """uint32 network addresses + prefix lengths -> NET_DT array."""
    addr = np.asarray(addr, dtype=np.uint32)
    plen = np.asarray(plen, dtype=np.int64)
    n = len(addr)
    out = np.zeros(n, NET_DT)
    out["ip_len"] = 4
    out["mask_len"] = 4
    be = addr.astype(">u4").view(np.uint8).reshape(n, 4)
    out["ip"][:, :4] = be
    out["mask"][:, :4] = _mask32(plen).astype(">u4").view(np.uint8).reshape(n, 4)
    return out


def v6_nets(hi, lo, plen):
    """(hi, lo) uint64 network halves + prefix lengths -> NET_DT array
    (mask bytes = Network.parseMask: 4 bytes when plen <= 32)."""
    hi = np.asarray(hi, dtype=np.uint64)
    lo = np.asarray(lo, dtype=np.uint64)
    plen = np.asarray(plen, dtype=np.int64)
    n = len(hi)
    out = np.zeros(n, NET_DT)
    out["ip_len"] = 16
    out["mask_len"] = np.where(plen > 32, 16, 4)
    out["ip"][:, :8] = hi.astype(">u8").view(np.uint8).reshape(n, 8)
    out["ip"][:, 8:] = lo.astype(">u8").view(np.uint8).reshape(n, 8)
    bits = np.arange(128)
    mbits = (bits[None, :] < plen[:, None]).astype(np.uint8)
    out["mask"] = np.packbits(mbits, axis=1)
    return out


def as_ctypes(arr, ctype):
    """Structured numpy array -> ctypes array of `ctype` over the same memory."""
    arr = np.ascontiguousarray(arr)
    n = max(1, len(arr))
    if len(arr) == 0:
        return (ctype * 1)(), 0, arr
    return (ctype * n).from_buffer(arr), len(arr), arr


# ---------------------------------------------------------------------------
# SecurityGroup rules + 5-tuples
# ---------------------------------------------------------------------------
def gen_sg_rules(n, seed, p_range=0.3, weighted=True):
    """n rules split TCP/UDP 50/50.  Returns (tcp RULE_DT, udp RULE_DT)."""
    rng = np.random.default_rng(seed)
    proto = rng.choice(np.array([6, 17]), n)
    if weighted:   # /8-/32 weighted to /16-/28
        u = rng.random(n)
        plen = np.where(u < 0.05, rng.integers(8, 16, n),
                        np.where(u < 0.90, rng.integers(16, 29, n), rng.integers(29, 33, n)))
    else:
        plen = rng.integers(8, 33, n)
    net = rng.integers(0, 2**32, n, dtype=np.uint64).astype(np.uint32) & _mask32(plen)
    single = rng.random(n) >= p_range
    a = rng.integers(0, 65536, n)
    w = np.minimum(rng.geometric(1 / 2048, n), 65535)
    b = np.minimum(a + w, 65535)
    lo = a
    hi = np.where(single, a, b)
    allow = (rng.random(n) < 0.5).astype(np.int32)
    # SecurityGroup.addRule rejects exact duplicates (SecurityGroup.java:67-74)
    key = np.stack([proto, net.astype(np.int64), plen, lo, hi], axis=1)
    _, first = np.unique(key, axis=0, return_index=True)
    keep = np.sort(first)
    rules = np.zeros(len(keep), RULE_DT)
    rules["net"] = v4_nets(net[keep], plen[keep])
    rules["min_port"] = lo[keep]
    rules["max_port"] = hi[keep]
    rules["allow"] = allow[keep]
    pk = proto[keep]
    return rules[pk == 6].copy(), rules[pk == 17].copy()


def rule_v4_fields(rules):
    ip = rules["net"]["ip"][:, :4].copy().view(">u4").reshape(-1).astype(np.uint32)
    mk = rules["net"]["mask"][:, :4].copy().view(">u4").reshape(-1).astype(np.uint32)
    return ip, mk


def gen_acl_queries(tcp, udp, n, seed, inside=0.5):
    """proto/src4/port: `inside` of the items hit a random rule's network and
    port range (same protocol), the rest are uniform."""
    rng = np.random.default_rng(seed)
    proto = rng.choice(np.array([6, 17], dtype=np.uint8), n)
    src = rng.integers(0, 2**32, n, dtype=np.uint64).astype(np.uint32)
    port = rng.integers(0, 65536, n).astype(np.uint16)
    pick = rng.random(n) < inside
    for p, rules in ((6, tcp), (17, udp)):
        if len(rules) == 0:
            continue
        sel = np.nonzero(pick & (proto == p))[0]
        r = rng.integers(0, len(rules), len(sel))
        ip, mk = rule_v4_fields(rules)
        src[sel] = ip[r] | (src[sel] & ~mk[r])
        lo = rules["min_port"][r].astype(np.int64)
        hi = rules["max_port"][r].astype(np.int64)
        port[sel] = (lo + (rng.random(len(sel)) * (hi - lo + 1)).astype(np.int64)).astype(np.uint16)
    return proto, src, port


# ---------------------------------------------------------------------------
# Route tables
# ---------------------------------------------------------------------------
def gen_v4_prefixes(n, seed, dist=((24, 24, 0.60), (16, 23, 0.35), (8, 15, 0.05))):
    """BGP-like IPv4 prefixes (unique), returned sorted shortest-first."""
    rng = np.random.default_rng(seed)
    m = int(n * 1.05) + 16
    u = rng.random(m)
    plen = np.empty(m, np.int64)
    acc = 0.0
    lo_u = 0.0
    for a, b, p in dist:
        acc += p
        sel = (u >= lo_u) & (u < acc)
        plen[sel] = rng.integers(a, b + 1, sel.sum())
        lo_u = acc
    plen[u >= lo_u] = dist[-1][1]
    net = rng.integers(0, 2**32, m, dtype=np.uint64).astype(np.uint32) & _mask32(plen)
    key = (net.astype(np.uint64) << np.uint64(8)) | plen.astype(np.uint64)
    _, first = np.unique(key, return_index=True)
    first = np.sort(first)[:n]
    net, plen = net[first], plen[first]
    order = np.argsort(plen, kind="stable")
    return net[order], plen[order]


def gen_v6_prefixes(n, seed):
    """IPv6 prefixes (/32-/48 dominant, some /64, a few /20-/31), unique,
    sorted shortest-first.  Addresses drawn under 2000::/3."""
    rng = np.random.default_rng(seed)
    m = int(n * 1.05) + 16
    u = rng.random(m)
    plen = np.where(u < 0.05, rng.integers(20, 32, m),
                    np.where(u < 0.90, rng.integers(32, 49, m), 64))
    hi = rng.integers(0, 2**61, m, dtype=np.uint64) | np.uint64(0x2000000000000000)
    shift = (64 - np.minimum(plen, 64)).astype(np.uint64)
    hmask = np.where(plen >= 64, np.uint64(0xFFFFFFFFFFFFFFFF),
                     (np.uint64(0xFFFFFFFFFFFFFFFF) << shift))
    hi = hi & hmask
    lo = np.zeros(m, np.uint64)
    key = np.stack([hi.view(np.int64), plen], axis=1)
    _, first = np.unique(key, axis=0, return_index=True)
    first = np.sort(first)[:n]
    hi, lo, plen = hi[first], lo[first], plen[first]
    order = np.argsort(plen, kind="stable")
    return hi[order], lo[order], plen[order]


def v4_lookups(net, plen, n, seed, inside=0.9):
    rng = np.random.default_rng(seed)
    out = rng.integers(0, 2**32, n, dtype=np.uint64).astype(np.uint32)
    sel = np.nonzero(rng.random(n) < inside)[0]
    r = rng.integers(0, len(net), len(sel))
    out[sel] = net[r] | (out[sel] & ~_mask32(plen[r]))
    return out


def v6_lookups(hi, lo, plen, n, seed, inside=0.9):
    """-> uint8 [n, 16]"""
    rng = np.random.default_rng(seed)
    qh = rng.integers(0, 2**64, n, dtype=np.uint64)
    ql = rng.integers(0, 2**64, n, dtype=np.uint64)
    sel = np.nonzero(rng.random(n) < inside)[0]
    r = rng.integers(0, len(hi), len(sel))
    p = plen[r]
    sh = (64 - np.minimum(p, 64)).astype(np.uint64)
    hm = np.where(p >= 64, np.uint64(0xFFFFFFFFFFFFFFFF), np.uint64(0xFFFFFFFFFFFFFFFF) << sh)
    qh[sel] = hi[r] | (qh[sel] & ~hm)
    out = np.empty((n, 16), np.uint8)
    out[:, :8] = qh.astype(">u8").view(np.uint8).reshape(n, 8)
    out[:, 8:] = ql.astype(">u8").view(np.uint8).reshape(n, 8)
    return out


def v4_to_bytes(a):
    a = np.asarray(a, dtype=np.uint32)
    return a.astype(">u4").view(np.uint8).reshape(len(a), 4)


# ---------------------------------------------------------------------------
# Upstream groups + hostnames
# ---------------------------------------------------------------------------
_TLDS = ["com", "net", "org", "io", "dev", "cn", "de", "co", "app", "info"]
_ALPHA = np.frombuffer(b"abcdefghijklmnopqrstuvwxyz0123456789", dtype=np.uint8)


def _labels(rng, k, lo=3, hi=10):
    lens = rng.integers(lo, hi + 1, k)
    chars = _ALPHA[rng.integers(0, 26, int(lens.sum()))].tobytes().decode()
    out, p = [], 0
    for L in lens:
        out.append(chars[p:p + L])
        p += L
    return out


def gen_groups(n, seed, port_frac=0.05, wildcard=True):
    """n ServerGroupHandles, each with a hint-host of 2-4 labels (unique),
    5 % with a hint-port, one "*" group (weight 0 everywhere: WRR unused).
    Returns (groups spec list, host strings)."""
    rng = np.random.default_rng(seed)
    hosts = set()
    out = []
    nl = rng.integers(2, 5, n * 2)
    labels = _labels(rng, int(nl.sum()) + 16)
    li = 0
    k = 0
    while len(out) < n:
        L = int(nl[k % len(nl)])
        k += 1
        parts = labels[li:li + L - 1]
        li += L - 1
        if li + 8 >= len(labels):
            labels = _labels(rng, len(labels))
            li = 0
        h = ".".join(parts + [_TLDS[int(rng.integers(0, len(_TLDS)))]])
        if h in hosts:
            continue
        hosts.add(h)
        out.append(h)
    groups = []
    ports = rng.integers(1, 65536, n)
    has_port = rng.random(n) < port_frac
    for i, h in enumerate(out):
        g = {"host": h}
        if has_port[i]:
            g["port"] = str(int(ports[i]))
        groups.append(({}, g))
    if wildcard:
        j = int(rng.integers(0, n))
        groups[j] = ({}, {"host": "*"})
        out[j] = "*"
    return groups, out


def gen_hostnames(group_hosts, n, seed, pool=None, dns=False, exact=0.4, sub=0.4, port_frac=0.1):
    """n hostnames: `exact` equal to a group's host, `sub` a sub-domain of
    one, the rest misses; `port_frac` carry ":port" (Host-header style,
    formatHost strips it and a leading "www.").  dns=True appends the
    trailing dot of a DNS qname instead.  A pool of distinct names is built
    and sampled so very large n stays fast.  Returns list[bytes]."""
    rng = np.random.default_rng(seed)
    pool = pool or min(n, 1 << 20)
    real = [h for h in group_hosts if h != "*"]
    gi = rng.integers(0, len(real), pool)
    u = rng.random(pool)
    lab = _labels(rng, pool)
    names = []
    for i in range(pool):
        if u[i] < exact:
            h = real[gi[i]]
        elif u[i] < exact + sub:
            h = ("www." if (i & 7) == 0 else lab[i] + ".") + real[gi[i]]
        else:
            h = lab[i] + "." + real[gi[i]].split(".")[0] + ".invalid"
        names.append(h)
    hp = rng.random(pool) < port_frac
    pv = rng.integers(1, 65536, pool)
    out = []
    for i, h in enumerate(names):
        if dns:
            h = h + "."
        elif hp[i]:
            h = "%s:%d" % (h, pv[i])
        out.append(h.encode())
    if n == pool:
        return out
    idx = rng.integers(0, pool, n)
    return [out[j] for j in idx]


def pack(names):
    """list[bytes] -> (blob uint8, off uint32[n+1])"""
    lens = np.fromiter((len(b) for b in names), dtype=np.int64, count=len(names))
    off = np.zeros(len(names) + 1, np.int64)
    np.cumsum(lens, out=off[1:])
    blob = np.frombuffer(b"".join(names) or b"\0", dtype=np.uint8).copy()
    return blob, off.astype(np.uint32)


def gen_vxlan_frames(n, seed):
    """n distinct VXLAN frames as the vswitch receives them (benchmark
    templates): 70 % IPv4/TCP (half with SYN-style options), 15 % IPv4/UDP,
    10 % IPv6/TCP, 5 % ARP; 0-64 payload bytes.  list[bytes]."""
    rng = np.random.default_rng(seed)
    out = []
    for _ in range(n):
        r = rng.random()
        rb = lambda k: rng.integers(0, 256, k).astype(np.uint8).tobytes()
        payload = rb(int(rng.integers(0, 65)))
        vx = bytes([8, 0, 0, 0]) + rb(3) + b"\0"
        eth = rb(12)
        if r < 0.95:
            opts = bytes([2, 4, 5, 180, 1, 3, 3, 6, 1, 1, 8, 10]) + rb(8) + bytes([4, 2, 0, 0]) \
                if (r < 0.70 and rng.random() < 0.5) else b""
            if r < 0.85 or r >= 0.85 + 0.10:
                if r < 0.70:
                    l4 = rb(12) + bytes([((20 + len(opts)) // 4) << 4, 0x18]) + rb(6) + opts + payload
                    proto = 6
                else:
                    l4 = rb(4) + bytes([0, 8 + len(payload) >> 8 & 255]) + rb(2) + payload
                    proto = 17
                total = 20 + len(l4)
                ip = bytes([0x45, 0, total >> 8, total & 255]) + rb(4) + bytes([64, proto]) + \
                    rb(2) + rb(8)
                out.append(vx + eth + b"\x08\x00" + ip + l4)
            else:
                l4 = rb(12) + bytes([5 << 4, 0x18]) + rb(6) + payload
                ip = bytes([0x60, 0, 0, 0, len(l4) >> 8, len(l4) & 255, 6, 64]) + rb(32)
                out.append(vx + eth + b"\x86\xdd" + ip + l4)
        else:
            out.append(vx + eth + b"\x08\x06" + bytes([0, 1, 8, 0, 6, 4]) + rb(2) + rb(20))
    return out

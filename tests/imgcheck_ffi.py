"""ctypes binding of the test-only image harness (tests/native/imgcheck.hip).

It walks the compiled table images on the host with the kernels' own probe
functions, so the compilers are checked against the oracle on CPU.
"""
import ctypes as C
import os
import subprocess

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
LIB = os.path.join(HERE, "native", "build", "libvc_imgcheck.so")
_lib = None


def lib():
    global _lib
    if _lib is None:
        subprocess.check_call(["make", "-s", "-C", os.path.join(HERE, "native")])
        L = C.CDLL(LIB)
        vp = C.c_void_p
        L.ic_acl.argtypes = [vp, C.c_int, vp, C.c_int, C.c_int, C.c_int, vp, vp, vp, C.c_int64, vp,
                             vp, vp]
        L.ic_acl_port.argtypes = [vp, C.c_int, C.c_uint32, vp, C.c_int64, vp]
        L.ic_route.argtypes = [vp, C.c_int, C.c_int, vp, C.c_int64, vp, vp, C.c_int]
        L.ic_hint.argtypes = [vp, C.c_int, vp, vp, vp, vp, vp, vp, vp, C.c_int64, vp]
        L.ic_hint_deferred.restype = C.c_int64
        L.ic_dns.argtypes = [vp, vp, vp, C.c_int, vp, C.c_int, vp, vp, C.c_int64, vp, vp]
        L.ic_certs.argtypes = [vp, vp, vp, C.c_int, C.c_int, vp, vp, vp, C.c_int64, vp]
        L.ic_mirror.argtypes = [vp, C.c_int, C.c_int32, vp, C.c_int64, vp]
        L.ic_mirror_switch.argtypes = [vp, C.c_int, C.c_int32, vp, vp, C.c_int64, C.c_int, vp]
        L.ic_mirror_sw.argtypes = [vp, C.c_int, C.c_int32, vp, C.c_int64, vp]
        L.ic_mirror_switch_sw.argtypes = [vp, C.c_int, C.c_int32, vp, vp, C.c_int64, C.c_int, vp,
                                          vp]
        L.ic_net_match.argtypes = [C.c_char_p, C.c_int, C.c_char_p, C.c_int, C.c_char_p, C.c_int]
        L.ic_packets.argtypes = [vp, vp, C.c_int64, C.c_int, vp, vp]
        L.ic_is_ipv6.argtypes = [C.c_char_p, C.c_int]
        L.ic_is_ip_literal.argtypes = [C.c_char_p, C.c_int]
        _lib = L
    return _lib


def P(a):
    if a is None:
        return None
    if isinstance(a, np.ndarray):
        return C.c_void_p(a.ctypes.data)
    return C.cast(a, C.c_void_p)


def acl(tcp, udp, dflt, family, proto, src, port):
    n = len(port)
    out = np.empty(n, np.int32)
    allow = np.empty(n, np.uint8)
    stats = np.zeros(10, np.int32)    # [list][family] nb, np; then v6 lookups on v4-only lists
    rc = lib().ic_acl(P(tcp), len(tcp), P(udp), len(udp), 1 if dflt else 0, family, P(proto),
                      P(src), P(port), n, P(out), P(allow), P(stats))
    assert rc == 0, rc
    return out, allow, stats


def acl_port(udp, port, keys):
    """the UDP list's IPv4 image at `port` (build_acl_port) against the
    general image at every interval edge and at `keys` -> (rule index per
    key, -1 = none; port table size)"""
    keys = np.ascontiguousarray(keys, np.uint32)
    out = np.empty(len(keys), np.int32)
    rc = lib().ic_acl_port(P(udp), len(udp), port, P(keys), len(keys), P(out))
    assert rc > 0, rc
    return out, rc


def route(rules, family, keys, root_bits=0):
    """root_bits 0: the library's default for the table size"""
    n = len(keys)
    out = np.empty(n, np.int32)
    # root bits, node units, one-prefix records, IPv6 keys the wide root
    # answers in one load (every IPv6 key is also checked through it: rc -201)
    stats = np.zeros(4, np.int32)
    rc = lib().ic_route(P(rules), len(rules), family, P(keys), n, P(out), P(stats), root_bits)
    assert rc == 0, rc
    return out, stats


def hint(group_arr, ng, hosts, ports, uris):
    hb, ho, hn = hosts
    n = len(ho) - 1
    ub = uo = un = None
    if uris is not None:
        ub, uo, un = uris
    out = np.empty(n, np.int32)
    rc = lib().ic_hint(P(group_arr), ng, P(hb), P(ho), P(hn), P(ports), P(ub), P(uo), P(un), n,
                       P(out))
    assert rc == 0, rc
    return out


def hint_deferred():
    """names of the last hint() call the deferring fast path left to the
    follow-up kernel (hint_defer_kernel)"""
    return int(lib().ic_hint_deferred())


def is_ipv6(s):
    b = s.encode() if isinstance(s, str) else s
    return bool(lib().ic_is_ipv6(b, len(b)))


def is_ip_literal(s):
    b = s.encode() if isinstance(s, str) else s
    return bool(lib().ic_is_ip_literal(b, len(b)))


def dns(pairs, group_arr, ng, qblob, qoff):
    keys = [k.encode() if isinstance(k, str) else k for k, _ in pairs]
    karr = (C.c_char_p * max(1, len(keys)))(*keys)
    kl = np.array([len(k) for k in keys] or [0], np.int32)
    kv = np.array([v for _, v in pairs] or [0], np.int32)
    n = len(qoff) - 1
    kind = np.empty(n, np.uint8)
    val = np.empty(n, np.int32)
    rc = lib().ic_dns(karr, P(kl), P(kv), len(keys), P(group_arr), ng, P(qblob), P(qoff), n,
                      P(kind), P(val))
    assert rc == 0, rc
    return kind, val


def packets(frames, layer):
    """the device parse_packet run on the host: list of dicts like
    oracle_ffi.parse_packet"""
    lens = np.array([len(f) for f in frames], np.int64)
    off = np.zeros(len(frames) + 1, np.uint32)
    off[1:] = np.cumsum(lens)
    blob = np.frombuffer(b"".join(frames) or b"\0", np.uint8).copy()
    n = len(frames)
    f = np.zeros((n, 8), np.int32)
    a = np.zeros((n, 32), np.uint8)
    assert lib().ic_packets(P(blob), P(off), n, layer, P(f), P(a)) == 0
    out = []
    for i in range(n):
        w = 16 if f[i, 1] == 6 else 4
        out.append({"status": int(f[i, 0]), "l3": int(f[i, 1]), "l4": int(f[i, 2]),
                    "proto": int(f[i, 3]), "vni": int(np.uint32(f[i, 4])),
                    "ether_type": int(f[i, 5]), "sport": int(f[i, 6]), "dport": int(f[i, 7]),
                    "src": bytes(a[i, :w]).hex(), "dst": bytes(a[i, 16:16 + w]).hex()})
    return out


def certs(holders, snis):
    """the device cert_one over a host-built certificate table; snis: list of
    bytes/str/None"""
    names = [s.encode() if isinstance(s, str) else s for hs in holders for s in hs]
    hold = np.array([h for h, hs in enumerate(holders) for _ in hs] or [0], np.int32)
    karr = (C.c_char_p * max(1, len(names)))(*names)
    kl = np.array([len(k) for k in names] or [0], np.int32)
    qs = [b"" if q is None else (q.encode() if isinstance(q, str) else q) for q in snis]
    qnull = np.array([q is None for q in snis] or [0], np.uint8)
    lens = np.array([len(q) for q in qs], np.int64)
    qoff = np.zeros(len(qs) + 1, np.uint32)
    qoff[1:] = np.cumsum(lens)
    qb = np.frombuffer(b"".join(qs) or b"\0", np.uint8).copy()
    out = np.empty(len(qs), np.int32)
    rc = lib().ic_certs(karr, P(kl), P(hold), len(names), len(holders), P(qb), P(qoff), P(qnull),
                        len(qs), P(out))
    assert rc == 0, rc
    return out


def mirror(filter_arr, nf, origin, items, n):
    """device mirror_item + mirror_eval on the host; items: VcMirrorItems"""
    out = np.empty(n, np.uint64)
    rc = lib().ic_mirror(C.cast(filter_arr, C.c_void_p), nf, origin, C.cast(C.pointer(items),
                         C.c_void_p), n, P(out))
    assert rc == 0, rc
    return out


def mirror_sw(filter_arr, nf, origin, items, n):
    """Mirror.mirror through the origin's bit-set image on the host; None
    when the origin has no such image"""
    out = np.empty(n, np.uint64)
    rc = lib().ic_mirror_sw(C.cast(filter_arr, C.c_void_p), nf, origin,
                            C.cast(C.pointer(items), C.c_void_p), n, P(out))
    assert rc in (0, 1), rc
    return None if rc == 1 else out


def mirror_switch(filter_arr, nf, origin, frames, layer):
    lens = np.array([len(f) for f in frames], np.int64)
    off = np.zeros(len(frames) + 1, np.uint32)
    off[1:] = np.cumsum(lens)
    blob = np.frombuffer(b"".join(frames) or b"\0", np.uint8).copy()
    out = np.empty(len(frames), np.uint64)
    rc = lib().ic_mirror_switch(C.cast(filter_arr, C.c_void_p), nf, origin, P(blob), P(off),
                                len(frames), layer, P(out))
    assert rc == 0, rc
    return out


def mirror_switch_sw(filter_arr, nf, origin, frames, layer):
    """switchPacket through the origin's bit-set image on the host ->
    (results, (nb4, nb6)), or None when the origin has no such image."""
    lens = np.array([len(f) for f in frames], np.int64)
    off = np.zeros(len(frames) + 1, np.uint32)
    off[1:] = np.cumsum(lens)
    blob = np.frombuffer(b"".join(frames) or b"\0", np.uint8).copy()
    out = np.empty(len(frames), np.uint64)
    nb = np.zeros(2, np.int32)
    rc = lib().ic_mirror_switch_sw(C.cast(filter_arr, C.c_void_p), nf, origin, P(blob), P(off),
                                   len(frames), layer, P(out), P(nb))
    assert rc in (0, 1), rc
    return None if rc == 1 else (out, tuple(int(x) for x in nb))

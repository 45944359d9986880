"""ctypes bindings for the CPU oracle (oracle/vc_oracle.c).

Test infrastructure only: the oracle is the parity checker.  Product code in
vproxy_amd/ never imports this module.
"""
import ctypes as C
import os
import subprocess

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LIB_PATH = os.path.join(ROOT, "oracle", "build", "libvc_oracle.so")

_lib = None


class VoNet(C.Structure):
    _fields_ = [("ip", C.c_uint8 * 16), ("mask", C.c_uint8 * 16),
                ("ip_len", C.c_int32), ("mask_len", C.c_int32)]


class VoSgRule(C.Structure):
    _fields_ = [("net", VoNet), ("min_port", C.c_int32), ("max_port", C.c_int32),
                ("allow", C.c_int32)]


class VoAnnos(C.Structure):
    _fields_ = [("host", C.c_char_p), ("host_len", C.c_int32), ("port", C.c_int32),
                ("uri", C.c_char_p), ("uri_len", C.c_int32)]


class VoGroup(C.Structure):
    _fields_ = [("handle", VoAnnos), ("group", VoAnnos)]


class VoHint(C.Structure):
    _fields_ = [("host", C.c_void_p), ("host_len", C.c_int32), ("port", C.c_int32),
                ("uri", C.c_void_p), ("uri_len", C.c_int32)]


class VoRouteTable(C.Structure):
    _fields_ = [("v4", C.POINTER(VoNet)), ("n4", C.c_int), ("cap4", C.c_int),
                ("v6", C.POINTER(VoNet)), ("n6", C.c_int), ("cap6", C.c_int)]


class VoServer(C.Structure):
    _fields_ = [("ip", C.c_uint8 * 16), ("ip_len", C.c_int32), ("port", C.c_int32),
                ("weight", C.c_int32), ("healthy", C.c_int32)]


class VoPkt(C.Structure):
    _fields_ = [("status", C.c_int), ("l3", C.c_int), ("l4", C.c_int), ("proto", C.c_int),
                ("vni", C.c_uint32), ("ether_type", C.c_int), ("src", C.c_uint8 * 16),
                ("dst", C.c_uint8 * 16), ("sport", C.c_int), ("dport", C.c_int)]


class VoMirrorFilter(C.Structure):
    _fields_ = [("origin", C.c_int32), ("mirror", C.c_int32), ("has_mac_x", C.c_int32),
                ("has_mac_y", C.c_int32), ("mac_x", C.c_uint8 * 6), ("mac_y", C.c_uint8 * 6),
                ("has_net_x", C.c_int32), ("has_net_y", C.c_int32), ("net_x", VoNet),
                ("net_y", VoNet), ("transport", C.c_int32), ("has_port_x", C.c_int32),
                ("has_port_y", C.c_int32), ("port_x", C.c_int32 * 2), ("port_y", C.c_int32 * 2),
                ("app", C.c_int32)]


class VoHosts(C.Structure):
    _fields_ = [("keys", C.POINTER(C.c_char_p)), ("key_lens", C.POINTER(C.c_int32)),
                ("values", C.POINTER(C.c_int32)), ("n", C.c_int)]


class VoDnsdOut(C.Structure):
    _fields_ = [("status", C.c_int32), ("acl", C.c_int32), ("nq", C.c_int32),
                ("qtype", C.c_int32 * 4), ("kind", C.c_int32 * 4), ("value", C.c_int32 * 4)]


def lib():
    global _lib
    if _lib is None:
        src = os.path.join(ROOT, "oracle", "vc_oracle.c")
        if (not os.path.exists(LIB_PATH) or
                os.path.getmtime(LIB_PATH) < os.path.getmtime(src)):
            subprocess.check_call(["make", "-s", "-C", os.path.join(ROOT, "oracle")])
        L = C.CDLL(LIB_PATH)
        P = C.POINTER
        u8p, i32p = P(C.c_uint8), P(C.c_int32)
        L.vo_parse_ipv4.argtypes = [C.c_char_p, C.c_int, u8p]
        L.vo_parse_ipv6.argtypes = [C.c_char_p, C.c_int, u8p]
        L.vo_parse_ip.argtypes = [C.c_char_p, C.c_int, u8p]
        L.vo_is_ipv6.argtypes = [C.c_char_p, C.c_int]
        L.vo_is_ip_literal.argtypes = [C.c_char_p, C.c_int]
        L.vo_parse_mask.argtypes = [C.c_int, u8p]
        L.vo_mask_int.argtypes = [u8p, C.c_int]
        L.vo_valid_network.argtypes = [u8p, C.c_int, u8p, C.c_int]
        L.vo_mask_match.argtypes = [u8p, C.c_int, u8p, C.c_int, u8p, C.c_int]
        L.vo_net_from_str.argtypes = [C.c_char_p, C.c_int, P(VoNet)]
        L.vo_net_contains_ip.argtypes = [P(VoNet), u8p, C.c_int]
        L.vo_net_contains_net.argtypes = [P(VoNet), P(VoNet)]
        L.vo_sg_allow.argtypes = [P(VoSgRule), C.c_int, P(VoSgRule), C.c_int, C.c_int, C.c_int,
                                  u8p, C.c_int, C.c_int, P(C.c_int)]
        L.vo_sg_allow_batch_v4.argtypes = [P(VoSgRule), C.c_int, P(VoSgRule), C.c_int, C.c_int,
                                           C.c_void_p, C.c_void_p, C.c_void_p, C.c_int64,
                                           C.c_void_p, C.c_void_p, C.c_int]
        L.vo_sg_allow_batch_v6.argtypes = L.vo_sg_allow_batch_v4.argtypes
        L.vo_rt_init.argtypes = [P(VoRouteTable)]
        L.vo_rt_free.argtypes = [P(VoRouteTable)]
        L.vo_rt_add.argtypes = [P(VoRouteTable), P(VoNet)]
        L.vo_rt_lookup.argtypes = [P(VoRouteTable), u8p, C.c_int]
        L.vo_rt_lookup_list.argtypes = [P(VoNet), C.c_int, u8p, C.c_int]
        L.vo_rt_lookup_batch_v4.argtypes = [P(VoNet), C.c_int, C.c_void_p, C.c_int64,
                                            C.c_void_p, C.c_int]
        L.vo_rt_lookup_batch_v6.argtypes = L.vo_rt_lookup_batch_v4.argtypes
        L.vo_hint_of.argtypes = [C.c_void_p, C.c_int, C.c_int, C.c_void_p, C.c_int]
        L.vo_hint_of.restype = VoHint
        L.vo_match_level.argtypes = [P(VoHint), P(VoAnnos), C.c_int]
        L.vo_search_for_group.argtypes = [P(VoGroup), C.c_int, P(VoHint)]
        L.vo_hint_batch.argtypes = [P(VoGroup), C.c_int, C.c_void_p, C.c_void_p, C.c_void_p,
                                    C.c_int64, C.c_void_p, C.c_int]
        L.vo_hint_uri_batch.argtypes = [P(VoGroup), C.c_int] + [C.c_void_p] * 6 + \
            [C.c_int64, C.c_void_p, C.c_int]
        L.vo_dns_classify.argtypes = [P(VoHosts), P(VoGroup), C.c_int, C.c_char_p, C.c_int,
                                      P(C.c_int32)]
        L.vo_hosts_parse.argtypes = [C.c_char_p, C.c_int, C.c_char_p, C.c_int, i32p, i32p, i32p,
                                     C.c_int, u8p, i32p, C.c_int]
        L.vo_parse_packet.argtypes = [u8p, C.c_int, C.c_int, P(VoPkt)]
        L.vo_source_hash.argtypes = [u8p, C.c_int]
        L.vo_source_hash.restype = C.c_int32
        L.vo_source_list.argtypes = [P(VoServer), C.c_int, C.c_int, i32p]
        L.vo_source_select.argtypes = [P(VoServer), C.c_int, C.c_int, u8p, C.c_int]
        L.vo_mirror_match.argtypes = [P(VoMirrorFilter), C.c_int, C.c_int, u8p, u8p, u8p, C.c_int,
                                      u8p, C.c_int, C.c_int, C.c_int, C.c_int, C.c_int]
        L.vo_mirror_match.restype = C.c_uint64
        L.vo_mirror_switch.argtypes = [P(VoMirrorFilter), C.c_int, C.c_int, u8p, C.c_int, C.c_int]
        L.vo_mirror_switch.restype = C.c_uint64
        L.vo_cert_choose.argtypes = [P(C.c_char_p), i32p, i32p, C.c_int, C.c_int, u8p, C.c_int,
                                     C.c_int]
        vp, i64 = C.c_void_p, C.c_int64
        L.vo_dns_batch.argtypes = [P(VoHosts), P(VoGroup), C.c_int, vp, vp, i64, vp, vp, C.c_int]
        L.vo_http_extract.argtypes = [vp, C.c_int, vp, P(C.c_int), vp, P(C.c_int)]
        L.vo_http_hint.argtypes = [P(VoGroup), C.c_int, vp, C.c_int, P(C.c_int)]
        L.vo_http_batch.argtypes = [P(VoGroup), C.c_int, vp, vp, i64, vp, vp, C.c_int]
        L.vo_parse_batch.argtypes = [vp, vp, i64, C.c_int, P(VoPkt), C.c_int]
        L.vo_switch_batch.argtypes = [P(VoSgRule), C.c_int, P(VoSgRule), C.c_int, C.c_int, vp, vp,
                                      i64, vp, C.c_int, P(VoNet), C.c_int, P(VoNet), C.c_int, vp,
                                      vp, vp, C.c_int]
        L.vo_cert_batch.argtypes = [P(C.c_char_p), i32p, i32p, C.c_int, C.c_int, vp, vp, vp, i64,
                                    vp, C.c_int]
        L.vo_mirror_switch_batch.argtypes = [P(VoMirrorFilter), C.c_int, C.c_int, vp, vp, i64,
                                             C.c_int, vp, C.c_int]
        L.vo_mirror_match_batch.argtypes = [P(VoMirrorFilter), C.c_int, C.c_int] + [vp] * 10 + \
            [i64, vp, C.c_int]
        L.vo_source_batch.argtypes = [P(VoServer), vp, C.c_int, C.c_int, vp, vp, i64, vp, C.c_int]
        L.vo_dns_datagram.argtypes = [P(VoSgRule), C.c_int, P(VoSgRule), C.c_int, C.c_int,
                                      P(VoHosts), P(VoGroup), C.c_int, vp, C.c_int, vp, C.c_int,
                                      C.c_int, P(VoDnsdOut)]
        L.vo_dnsd_batch.argtypes = [P(VoSgRule), C.c_int, P(VoSgRule), C.c_int, C.c_int,
                                    P(VoHosts), P(VoGroup), C.c_int, vp, vp, i64, vp, vp, vp, vp,
                                    P(VoDnsdOut), C.c_int]
        _lib = L
    return _lib


def _b(s):
    return s.encode() if isinstance(s, str) else s


def parse_ip(s):
    b = (C.c_uint8 * 16)()
    s = _b(s)
    n = lib().vo_parse_ip(s, len(s), b)
    return None if n < 0 else bytes(b[:n])


def parse_ipv4(s):
    b = (C.c_uint8 * 16)()
    s = _b(s)
    n = lib().vo_parse_ipv4(s, len(s), b)
    return None if n < 0 else bytes(b[:n])


def parse_ipv6(s):
    b = (C.c_uint8 * 16)()
    s = _b(s)
    n = lib().vo_parse_ipv6(s, len(s), b)
    return None if n < 0 else bytes(b[:n])


def is_ip_literal(s):
    s = _b(s)
    return bool(lib().vo_is_ip_literal(s, len(s)))


def parse_mask(m):
    b = (C.c_uint8 * 16)()
    n = lib().vo_parse_mask(m, b)
    if n < 0:
        raise ValueError("unknown mask %d" % m)
    return bytes(b[:n])


def _u8(b):
    return (C.c_uint8 * max(1, len(b))).from_buffer_copy(b if b else b"\0")


def valid_network(addr, mask):
    return bool(lib().vo_valid_network(_u8(addr), len(addr), _u8(mask), len(mask)))


def mask_match(inp, rule, mask):
    return bool(lib().vo_mask_match(_u8(inp), len(inp), _u8(rule), len(rule), _u8(mask), len(mask)))


def net(s):
    n = VoNet()
    s = _b(s)
    if lib().vo_net_from_str(s, len(s), C.byref(n)) != 0:
        raise ValueError("invalid network %r" % s)
    return n


def net_str(n):
    """Network.toString (Network.java:66-69) -- canonical text for comparisons."""
    ip = bytes(n.ip[:n.ip_len])
    mi = lib().vo_mask_int((C.c_uint8 * 16)(*n.mask), n.mask_len)
    if n.ip_len == 4:
        s = ".".join(str(x) for x in ip)
    else:
        import ipaddress
        s = str(ipaddress.IPv6Address(ip))
    return "%s/%d" % (s, mi)


def sg_rule(netstr, min_port, max_port, allow):
    r = VoSgRule()
    r.net = net(netstr)
    r.min_port, r.max_port, r.allow = min_port, max_port, 1 if allow else 0
    return r


def sg_rule_arr(rules):
    arr = (VoSgRule * max(1, len(rules)))()
    for i, r in enumerate(rules):
        arr[i] = r
    return arr


def sg_allow(tcp, udp, default_allow, proto, ip_bytes, port):
    v = C.c_int()
    idx = lib().vo_sg_allow(sg_rule_arr(tcp), len(tcp), sg_rule_arr(udp), len(udp),
                            1 if default_allow else 0, proto, _u8(ip_bytes), len(ip_bytes), port,
                            C.byref(v))
    return idx, bool(v.value)


def _ptr(a):
    # data_as keeps a reference to the array in the pointer, so a converted
    # temporary (e.g. _ptr(np.ascontiguousarray(x, np.uint32))) lives until
    # the C call that takes the pointer returns
    return a.ctypes.data_as(C.c_void_p) if a is not None else None


def sg_allow_batch_v4(tcp, udp, default_allow, proto, src4, port, nthreads=1):
    n = len(src4)
    out = np.empty(n, np.int32)
    ver = np.empty(n, np.uint8)
    ta, ua = sg_rule_arr(tcp), sg_rule_arr(udp)
    lib().vo_sg_allow_batch_v4(ta, len(tcp), ua, len(udp), 1 if default_allow else 0,
                               _ptr(proto), _ptr(src4), _ptr(port), n, _ptr(out), _ptr(ver),
                               nthreads)
    return out, ver


def sg_allow_batch_v6(tcp, udp, default_allow, proto, src6, port, nthreads=1):
    n = len(port)
    out = np.empty(n, np.int32)
    ver = np.empty(n, np.uint8)
    ta, ua = sg_rule_arr(tcp), sg_rule_arr(udp)
    lib().vo_sg_allow_batch_v6(ta, len(tcp), ua, len(udp), 1 if default_allow else 0,
                               _ptr(proto), _ptr(src6), _ptr(port), n, _ptr(out), _ptr(ver),
                               nthreads)
    return out, ver


class RouteTable:
    """Oracle RouteTable: RouteTable.addRule ordering + linear lookup."""

    def __init__(self):
        self.t = VoRouteTable()
        lib().vo_rt_init(C.byref(self.t))

    def __del__(self):
        try:
            lib().vo_rt_free(C.byref(self.t))
        except Exception:
            pass

    def add(self, netstr):
        n = net(netstr) if isinstance(netstr, (str, bytes)) else netstr
        return lib().vo_rt_add(C.byref(self.t), C.byref(n)) == 0

    def rules(self):
        return ([net_str(self.t.v4[i]) for i in range(self.t.n4)] +
                [net_str(self.t.v6[i]) for i in range(self.t.n6)])

    def lookup(self, ip_bytes):
        return lib().vo_rt_lookup(C.byref(self.t), _u8(ip_bytes), len(ip_bytes))


def net_list(nets):
    arr = (VoNet * max(1, len(nets)))()
    for i, n in enumerate(nets):
        arr[i] = n
    return arr


def rt_lookup_batch_v4(v4_nets_arr, n4, dst4, nthreads=1):
    out = np.empty(len(dst4), np.int32)
    lib().vo_rt_lookup_batch_v4(v4_nets_arr, n4, _ptr(dst4), len(dst4), _ptr(out), nthreads)
    return out


def rt_lookup_batch_v6(v6_nets_arr, n6, dst6, nthreads=1):
    n = dst6.shape[0]
    out = np.empty(n, np.int32)
    lib().vo_rt_lookup_batch_v6(v6_nets_arr, n6, _ptr(dst6), n, _ptr(out), nthreads)
    return out


def parse_java_int(s):
    """Integer.parseInt with Annotations' failure -> 0 (Annotations.java:45-58)."""
    if isinstance(s, int):
        return s
    try:
        if s is None or not s or s.strip() != s:
            raise ValueError
        v = int(s, 10)
        if v < -2**31 or v > 2**31 - 1 or "_" in s:
            raise ValueError
        return v
    except ValueError:
        return 0


class Groups:
    """Keeps the byte buffers alive for a vo_group array."""

    def __init__(self, groups):
        self.keep = []
        self.arr = (VoGroup * max(1, len(groups)))()
        self.n = len(groups)
        for i, (ha, ga) in enumerate(groups):
            self.arr[i].handle = self._annos(ha)
            self.arr[i].group = self._annos(ga)

    def _annos(self, a):
        x = VoAnnos()
        h, u = a.get("host"), a.get("uri")
        if h is not None:
            hb = _b(h)
            self.keep.append(hb)
            x.host, x.host_len = hb, len(hb)
        x.port = parse_java_int(a.get("port", 0))
        if u is not None:
            ub = _b(u)
            self.keep.append(ub)
            x.uri, x.uri_len = ub, len(ub)
        return x


def hint_of(host=None, port=0, uri=None):
    hb = _b(host) if host is not None else None
    ub = _b(uri) if uri is not None else None
    hbuf = C.create_string_buffer(hb, len(hb)) if hb is not None else None
    ubuf = C.create_string_buffer(ub, len(ub)) if ub is not None else None
    h = lib().vo_hint_of(C.cast(hbuf, C.c_void_p) if hbuf is not None else None,
                         len(hb) if hb is not None else 0, port,
                         C.cast(ubuf, C.c_void_p) if ubuf is not None else None,
                         len(ub) if ub is not None else 0)
    return h, (hbuf, ubuf)


def search_for_group(groups, host=None, port=0, uri=None):
    g = groups if isinstance(groups, Groups) else Groups(groups)
    h, keep = hint_of(host, port, uri)
    return lib().vo_search_for_group(g.arr, g.n, C.byref(h))


class Hosts:
    def __init__(self, pairs):
        self.keys = [_b(k) for k, _ in pairs]
        n = len(pairs)
        self.karr = (C.c_char_p * max(1, n))(*self.keys)
        self.larr = (C.c_int32 * max(1, n))(*[len(k) for k in self.keys])
        self.varr = (C.c_int32 * max(1, n))(*[v for _, v in pairs])
        self.h = VoHosts(self.karr, self.larr, self.varr, n)


def dns_classify(hosts, groups, qname):
    g = groups if isinstance(groups, Groups) else Groups(groups)
    h = hosts if isinstance(hosts, Hosts) else Hosts(hosts)
    q = _b(qname)
    v = C.c_int32()
    kind = lib().vo_dns_classify(C.byref(h.h), g.arr, g.n, q, len(q), C.byref(v))
    return kind, v.value


def hosts_parse(text):
    t = _b(text)
    cap = 4 * len(t) + 16
    keybuf = C.create_string_buffer(cap * 2)
    ko = (C.c_int32 * cap)()
    kl = (C.c_int32 * cap)()
    kv = (C.c_int32 * cap)()
    lip = (C.c_uint8 * (16 * cap))()
    lil = (C.c_int32 * cap)()
    n = lib().vo_hosts_parse(t, len(t), keybuf, cap * 2, ko, kl, kv, cap, lip, lil, cap)
    assert n >= 0
    raw = keybuf.raw
    pairs = [(raw[ko[i]:ko[i] + kl[i]].decode(), kv[i]) for i in range(n)]
    nlines = (max(kv[i] for i in range(n)) + 1) if n else 0
    ips = [bytes(lip[16 * j:16 * j + lil[j]]) for j in range(nlines)]
    return pairs, ips


# ---- numpy-layout helpers (vo_net / vo_sg_rule == workloads.NET_DT / RULE_DT) ----
def _cast(arr, T):
    return C.cast(C.c_void_p(arr.ctypes.data), C.POINTER(T))


def sg_batch_v4_np(tcp, udp, dflt, proto, src4, port, nthreads=1):
    n = len(src4)
    out = np.empty(n, np.int32)
    ver = np.empty(n, np.uint8)
    t = tcp if len(tcp) else np.zeros(1, tcp.dtype)
    u = udp if len(udp) else np.zeros(1, udp.dtype)
    lib().vo_sg_allow_batch_v4(_cast(t, VoSgRule), len(tcp), _cast(u, VoSgRule), len(udp),
                               1 if dflt else 0, _ptr(np.ascontiguousarray(proto, np.uint8)),
                               _ptr(np.ascontiguousarray(src4, np.uint32)),
                               _ptr(np.ascontiguousarray(port, np.uint16)), n, _ptr(out),
                               _ptr(ver), nthreads)
    return out, ver


def sg_batch_v6_np(tcp, udp, dflt, proto, src6, port, nthreads=1):
    n = len(port)
    out = np.empty(n, np.int32)
    ver = np.empty(n, np.uint8)
    t = tcp if len(tcp) else np.zeros(1, tcp.dtype)
    u = udp if len(udp) else np.zeros(1, udp.dtype)
    lib().vo_sg_allow_batch_v6(_cast(t, VoSgRule), len(tcp), _cast(u, VoSgRule), len(udp),
                               1 if dflt else 0, _ptr(np.ascontiguousarray(proto, np.uint8)),
                               _ptr(np.ascontiguousarray(src6, np.uint8)),
                               _ptr(np.ascontiguousarray(port, np.uint16)), n, _ptr(out),
                               _ptr(ver), nthreads)
    return out, ver


def rt_batch_v4_np(nets, dst4, nthreads=1):
    a = nets if len(nets) else np.zeros(1, nets.dtype)
    out = np.empty(len(dst4), np.int32)
    lib().vo_rt_lookup_batch_v4(_cast(a, VoNet), len(nets),
                                _ptr(np.ascontiguousarray(dst4, np.uint32)), len(dst4), _ptr(out),
                                nthreads)
    return out


def rt_batch_v6_np(nets, dst6, nthreads=1):
    a = nets if len(nets) else np.zeros(1, nets.dtype)
    out = np.empty(len(dst6), np.int32)
    lib().vo_rt_lookup_batch_v6(_cast(a, VoNet), len(nets),
                                _ptr(np.ascontiguousarray(dst6, np.uint8)), len(dst6), _ptr(out),
                                nthreads)
    return out


def rt_table_np(table):
    """oracle RouteTable lists -> (v4 NET array, v6 NET array) numpy views (copies)."""
    from vproxy_amd.workloads import NET_DT
    t = table.t
    v4 = np.ctypeslib.as_array(C.cast(t.v4, C.POINTER(C.c_uint8)), (t.n4 * 40,)).copy() \
        if t.n4 else np.zeros(0, np.uint8)
    v6 = np.ctypeslib.as_array(C.cast(t.v6, C.POINTER(C.c_uint8)), (t.n6 * 40,)).copy() \
        if t.n6 else np.zeros(0, np.uint8)
    return v4.view(NET_DT), v6.view(NET_DT)


def rt_add_np(table, nets):
    """add NET_DT rows in order through RouteTable.addRule's heuristic."""
    for i in range(len(nets)):
        n = VoNet.from_buffer_copy(nets[i].tobytes())
        lib().vo_rt_add(C.byref(table.t), C.byref(n))


def hint_batch_np(groups, blob, off, port, nthreads=1):
    g = groups if isinstance(groups, Groups) else Groups(groups)
    n = len(off) - 1
    out = np.empty(n, np.int32)
    lib().vo_hint_batch(g.arr, g.n, _ptr(np.ascontiguousarray(blob, np.uint8)),
                        _ptr(np.ascontiguousarray(off, np.uint32)),
                        _ptr(np.ascontiguousarray(port, np.uint16)) if port is not None else None,
                        n, _ptr(out), nthreads)
    return out


def hint_uri_batch_np(groups, hblob, hoff, ublob, uoff, unull=None, port=None, nthreads=1):
    """searchForGroup(Hint.ofHostPortUri(host, port, uri)) per item (vo_hint_uri_batch)."""
    g = groups if isinstance(groups, Groups) else Groups(groups)
    n = len(hoff) - 1
    out = np.empty(n, np.int32)
    keep = [np.ascontiguousarray(hblob, np.uint8), np.ascontiguousarray(hoff, np.uint32),
            np.ascontiguousarray(ublob, np.uint8), np.ascontiguousarray(uoff, np.uint32),
            None if unull is None else np.ascontiguousarray(unull, np.uint8),
            None if port is None else np.ascontiguousarray(port, np.uint16)]
    lib().vo_hint_uri_batch(g.arr, g.n, *[_ptr(k) if k is not None else None for k in keep],
                            n, _ptr(out), nthreads)
    return out


# ---- ServerGroup source hashing (ServerGroup.java:377-490) ----
def servers_arr(servers):
    """[(ip bytes, port, weight, healthy)] -> VoServer array"""
    arr = (VoServer * max(1, len(servers)))()
    for i, (ip, port, w, h) in enumerate(servers):
        arr[i].ip[:len(ip)] = list(ip)
        arr[i].ip_len = len(ip)
        arr[i].port = port
        arr[i].weight = w
        arr[i].healthy = 1 if h else 0
    return arr


def source_hash(b):
    return lib().vo_source_hash(_u8(bytes(b)), len(b))


def source_list(servers, view):
    arr = servers_arr(servers)
    order = (C.c_int32 * max(1, len(servers)))()
    k = lib().vo_source_list(arr, len(servers), view, order)
    return list(order[:k])


def source_select(servers, view, src):
    arr = servers_arr(servers)
    return lib().vo_source_select(arr, len(servers), view, _u8(bytes(src)), len(src))


# ---- packet header extraction (base/src/main/java/vpacket) ----
def parse_packet(b, layer):
    """-> dict of the oracle's fields (src/dst as hex of 4 or 16 bytes)"""
    o = VoPkt()
    lib().vo_parse_packet(_u8(bytes(b)), len(b), layer, C.byref(o))
    n = 16 if o.l3 == 6 else 4
    return {"status": o.status, "l3": o.l3, "l4": o.l4, "proto": o.proto, "vni": o.vni,
            "ether_type": o.ether_type, "src": bytes(o.src[:n]).hex(),
            "dst": bytes(o.dst[:n]).hex(), "sport": o.sport, "dport": o.dport}


# ---- SSLContextHolder.choose (SSLContextHolder.java:51-186) ----
class Certs:
    """holders: list (add() order) of name lists (CN + SAN dNSNames)."""

    def __init__(self, holders):
        self.n_holders = len(holders)
        self.names = [_b(s) for hs in holders for s in hs]
        hold = [h for h, hs in enumerate(holders) for _ in hs]
        n = len(self.names)
        self.karr = (C.c_char_p * max(1, n))(*self.names)
        self.larr = (C.c_int32 * max(1, n))(*[len(k) for k in self.names])
        self.harr = (C.c_int32 * max(1, n))(*hold)

    def choose(self, sni):
        if sni is None:
            return lib().vo_cert_choose(self.karr, self.larr, self.harr, len(self.names),
                                        self.n_holders, _u8(b""), 0, 1)
        s = _b(sni)
        return lib().vo_cert_choose(self.karr, self.larr, self.harr, len(self.names),
                                    self.n_holders, _u8(s), len(s), 0)


# ---- traffic-mirror filters (vmirror/FilterConfig.java, Mirror.java) ----
def mirror_filters(filters, ids):
    """dict configs -> VoMirrorFilter array, parsed as Mirror.parseAndLoadFilter
    (Mirror.java:545-601) with the oracle's own Network parser; strings
    interned through `ids` (dict, extended in place)."""
    def iid(s):
        if s is None:
            return -1
        return ids.setdefault(s, len(ids))

    def mac(s):
        return [int(p, 16) & 0xFF for p in s.split(":")]

    arr = (VoMirrorFilter * max(1, len(filters)))()
    for i, f in enumerate(filters):
        r = arr[i]
        r.origin, r.mirror = iid(f["origin"]), int(f["mirror"])
        if "mac" in f:
            r.has_mac_x, r.mac_x[:] = 1, mac(f["mac"])
            if "mac2" in f:
                r.has_mac_y, r.mac_y[:] = 1, mac(f["mac2"])
        if "network" in f:
            r.has_net_x, r.net_x = 1, net(f["network"])
            if "network2" in f:
                r.has_net_y, r.net_y = 1, net(f["network2"])
        r.transport = iid(f.get("transportLayerProtocol"))
        if "port" in f:
            r.has_port_x, r.port_x[:] = 1, list(f["port"])
            if "port2" in f:
                r.has_port_y, r.port_y[:] = 1, list(f["port2"])
        r.app = iid(f.get("applicationLayerProtocol"))
    return arr


def mirror_match(arr, n, origin, mac_src, mac_dst, ip_src, ip_dst, transport, port_src,
                 port_dst, app):
    s = bytes(ip_src or b"")
    d = bytes(ip_dst or b"")
    return int(lib().vo_mirror_match(arr, n, origin, _u8(bytes(mac_src)), _u8(bytes(mac_dst)),
                                     _u8(s), len(s), _u8(d), len(d), transport, port_src,
                                     port_dst, app))


def mirror_switch(arr, n, origin, frame, layer):
    return int(lib().vo_mirror_switch(arr, n, origin, _u8(bytes(frame)), len(frame), layer))


# ---- batched forms (pthread partitions): checkers and bench cpu_baseline ----
def _u32a(x):
    return np.ascontiguousarray(x, np.uint32)


def dns_batch_np(hosts, groups, blob, off, nthreads=1):
    g = groups if isinstance(groups, Groups) else Groups(groups)
    h = hosts if isinstance(hosts, Hosts) else Hosts(hosts)
    n = len(off) - 1
    kind, value = np.empty(n, np.uint8), np.empty(n, np.int32)
    lib().vo_dns_batch(C.byref(h.h), g.arr, g.n, _ptr(np.ascontiguousarray(blob, np.uint8)),
                       _ptr(_u32a(off)), n, _ptr(kind), _ptr(value), nthreads)
    return kind, value


def http_extract(head):
    """HttpSubContext's theUri / theHostHeader after feeding `head` (bytes):
    (uri or None, host or None), raw bytes (one per Java char)."""
    head = bytes(head)
    n = len(head)
    hb = C.create_string_buffer(head, max(1, n))
    ub, hob = C.create_string_buffer(max(1, n)), C.create_string_buffer(max(1, n))
    ul, hl = C.c_int(), C.c_int()
    k = lib().vo_http_extract(C.cast(hb, C.c_void_p), n, C.cast(ub, C.c_void_p), C.byref(ul),
                              C.cast(hob, C.c_void_p), C.byref(hl))
    return (ub.raw[:ul.value] if k & 1 else None), (hob.raw[:hl.value] if k & 2 else None)


def http_hint(groups, head):
    """-> (group, kind) of HttpContext.connectionHint + Upstream.searchForGroup"""
    g = groups if isinstance(groups, Groups) else Groups(groups)
    head = bytes(head)
    hb = C.create_string_buffer(head, max(1, len(head)))
    k = C.c_int()
    r = lib().vo_http_hint(g.arr, g.n, C.cast(hb, C.c_void_p), len(head), C.byref(k))
    return r, k.value


def http_batch_np(groups, blob, off, nthreads=1):
    g = groups if isinstance(groups, Groups) else Groups(groups)
    n = len(off) - 1
    kind, group = np.empty(n, np.uint8), np.empty(n, np.int32)
    lib().vo_http_batch(g.arr, g.n, _ptr(np.ascontiguousarray(blob, np.uint8)), _ptr(_u32a(off)),
                        n, _ptr(kind), _ptr(group), nthreads)
    return kind, group


def parse_batch_np(blob, off, layer, nthreads=1):
    """-> ctypes array of VoPkt, one per frame"""
    n = len(off) - 1
    out = (VoPkt * max(1, n))()
    lib().vo_parse_batch(_ptr(np.ascontiguousarray(blob, np.uint8)), _ptr(_u32a(off)), n, layer,
                         out, nthreads)
    return out


def switch_batch_np(tcp, udp, dflt, blob, off, remote4, bind_port, v4, v6, nthreads=1):
    n = len(off) - 1
    acl, allow, route = np.empty(n, np.int32), np.empty(n, np.uint8), np.empty(n, np.int32)
    t = tcp if len(tcp) else np.zeros(1, tcp.dtype)
    u = udp if len(udp) else np.zeros(1, udp.dtype)
    a4 = v4 if len(v4) else np.zeros(1, v4.dtype)
    a6 = v6 if len(v6) else np.zeros(1, v6.dtype)
    lib().vo_switch_batch(_cast(t, VoSgRule), len(tcp), _cast(u, VoSgRule), len(udp),
                          1 if dflt else 0, _ptr(np.ascontiguousarray(blob, np.uint8)),
                          _ptr(_u32a(off)), n, _ptr(_u32a(remote4)), bind_port,
                          _cast(a4, VoNet), len(v4), _cast(a6, VoNet), len(v6), _ptr(acl),
                          _ptr(allow), _ptr(route), nthreads)
    return acl, allow, route


def cert_batch_np(certs, blob, off, nthreads=1):
    n = len(off) - 1
    out = np.empty(n, np.int32)
    lib().vo_cert_batch(certs.karr, certs.larr, certs.harr, len(certs.names), certs.n_holders,
                        _ptr(np.ascontiguousarray(blob, np.uint8)), _ptr(_u32a(off)), None, n,
                        _ptr(out), nthreads)
    return out


def mirror_switch_batch_np(arr, nf, origin, blob, off, layer, nthreads=1):
    n = len(off) - 1
    out = np.empty(n, np.uint64)
    lib().vo_mirror_switch_batch(arr, nf, origin, _ptr(np.ascontiguousarray(blob, np.uint8)),
                                 _ptr(_u32a(off)), n, layer, _ptr(out), nthreads)
    return out


def mirror_match_batch_np(arr, nf, origin, cols, nthreads=1):
    """vo_mirror_match over vc_mirror_items-shaped numpy columns (every
    column present: mac_src / mac_dst 6 B per item, ip_*_len, ip_* 16 B rows,
    transport / port_src / port_dst / app int32)."""
    n = len(cols["ip_src_len"])
    c = {k: np.ascontiguousarray(v) for k, v in cols.items()}
    out = np.empty(n, np.uint64)
    lib().vo_mirror_match_batch(arr, nf, origin, _ptr(c["mac_src"]), _ptr(c["mac_dst"]),
                                _ptr(c["ip_src_len"]), _ptr(c["ip_dst_len"]), _ptr(c["ip_src"]),
                                _ptr(c["ip_dst"]), _ptr(c["transport"]), _ptr(c["port_src"]),
                                _ptr(c["port_dst"]), _ptr(c["app"]), n, _ptr(out), nthreads)
    return out


class SourceGroups:
    """groups: list of server lists [(ip bytes, port, weight, healthy)], flattened once."""

    def __init__(self, groups):
        self.arr = servers_arr([s for g in groups for s in g])
        self.goff = np.zeros(len(groups) + 1, np.int32)
        self.goff[1:] = np.cumsum([len(g) for g in groups])
        self.n = len(groups)


def source_batch_np(groups, view, grp, src4, nthreads=1):
    """-> index within the item's group, or -1"""
    sg = groups if isinstance(groups, SourceGroups) else SourceGroups(groups)
    n = len(grp)
    out = np.empty(n, np.int32)
    lib().vo_source_batch(sg.arr, _ptr(sg.goff), sg.n, view,
                          _ptr(np.ascontiguousarray(grp, np.int32)), _ptr(_u32a(src4)), n,
                          _ptr(out), nthreads)
    return out


def dnsd_batch_np(tcp, udp, dflt, hosts, groups, blob, off, family, remote4, remote6,
                  remote_port, nthreads=1):
    """DNSServer drain loop per datagram (vo_dnsd_batch) -> dict of numpy
    arrays shaped like Classifier.dns_datagrams' (kind/value/qtype only for
    q < nq; the rest zero)."""
    g = groups if isinstance(groups, Groups) else Groups(groups)
    h = hosts if isinstance(hosts, Hosts) else Hosts(hosts)
    n = len(off) - 1
    out = (VoDnsdOut * max(1, n))()
    t = tcp if len(tcp) else np.zeros(1, tcp.dtype)
    u = udp if len(udp) else np.zeros(1, udp.dtype)
    fam = None if family is None else np.ascontiguousarray(family, np.uint8)
    r6 = None if remote6 is None else np.ascontiguousarray(remote6, np.uint8)
    lib().vo_dnsd_batch(_cast(t, VoSgRule), len(tcp), _cast(u, VoSgRule), len(udp),
                        1 if dflt else 0, C.byref(h.h), g.arr, g.n,
                        _ptr(np.ascontiguousarray(blob, np.uint8)), _ptr(_u32a(off)), n,
                        _ptr(fam), _ptr(_u32a(remote4)), _ptr(r6),
                        _ptr(np.ascontiguousarray(remote_port, np.uint16)), out, nthreads)
    a = np.frombuffer(out, dtype=np.int32).reshape(max(1, n), 15)[:n]
    nq = a[:, 2].astype(np.uint8)
    live = np.arange(4)[None, :] < nq[:, None]
    return {"status": a[:, 0].astype(np.uint8), "acl": a[:, 1].copy(), "nq": nq,
            "qtype": np.where(live, a[:, 3:7], 0).astype(np.uint16),
            "kind": np.where(live, a[:, 7:11], 0).astype(np.uint8),
            "value": np.where(live, a[:, 11:15], 0).astype(np.int32)}

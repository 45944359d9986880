"""Python face of the MI355X classifier, named after the reference's classes.

    Network         base/src/main/java/vproxybase/util/Network.java
    SecurityGroup   core/src/main/java/vproxy/component/secure/SecurityGroup.java
    RouteTable      core/src/main/java/vswitch/RouteTable.java
    Upstream hints  core/src/main/java/vproxy/component/svrgroup/Upstream.java + Hint.java
    DNS             core/src/main/java/vproxy/dns/DNSServer.java:116-166

Everything here is plumbing over the C ABI in include/vclassify.h: rule
containers live in C++ (vproxy_amd/csrc/host), classification runs in the
HIP kernels.  Batches may be numpy arrays (host memory; synchronous, PCIe
included) or torch CUDA tensors (device memory; asynchronous on torch's
current stream).
"""
import ctypes as C
import ipaddress

import numpy as np

from . import _lib
from ._lib import (DNSD_MAXQ, PROTO_TCP, PROTO_UDP, IllegalArgumentException, VcAclRule,
                   VcAnnos, VcDnsdOut, VcGroupAnnos, VcNet, VcPktOut, VcServer, check, lib)

HINT_HOST = "vproxy/hint-host"   # AnnotationKeys.ServerGroup_HintHost
HINT_PORT = "vproxy/hint-port"   # AnnotationKeys.ServerGroup_HintPort
HINT_URI = "vproxy/hint-uri"     # AnnotationKeys.ServerGroup_HintUri


def _b(s):
    return s.encode() if isinstance(s, str) else bytes(s)


def parse_ip(s):
    """IP.parseIpString: bytes (4 or 16) or None."""
    out = (C.c_uint8 * 16)()
    n = lib().vc_ip_parse(_b(s), out)
    return None if n < 0 else bytes(out[:n])


class Network:
    """vproxybase.util.Network (ip bytes + parseMask bytes)."""

    def __init__(self, spec=None, *, ip=None, prefix=None, raw=None):
        self.c = VcNet()
        if raw is not None:
            C.memmove(C.byref(self.c), C.byref(raw), C.sizeof(VcNet))
        elif spec is not None:
            check(lib().vc_net_parse(_b(spec), C.byref(self.c)))
        else:
            ipb = _b(ip) if not isinstance(ip, (bytes, bytearray)) else bytes(ip)
            if isinstance(ip, str):
                ipb = parse_ip(ip)
                if ipb is None:
                    raise _lib.IllegalArgumentException("not an ip: %s" % ip)
            buf = (C.c_uint8 * 16).from_buffer_copy(ipb.ljust(16, b"\0"))
            check(lib().vc_net_from_prefix(buf, len(ipb), int(prefix), C.byref(self.c)))

    @property
    def ip(self):
        return bytes(self.c.ip[:self.c.ip_len])

    @property
    def mask(self):
        return bytes(self.c.mask[:self.c.mask_len])

    @property
    def prefix(self):
        """Network.getMask -> maskInt (Network.java:135-145)."""
        zeros = 0
        for b in reversed(self.mask):
            cnt = 8 if b == 0 else (b & -b).bit_length() - 1
            if cnt == 0:
                break
            zeros += cnt
        return len(self.mask) * 8 - zeros

    def contains(self, ip):
        ipb = parse_ip(ip) if isinstance(ip, str) else bytes(ip)
        buf = (C.c_uint8 * 16).from_buffer_copy(ipb.ljust(16, b"\0"))
        return bool(check(lib().vc_net_contains_ip(C.byref(self.c), buf, len(ipb))))

    def __str__(self):
        """Network.toString (Network.java:66-69)."""
        ip = self.ip
        s = ".".join(map(str, ip)) if len(ip) == 4 else str(ipaddress.IPv6Address(ip))
        return "%s/%d" % (s, self.prefix)

    __repr__ = __str__

    def __eq__(self, o):
        return isinstance(o, Network) and self.ip == o.ip and self.mask == o.mask

    def __hash__(self):
        return hash((self.ip, self.mask))


def _proto(p):
    if isinstance(p, str):
        if p in ("TCP", "tcp"):          # ProtocolHandle.get (ProtocolHandle.java:20-31)
            return PROTO_TCP
        if p in ("UDP", "udp"):
            return PROTO_UDP
        raise _lib.IllegalArgumentException("unknown protocol %s" % p)
    return int(p)


class SecurityGroup:
    """Mirror of SecurityGroup (list order, duplicate checks) in C++."""

    def __init__(self, alias, default_allow):
        self.h = C.c_void_p()
        check(lib().vc_secgroup_new(_b(alias), 1 if default_allow else 0, C.byref(self.h)))
        self.alias = alias
        self._default = bool(default_allow)

    def __del__(self):
        try:
            if getattr(self, "h", None) and self.h.value:
                lib().vc_secgroup_free(self.h)
                self.h = C.c_void_p()
        except Exception:       # interpreter shutdown: module globals already gone
            pass

    @property
    def default_allow(self):
        return self._default

    @default_allow.setter
    def default_allow(self, v):
        check(lib().vc_secgroup_set_default(self.h, 1 if v else 0))
        self._default = bool(v)

    def add_rule(self, alias, network, protocol, min_port, max_port, allow):
        net = network if isinstance(network, Network) else Network(network)
        check(lib().vc_secgroup_add_rule(self.h, _b(alias), C.byref(net.c), _proto(protocol),
                                         int(min_port), int(max_port), 1 if allow else 0))

    def remove_rule(self, alias):
        check(lib().vc_secgroup_remove_rule(self.h, _b(alias)))

    def rules(self, protocol):
        n = check(lib().vc_secgroup_rules(self.h, _proto(protocol), None, 0))
        arr = (VcAclRule * max(1, n))()
        lib().vc_secgroup_rules(self.h, _proto(protocol), arr, n)
        return [arr[i] for i in range(n)]


class RouteTable:
    """Mirror of vswitch.RouteTable (insertion-order heuristic) in C++."""

    def __init__(self, v4network=None, v6network=None, vni=0):
        self.h = C.c_void_p()
        a = Network(v4network) if isinstance(v4network, str) else v4network
        b = Network(v6network) if isinstance(v6network, str) else v6network
        check(lib().vc_routetable_new(C.byref(a.c) if a else None, C.byref(b.c) if b else None,
                                      int(vni), C.byref(self.h)))

    def __del__(self):
        try:
            if getattr(self, "h", None) and self.h.value:
                lib().vc_routetable_free(self.h)
                self.h = C.c_void_p()
        except Exception:       # interpreter shutdown: module globals already gone
            pass

    def add_rule(self, alias, network, to_vni=0, via=None):
        net = network if isinstance(network, Network) else Network(network)
        ipb = None
        if via is not None:
            ipb = parse_ip(via) if isinstance(via, str) else bytes(via)
        buf = (C.c_uint8 * 16).from_buffer_copy(ipb.ljust(16, b"\0")) if ipb else None
        check(lib().vc_routetable_add_rule(self.h, _b(alias), C.byref(net.c), int(to_vni), buf,
                                           len(ipb) if ipb else 0))

    def add_rules(self, alias_prefix, networks, to_vni=0, n=None):
        """Bulk addRule in the given order (exact same lists as one by one).
        networks: list of Network/str, or a VcNet ctypes array with count n."""
        if isinstance(networks, C.Array):
            arr, n = networks, (len(networks) if n is None else n)
        else:
            arr, n = net_array(networks), len(networks)
        return check(lib().vc_routetable_add_rules(self.h, _b(alias_prefix), arr, n,
                                                    int(to_vni))) == 1

    def del_rule(self, alias):
        check(lib().vc_routetable_del_rule(self.h, _b(alias)))

    def rules_raw(self, family):
        n = check(lib().vc_routetable_rules(self.h, family, None, 0))
        arr = (VcNet * max(1, n))()
        lib().vc_routetable_rules(self.h, family, arr, n)
        return arr, n

    def rules(self, family):
        arr, n = self.rules_raw(family)
        return [Network(raw=arr[i]) for i in range(n)]

    def get_rules(self):
        """RouteTable.getRules(): v4 list then v6 list."""
        return self.rules(4) + self.rules(6)


def net_array(nets):
    arr = (VcNet * max(1, len(nets)))()
    for i, n in enumerate(nets):
        n = n if isinstance(n, Network) else Network(n)
        C.memmove(C.byref(arr[i]), C.byref(n.c), C.sizeof(VcNet))
    return arr


def acl_rule_array(rules):
    """rules: iterable of (network, min_port, max_port, allow) or VcAclRule."""
    rules = list(rules)
    arr = (VcAclRule * max(1, len(rules)))()
    for i, r in enumerate(rules):
        if isinstance(r, VcAclRule):
            arr[i] = r
            continue
        net, lo, hi, allow = r
        net = net if isinstance(net, Network) else Network(net)
        C.memmove(C.byref(arr[i].net), C.byref(net.c), C.sizeof(VcNet))
        arr[i].min_port, arr[i].max_port, arr[i].allow = int(lo), int(hi), 1 if allow else 0
    return arr, len(rules)


def java_parse_int(s):
    """Integer.parseInt, Annotations' failure -> 0 (Annotations.java:45-58)."""
    if s is None:
        return 0
    if isinstance(s, int):
        return s
    t = s[1:] if s[:1] in ("+", "-") else s
    if not t or not all("0" <= ch <= "9" for ch in t):
        return 0
    v = int(s)
    return v if -2**31 <= v < 2**31 else 0


class Annotations:
    """The hint fields of vproxybase.util.Annotations."""

    def __init__(self, m=None, *, host=None, port=0, uri=None):
        if m is not None:
            host = m.get(HINT_HOST, m.get("host"))
            port = java_parse_int(m.get(HINT_PORT, m.get("port")))
            uri = m.get(HINT_URI, m.get("uri"))
        self.host, self.port, self.uri = host, int(port or 0), uri


class _Keep:
    def __init__(self):
        self.items = []

    def s(self, v):
        if v is None:
            return None, 0
        b = _b(v)
        self.items.append(b)
        return b, len(b)


def group_array(groups):
    """groups: list of (handle annotations, group annotations); each an
    Annotations or a dict with hint keys."""
    keep = _Keep()
    arr = (VcGroupAnnos * max(1, len(groups)))()
    for i, (ha, ga) in enumerate(groups):
        for slot, a in (("handle", ha), ("group", ga)):
            a = a if isinstance(a, Annotations) else Annotations(a or {})
            x = getattr(arr[i], slot)
            x.host, x.host_len = keep.s(a.host)
            x.port = a.port
            x.uri, x.uri_len = keep.s(a.uri)
    return arr, len(groups), keep


def pack_strings(items):
    """list of str/bytes/None -> (blob uint8, off uint32[n+1], null uint8 or None)."""
    bs = [None if x is None else _b(x) for x in items]
    lens = np.fromiter((0 if b is None else len(b) for b in bs), dtype=np.int64, count=len(bs))
    off = np.zeros(len(bs) + 1, dtype=np.int64)
    np.cumsum(lens, out=off[1:])
    if off[-1] >= 2**32:
        raise _lib.IllegalArgumentException("string blob exceeds 4 GiB")
    blob = np.frombuffer(b"".join(b for b in bs if b is not None) or b"\0", dtype=np.uint8)
    null = None
    if any(b is None for b in bs):
        null = np.fromiter((b is None for b in bs), dtype=np.uint8, count=len(bs))
    return blob.copy(), off.astype(np.uint32), null


def server_array(groups):
    """ServerGroup server lists -> (vc_server array, group_off int32 array).
    groups: one list per group of (ip, port, weight, healthy) with ip a
    string or raw 4/16 bytes, in ServerGroup.getServerHandles() order."""
    flat = [sv for g in groups for sv in g]
    arr = (VcServer * max(1, len(flat)))()
    for i, (ip, port, weight, healthy) in enumerate(flat):
        b = parse_ip(ip) if isinstance(ip, str) else bytes(ip)
        if b is None or len(b) not in (4, 16):
            raise _lib.IllegalArgumentException("bad server address %r" % (ip,))
        arr[i].ip[:len(b)] = list(b)
        arr[i].ip_len = len(b)
        arr[i].port = int(port)
        arr[i].weight = int(weight)
        arr[i].healthy = 1 if healthy else 0
    off = np.zeros(len(groups) + 1, np.int32)
    off[1:] = np.cumsum([len(g) for g in groups])
    return arr, off


def cn_of_dn(dn):
    """The CN of an RFC 2253 subject name as checkSNI takes it: the first
    comma-separated piece starting with "CN=" (SSLContextHolder.java:89-104)."""
    for s in dn.split(","):
        if s.startswith("CN="):
            return s[3:]
    return None


def _is_dev(x):
    return x is not None and hasattr(x, "is_cuda") and x.is_cuda


def _ptr(x):
    if x is None:
        return None
    if hasattr(x, "data_ptr"):
        return C.c_void_p(x.data_ptr())
    return C.c_void_p(x.ctypes.data)


def _rows16(x, what):
    """Row count of an IPv6 address array: [m, 16] bytes, or flat bytes of a
    length divisible by 16 (m = len / 16).  Anything else is refused before
    a kernel is handed a row count its buffer does not hold."""
    shape = tuple(x.shape)
    itemsize = x.element_size() if hasattr(x, "element_size") else x.itemsize
    if itemsize != 1:
        raise IllegalArgumentException("%s: uint8 bytes expected" % what)
    if len(shape) == 2 and shape[1] == 16:
        return shape[0]
    if len(shape) == 1 and shape[0] % 16 == 0:
        return shape[0] // 16
    raise IllegalArgumentException("%s: shape %s is not rows of 16 bytes" % (what, shape))


def _stream():
    import torch
    return C.c_void_p(torch.cuda.current_stream().cuda_stream)


class Pin:
    """vc_pin: the snapshots current when it was taken.  A `with` block
    binds it to the calling thread (vc_pin_bind), so that thread's calls on
    the classifier use them; release() drops it."""

    def __init__(self, clf, kinds=None):
        self.clf = clf
        self.h = C.c_void_p()
        check(lib().vc_pin_acquire(clf.h, _lib.SNAP_ALL if kinds is None else int(kinds),
                                   C.byref(self.h)))

    def generation(self, kind):
        g = C.c_uint64()
        check(lib().vc_pin_generation(self.h, int(kind), C.byref(g)))
        return g.value

    def bind(self):
        check(lib().vc_pin_bind(self.clf.h, self.h))

    def unbind(self):
        check(lib().vc_pin_bind(self.clf.h, None))

    def __enter__(self):
        self.bind()
        return self

    def __exit__(self, *exc):
        self.unbind()

    def release(self):
        if self.h and self.h.value:
            lib().vc_pin_release(self.h)
            self.h = C.c_void_p()

    def __del__(self):
        try:
            self.release()
        except Exception:       # interpreter shutdown
            pass


class Classifier:
    """One libvclassify context on one GPU.  Raises DeviceError without a
    usable gfx950 device: there is no CPU path."""

    def __init__(self, device=0):
        self.h = C.c_void_p()
        check(lib().vc_create(int(device), C.byref(self.h)))
        self.device = device

    def close(self):
        if self.h and self.h.value:
            lib().vc_destroy(self.h)
            self.h = C.c_void_p()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    # ---------------- snapshots ----------------
    def pin(self, kinds=None):
        """Pin the current snapshots (vc_pin_acquire; kinds = bit set of
        1 << SNAP_*, default all).  `with clf.pin() as p:` binds it to this
        thread for the block's calls."""
        return Pin(self, kinds)

    def generation(self, kind):
        g = C.c_uint64()
        check(lib().vc_generation(self.h, int(kind), C.byref(g)))
        return g.value

    # ---------------- compile ----------------
    def compile_acl(self, tcp_rules, udp_rules, default_allow):
        t, nt = acl_rule_array(tcp_rules)
        u, nu = acl_rule_array(udp_rules)
        check(lib().vc_compile_acl(self.h, t, nt, u, nu, 1 if default_allow else 0))

    def compile_security_group(self, sg):
        check(lib().vc_secgroup_compile(self.h, sg.h))

    def compile_routes(self, v4, v6=()):
        a = v4 if isinstance(v4, C.Array) else net_array(v4)
        b = v6 if isinstance(v6, C.Array) else net_array(v6)
        na = len(v4) if not isinstance(v4, C.Array) else len(a)
        nb = len(v6) if not isinstance(v6, C.Array) else len(b)
        check(lib().vc_compile_routes(self.h, a, na, b, nb))

    def compile_routes_raw(self, v4arr, n4, v6arr, n6):
        check(lib().vc_compile_routes(self.h, v4arr, n4, v6arr, n6))

    def compile_route_table(self, rt):
        check(lib().vc_routetable_compile(self.h, rt.h))

    def compile_vni_routes(self, tables):
        """Switch.tables (Switch.java:560-566): the route table of each VNI
        for switch_classify.  tables: list of (vni, nets4, nets6), nets as
        workloads.NET_DT arrays in list order; [] removes them."""
        from .workloads import NET_DT
        vni = np.array([t[0] for t in tables] or [0], np.int32)
        o4 = np.zeros(len(tables) + 1, np.int32)
        o6 = np.zeros(len(tables) + 1, np.int32)
        o4[1:] = np.cumsum([len(t[1]) for t in tables]) if tables else []
        o6[1:] = np.cumsum([len(t[2]) for t in tables]) if tables else []
        a4 = np.concatenate([t[1] for t in tables] + [np.zeros(1, NET_DT)])
        a6 = np.concatenate([t[2] for t in tables] + [np.zeros(1, NET_DT)])
        check(lib().vc_compile_vni_routes(self.h, _ptr(vni), _ptr(a4), _ptr(o4), _ptr(a6),
                                          _ptr(o6), len(tables)))

    def compile_route_tables_vni(self, rts):
        """Switch.tables from RouteTable mirrors, each under its own VNI."""
        arr = (C.c_void_p * max(1, len(rts)))(*[rt.h.value for rt in rts])
        check(lib().vc_routetables_compile_vni(self.h, arr, len(rts)))

    def compile_upstream(self, groups):
        arr, n, keep = group_array(groups)
        check(lib().vc_compile_upstream(self.h, arr, n))

    def compile_hosts(self, pairs):
        keys = [_b(k) for k, _ in pairs]
        karr = (C.c_char_p * max(1, len(keys)))(*keys)
        lens = np.array([len(k) for k in keys] or [0], dtype=np.int32)
        vals = np.array([v for _, v in pairs] or [0], dtype=np.int32)
        check(lib().vc_compile_hosts(self.h, karr, _ptr(lens), _ptr(vals), len(keys)))

    def compile_hosts_text(self, text):
        t = _b(text)
        check(lib().vc_compile_hosts_text(self.h, t, len(t)))

    # ---------------- classify ----------------
    def acl_v4(self, proto, src4, port, out_idx=None, out_allow=None, want_allow=True):
        """Batched SecurityGroup.allow over IPv4 sources -> (idx, allow)."""
        n = len(src4)
        if _is_dev(src4):
            import torch
            out_idx = out_idx if out_idx is not None else torch.empty(n, dtype=torch.int32,
                                                                      device=src4.device)
            if want_allow and out_allow is None:
                out_allow = torch.empty(n, dtype=torch.uint8, device=src4.device)
            check(lib().vc_acl_classify_v4_dev(self.h, _ptr(proto), _ptr(src4), _ptr(port), n,
                                               _ptr(out_idx), _ptr(out_allow), _stream()))
        else:
            proto, src4, port = (np.ascontiguousarray(proto, np.uint8),
                                 np.ascontiguousarray(src4, np.uint32),
                                 np.ascontiguousarray(port, np.uint16))
            out_idx = np.empty(n, np.int32)
            out_allow = np.empty(n, np.uint8) if want_allow else None
            check(lib().vc_acl_classify_v4(self.h, _ptr(proto), _ptr(src4), _ptr(port), n,
                                           _ptr(out_idx), _ptr(out_allow)))
        return out_idx, out_allow

    def acl_v6(self, proto, src6, port, want_allow=True):
        n = len(port)
        if _is_dev(src6):
            import torch
            out_idx = torch.empty(n, dtype=torch.int32, device=src6.device)
            out_allow = torch.empty(n, dtype=torch.uint8, device=src6.device) if want_allow else None
            check(lib().vc_acl_classify_v6_dev(self.h, _ptr(proto), _ptr(src6), _ptr(port), n,
                                               _ptr(out_idx), _ptr(out_allow), _stream()))
        else:
            proto, src6, port = (np.ascontiguousarray(proto, np.uint8),
                                 np.ascontiguousarray(src6, np.uint8),
                                 np.ascontiguousarray(port, np.uint16))
            out_idx = np.empty(n, np.int32)
            out_allow = np.empty(n, np.uint8) if want_allow else None
            check(lib().vc_acl_classify_v6(self.h, _ptr(proto), _ptr(src6), _ptr(port), n,
                                           _ptr(out_idx), _ptr(out_allow)))
        return out_idx, out_allow

    def route_v4(self, dst4, out=None):
        n = len(dst4)
        if _is_dev(dst4):
            import torch
            out = out if out is not None else torch.empty(n, dtype=torch.int32, device=dst4.device)
            check(lib().vc_route_lookup_v4_dev(self.h, _ptr(dst4), n, _ptr(out), _stream()))
        else:
            dst4 = np.ascontiguousarray(dst4, np.uint32)
            out = np.empty(n, np.int32)
            check(lib().vc_route_lookup_v4(self.h, _ptr(dst4), n, _ptr(out)))
        return out

    def route_v6(self, dst6, out=None):
        n = len(dst6)
        if _is_dev(dst6):
            import torch
            out = out if out is not None else torch.empty(n, dtype=torch.int32, device=dst6.device)
            check(lib().vc_route_lookup_v6_dev(self.h, _ptr(dst6), n, _ptr(out), _stream()))
        else:
            dst6 = np.ascontiguousarray(dst6, np.uint8)
            out = np.empty(n, np.int32)
            check(lib().vc_route_lookup_v6(self.h, _ptr(dst6), n, _ptr(out)))
        return out

    def hint_search(self, hosts, ports=None, uris=None):
        """Batched Upstream.searchForGroup(Hint.ofHostPortUri(host, port, uri)).
        hosts/uris: lists of str/None (host path) or packed (blob, off, null)
        tuples of torch CUDA tensors (device path)."""
        if isinstance(hosts, tuple) and _is_dev(hosts[0]):
            import torch
            hb, ho, hn = hosts
            n = len(ho) - 1
            ub, uo, un = uris if uris is not None else (None, None, None)
            out = torch.empty(n, dtype=torch.int32, device=hb.device)
            check(lib().vc_hint_search_dev(self.h, _ptr(hb), _ptr(ho), _ptr(hn), _ptr(ports),
                                           _ptr(ub), _ptr(uo), _ptr(un), n, _ptr(out), _stream()))
            return out
        n = len(hosts)
        hb, ho, hn = pack_strings(hosts)
        ub = uo = un = None
        if uris is not None:
            ub, uo, un = pack_strings(uris)
        p = np.ascontiguousarray(ports if ports is not None else np.zeros(n), np.uint16)
        out = np.empty(n, np.int32)
        check(lib().vc_hint_search(self.h, _ptr(hb), _ptr(ho), _ptr(hn), _ptr(p), _ptr(ub),
                                   _ptr(uo), _ptr(un), n, _ptr(out)))
        return out

    def dns_classify(self, qnames):
        """Batched DNSServer.handleRequest classification -> (kind, value)."""
        if isinstance(qnames, tuple) and _is_dev(qnames[0]):
            import torch
            qb, qo = qnames[0], qnames[1]
            n = len(qo) - 1
            kind = torch.empty(n, dtype=torch.uint8, device=qb.device)
            val = torch.empty(n, dtype=torch.int32, device=qb.device)
            check(lib().vc_dns_classify_dev(self.h, _ptr(qb), _ptr(qo), n, _ptr(kind), _ptr(val),
                                            _stream()))
            return kind, val
        n = len(qnames)
        qb, qo, _ = pack_strings(qnames)
        kind = np.empty(n, np.uint8)
        val = np.empty(n, np.int32)
        check(lib().vc_dns_classify(self.h, _ptr(qb), _ptr(qo), n, _ptr(kind), _ptr(val)))
        return kind, val

    def http_hint(self, heads):
        """HttpContext.connectionHint + Upstream.searchForGroup per HTTP/1
        request head (vc_http_hint[_dev], HttpContext.java:55-71 over
        HttpSubContext's request line and headers) -> (group, kind): group =
        handle index or -1, kind = VC_HTTP_* (0: null hint).  heads: a list
        of bytes, or (blob, off) torch CUDA tensors (int32 off, n + 1)."""
        if isinstance(heads, tuple) and _is_dev(heads[0]):
            import torch
            hb, ho = heads[0], heads[1]
            # refused before the kernel sees them: an int64 offsets tensor
            # would be read as uint32 pairs, a wider blob dtype would make
            # numel() undercount its bytes
            if hb.dtype != torch.uint8 or not hb.is_contiguous():
                raise IllegalArgumentException("http heads: a contiguous uint8 blob expected")
            if (ho.dtype not in (torch.int32, getattr(torch, "uint32", torch.int32)) or
                    not ho.is_contiguous() or ho.dim() != 1 or len(ho) < 1 or
                    ho.device != hb.device):
                raise IllegalArgumentException(
                    "http heads: contiguous 32-bit offsets (n + 1) on the blob's device expected")
            n = len(ho) - 1
            grp = torch.empty(n, dtype=torch.int32, device=hb.device)
            kind = torch.empty(n, dtype=torch.uint8, device=hb.device)
            check(lib().vc_http_hint_dev(self.h, _ptr(hb), hb.numel(), _ptr(ho), n, _ptr(grp),
                                         _ptr(kind), _stream()))
            return grp, kind
        n = len(heads)
        hb, ho, _ = pack_strings(heads)
        grp = np.empty(n, np.int32)
        kind = np.empty(n, np.uint8)
        check(lib().vc_http_hint(self.h, _ptr(hb), _ptr(ho), n, _ptr(grp), _ptr(kind)))
        return grp, kind

    def dns_datagrams(self, datagrams, remote4, remote_port, remote6=None, remote_family=None):
        """DNSServer's drain loop per datagram (vc_dns_datagrams[_dev],
        DNSServer.java:457-500): securityGroup.allow(UDP, remote, remote
        port), Formatter.parsePackets, isResponse / opcode / handleRequest's
        question classification.  datagrams: (blob, off) torch CUDA tensors
        or numpy arrays, or a list of bytes; remote4 uint32 keys, remote_port
        uint16, remote6 [n, 16] uint8 and remote_family uint8 (4/6) optional.
        Returns dict(status, acl, nq, qtype[n, MAXQ], kind[n, MAXQ],
        value[n, MAXQ]); kind / value / qtype are meaningful for q < nq."""
        if isinstance(datagrams, (list, tuple)) and not (
                len(datagrams) == 2 and hasattr(datagrams[1], "dtype")):
            blob, off, _ = pack_strings(datagrams)
        else:
            blob, off = datagrams
        n = len(off) - 1
        if _is_dev(blob):
            import torch
            dev = blob.device
            mk = lambda shape, dt: torch.empty(shape, dtype=dt, device=dev)
            res = {"status": mk(n, torch.uint8), "acl": mk(n, torch.int32),
                   "nq": mk(n, torch.uint8), "qtype": mk((n, DNSD_MAXQ), torch.int16),
                   "kind": mk((n, DNSD_MAXQ), torch.uint8),
                   "value": mk((n, DNSD_MAXQ), torch.int32)}
            o = VcDnsdOut(**{k: v.data_ptr() for k, v in res.items()})
            check(lib().vc_dns_datagrams_dev(self.h, _ptr(blob), _ptr(off), n,
                                             _ptr(remote_family), _ptr(remote4), _ptr(remote6),
                                             _ptr(remote_port), C.byref(o), _stream()))
            return res
        res = {"status": np.empty(n, np.uint8), "acl": np.empty(n, np.int32),
               "nq": np.empty(n, np.uint8), "qtype": np.zeros((n, DNSD_MAXQ), np.uint16),
               "kind": np.zeros((n, DNSD_MAXQ), np.uint8),
               "value": np.zeros((n, DNSD_MAXQ), np.int32)}
        keep = [np.ascontiguousarray(blob, np.uint8), np.ascontiguousarray(off, np.uint32),
                np.ascontiguousarray(remote4, np.uint32),
                np.ascontiguousarray(remote_port, np.uint16)]
        fam = None if remote_family is None else np.ascontiguousarray(remote_family, np.uint8)
        r6 = None if remote6 is None else np.ascontiguousarray(remote6, np.uint8).reshape(-1, 16)
        o = VcDnsdOut(**{k: v.ctypes.data for k, v in res.items()})
        check(lib().vc_dns_datagrams(self.h, _ptr(keep[0]), _ptr(keep[1]), n, _ptr(fam),
                                     _ptr(keep[2]), _ptr(r6), _ptr(keep[3]), C.byref(o)))
        return res

    def pipeline_v4(self, proto, src4, dst4, dport, host_id, pool_group, outs=None,
                    want_allow=False, kernel_done_event=None, count_stream=None):
        """Combined ACL -> route -> host pipeline on device tensors (IPv4).
        kernel_done_event: optional raw hipEvent_t (int) recorded right after
        the classify kernel; count_stream: optional torch stream the
        hit-counter finish passes run on (after the kernel)."""
        return self.pipeline(proto, src4, dst4, dport, host_id, pool_group, outs=outs,
                             want_allow=want_allow, kernel_done_event=kernel_done_event,
                             count_stream=count_stream)

    def pipeline(self, proto, src4, dst4, dport, host_id=None, pool_group=None, family=None,
                 src6=None, dst6=None, outs=None, want_allow=False, kernel_done_event=None,
                 count_stream=None, compact6=False):
        """vc_pipeline(_dev): per packet SecurityGroup.allow(proto, src, dport)
        -> RouteTable.lookup(dst) (rulesV4 or rulesV6 by `family`, 4 or 6)
        -> pool_group[host_id].  torch CUDA tensors run on the device
        (asynchronous, torch's current stream); numpy arrays take the host
        entry point (synchronous, PCIe included).  src6/dst6: n x 16 bytes, or
        with compact6 (vc_pipeline_c6_dev, or vc_pipeline_c6 for numpy) one
        row per IPv6 packet in packet order.  Returns (acl, route, group, allow)."""
        n = len(proto)
        dev = _is_dev(proto)
        n6 = 0
        if src6 is not None or dst6 is not None:
            if src6 is None or dst6 is None:
                raise IllegalArgumentException("src6 and dst6 come together")
            n6 = _rows16(src6, "src6")
            if _rows16(dst6, "dst6") != n6:
                raise IllegalArgumentException("src6 has %d rows, dst6 %d" % (n6, _rows16(dst6, "dst6")))
            if not compact6 and n6 != n:
                raise IllegalArgumentException("src6/dst6: %d rows for %d packets (one row per "
                                               "packet without compact6)" % (n6, n))
            if compact6 and n6 > n:
                raise IllegalArgumentException("compact6: %d IPv6 rows for %d packets" % (n6, n))
        elif compact6 and family is not None:
            raise IllegalArgumentException("compact6 needs src6 / dst6 rows")
        if dev:
            import torch
            mk = lambda dt: torch.empty(n, dtype=dt, device=proto.device)
            if outs is None:
                outs = (mk(torch.int32), mk(torch.int32), mk(torch.int32),
                        mk(torch.uint8) if want_allow else None)
        else:
            conv = lambda x, dt: None if x is None else np.ascontiguousarray(x, dt)
            proto, src4, dst4 = conv(proto, np.uint8), conv(src4, np.uint32), conv(dst4, np.uint32)
            dport, host_id = conv(dport, np.uint16), conv(host_id, np.uint32)
            pool_group, family = conv(pool_group, np.int32), conv(family, np.uint8)
            src6, dst6 = conv(src6, np.uint8), conv(dst6, np.uint8)
            if outs is None:
                outs = (np.empty(n, np.int32), np.empty(n, np.int32), np.empty(n, np.int32),
                        np.empty(n, np.uint8) if want_allow else None)
        keep = (proto, src4, dst4, dport, host_id, pool_group, family, src6, dst6)
        pk = _lib.VcPackets(*[x.value if x is not None else None for x in
                              (_ptr(family), _ptr(proto), _ptr(src4), _ptr(dst4), _ptr(src6),
                               _ptr(dst6), _ptr(dport), _ptr(host_id))])
        a, r, g, al = outs
        po = _lib.VcPipelineOut(*[x.value if x is not None else None for x in
                                  (_ptr(a), _ptr(r), _ptr(g), _ptr(al))])
        n_pool = len(pool_group) if pool_group is not None else 0
        if dev and compact6:
            check(lib().vc_pipeline_c6_dev(self.h, C.byref(pk), n, n6, _ptr(pool_group),
                                           n_pool, C.byref(po), _stream(),
                                           C.c_void_p(count_stream.cuda_stream)
                                           if count_stream is not None else None,
                                           C.c_void_p(kernel_done_event)
                                           if kernel_done_event else None))
        elif dev:
            check(lib().vc_pipeline_dev(self.h, C.byref(pk), n, _ptr(pool_group), n_pool,
                                        C.byref(po), _stream(),
                                        C.c_void_p(count_stream.cuda_stream)
                                        if count_stream is not None else None,
                                        C.c_void_p(kernel_done_event)
                                        if kernel_done_event else None))
        elif compact6:
            check(lib().vc_pipeline_c6(self.h, C.byref(pk), n, n6, _ptr(pool_group),
                                       n_pool, C.byref(po)))
        else:
            check(lib().vc_pipeline(self.h, C.byref(pk), n, _ptr(pool_group), n_pool,
                                    C.byref(po)))
        del keep
        return outs

    # ---------------- header extraction ----------------
    _PKT_FIELDS = (("status", 1, "u8"), ("l3", 1, "u8"), ("l4", 1, "u8"), ("proto", 1, "u8"),
                   ("vni", 1, "u32"), ("ether_type", 1, "u16"), ("src4", 1, "u32"),
                   ("dst4", 1, "u32"), ("src6", 16, "u8"), ("dst6", 16, "u8"),
                   ("sport", 1, "u16"), ("dport", 1, "u16"))

    def parse_packets(self, frames, layer=0):
        """VXLanPacket/EthernetPacket/Ipv4Packet/Ipv6Packet.from over a batch
        of raw frames: a list of bytes (host path) or (blob, off) torch
        tensors (device path).  Returns a dict of arrays (vclassify.h
        vc_pkt_out); src6/dst6 are n x 16."""
        if isinstance(frames, tuple) and _is_dev(frames[0]):
            import torch
            blob, off = frames
            n = len(off) - 1
            tdt = {"u8": torch.uint8, "u16": torch.int16, "u32": torch.int32}
            res = {k: torch.empty((n, w) if w > 1 else (n,), dtype=tdt[t], device=blob.device)
                   for k, w, t in self._PKT_FIELDS}
            o = VcPktOut(**{k: v.data_ptr() for k, v in res.items()})
            check(lib().vc_parse_packets_dev(self.h, _ptr(blob), _ptr(off), n, int(layer),
                                             C.byref(o), _stream()))
            return res
        lens = np.array([len(f) for f in frames], np.int64)
        off = np.zeros(len(frames) + 1, np.uint32)
        off[1:] = np.cumsum(lens)
        blob = np.frombuffer(b"".join(bytes(f) for f in frames) or b"\0", np.uint8).copy()
        n = len(frames)
        ndt = {"u8": np.uint8, "u16": np.uint16, "u32": np.uint32}
        res = {k: np.zeros((n, w) if w > 1 else (n,), ndt[t]) for k, w, t in self._PKT_FIELDS}
        o = VcPktOut(**{k: v.ctypes.data for k, v in res.items()})
        check(lib().vc_parse_packets(self.h, _ptr(blob), _ptr(off), n, int(layer), C.byref(o)))
        return res

    def switch_classify(self, frames, remote4, bind_port, remote6=None, remote_family=None,
                        layer=0):
        """Switch.PacketHandler.readable per datagram in one kernel
        (vc_switch_classify_dev): bareVXLanAccess.allow(UDP, remote,
        bind_port), the VXLAN parse and RouteTable.lookup(inner dst).
        frames: (blob, off) torch CUDA tensors; remote4 int32 tensor,
        remote6 [n, 16] uint8, remote_family uint8 (4/6).  Returns
        (parse fields dict, acl, allow, route)."""
        import torch
        blob, off = frames
        n = len(off) - 1
        dev = blob.device
        tdt = {"u8": torch.uint8, "u16": torch.int16, "u32": torch.int32}
        res = {k: torch.empty((n, w) if w > 1 else (n,), dtype=tdt[t], device=dev)
               for k, w, t in self._PKT_FIELDS}
        o = VcPktOut(**{k: v.data_ptr() for k, v in res.items()})
        acl = torch.empty(n, dtype=torch.int32, device=dev)
        allow = torch.empty(n, dtype=torch.uint8, device=dev)
        route = torch.empty(n, dtype=torch.int32, device=dev)
        check(lib().vc_switch_classify_dev(self.h, _ptr(blob), _ptr(off), n, int(layer),
                                           _ptr(remote_family), _ptr(remote4), _ptr(remote6),
                                           int(bind_port), C.byref(o), _ptr(acl), _ptr(allow),
                                           _ptr(route), _stream()))
        return res, acl, allow, route

    # ---------------- ServerGroup source hashing ----------------
    def compile_servers(self, groups):
        """Server lists per group (see server_array)."""
        arr, off = server_array(groups)
        self._server_off = off
        check(lib().vc_compile_servers(self.h, arr, _ptr(off), len(groups)))

    def set_server_health(self, healthy):
        h = np.ascontiguousarray(healthy, np.uint8)
        check(lib().vc_servers_set_health(self.h, _ptr(h), len(h)))

    def source_select(self, group, src, view=0):
        """ServerGroup.next/nextIPv4/nextIPv6(source) (method source) per item:
        group indices + client addresses (uint32 v4 keys, or n x 16 bytes for
        IPv6) -> server index within the group, -1 = null."""
        n = len(group)
        v6 = (src.dtype == np.uint8 or (hasattr(src, "dtype") and "uint8" in str(src.dtype))) \
            and src.ndim == 2
        if _is_dev(group):
            import torch
            out = torch.empty(n, dtype=torch.int32, device=group.device)
            f = lib().vc_source_select_v6_dev if v6 else lib().vc_source_select_v4_dev
            check(f(self.h, _ptr(group), _ptr(src), n, int(view), _ptr(out), _stream()))
            return out
        group = np.ascontiguousarray(group, np.int32)
        src = np.ascontiguousarray(src, np.uint8 if v6 else np.uint32)
        out = np.empty(n, np.int32)
        f = lib().vc_source_select_v6 if v6 else lib().vc_source_select_v4
        check(f(self.h, _ptr(group), _ptr(src), n, int(view), _ptr(out)))
        return out

    # ---------------- TLS certificate choice by SNI ----------------
    def compile_certs(self, holders):
        """SSLContextHolder.add for every holder in order (SSLContextHolder.java:47-49):
        holders = list of name lists, each the CNs and SAN dNSNames of the
        holder's certificates (see cn_of_dn)."""
        names = [_b(s) for hs in holders for s in hs]
        hold = np.array([h for h, hs in enumerate(holders) for _ in hs] or [0], np.int32)
        karr = (C.c_char_p * max(1, len(names)))(*names)
        lens = np.array([len(s) for s in names] or [0], np.int32)
        check(lib().vc_compile_certs(self.h, karr, _ptr(lens), _ptr(hold), len(names),
                                     len(holders)))

    def cert_choose(self, snis):
        """Batched SSLContextHolder.choose(sni) -> holder index (-1: no holders).
        snis: list of str/bytes/None, or a packed (blob, off, null) tuple of
        torch CUDA tensors (device path)."""
        if isinstance(snis, tuple) and _is_dev(snis[0]):
            import torch
            b, o, nul = snis
            n = len(o) - 1
            out = torch.empty(n, dtype=torch.int32, device=b.device)
            check(lib().vc_cert_choose_dev(self.h, _ptr(b), _ptr(o), _ptr(nul), n, _ptr(out),
                                           _stream()))
            return out
        n = len(snis)
        b, o, nul = pack_strings(snis)
        out = np.empty(n, np.int32)
        check(lib().vc_cert_choose(self.h, _ptr(b), _ptr(o), _ptr(nul), n, _ptr(out)))
        return out

    # ---------------- traffic-mirror filters ----------------
    def compile_mirror(self, filters):
        """Mirror's filter list (dict configs, list order); returns the
        MirrorFilters interning used for origins / protocol names."""
        from .mirror import MirrorFilters
        mf = MirrorFilters()
        arr, n = mf.build(filters)
        check(lib().vc_compile_mirror(self.h, arr, n))
        self._mirror = mf
        return mf

    def mirror_match(self, origin, cols, n):
        """Mirror.mirror's filter step per item -> uint64 mirror bit sets.
        cols: vc_mirror_items arrays (numpy: host path; torch CUDA: device
        path), protocol columns already interned (MirrorFilters.id_of)."""
        from .mirror import items_struct
        oid = self._mirror.id_of(origin, create=False)
        it = items_struct(cols)
        if any(_is_dev(v) for v in cols.values()):
            import torch
            dev = next(v for v in cols.values() if _is_dev(v)).device
            out = torch.empty(n, dtype=torch.int64, device=dev)
            check(lib().vc_mirror_match_dev(self.h, oid, C.byref(it), n, _ptr(out), _stream()))
            return out
        out = np.empty(n, np.uint64)
        check(lib().vc_mirror_match(self.h, oid, C.byref(it), n, _ptr(out)))
        return out

    def mirror_switch(self, origin, frames, layer=0):
        """Mirror.switchPacket per raw frame -> uint64 mirror bit sets.
        frames: list of bytes, or a (blob, off) tuple of torch CUDA tensors."""
        oid = self._mirror.id_of(origin, create=False)
        if isinstance(frames, tuple) and _is_dev(frames[0]):
            import torch
            b, o = frames
            n = len(o) - 1
            out = torch.empty(n, dtype=torch.int64, device=b.device)
            check(lib().vc_mirror_switch_dev(self.h, oid, _ptr(b), _ptr(o), n, int(layer),
                                             _ptr(out), _stream()))
            return out
        n = len(frames)
        b, o, _ = pack_strings(frames)
        out = np.empty(n, np.uint64)
        check(lib().vc_mirror_switch(self.h, oid, _ptr(b), _ptr(o), n, int(layer), _ptr(out)))
        return out

    # ---------------- counters ----------------
    def counters_enable(self, on=True):
        check(lib().vc_counters_enable(self.h, 1 if on else 0))

    def counters_device(self, kind):
        p = C.c_void_p()
        n = C.c_int64()
        check(lib().vc_counters_device(self.h, kind, C.byref(p), C.byref(n)))
        return p.value, n.value

    def counters_read(self, kind):
        _, n = self.counters_device(kind)
        out = np.zeros(max(1, n), np.uint64)
        check(lib().vc_counters_read(self.h, kind, _ptr(out), n))
        return out[:n]

    def counters_reset(self):
        check(lib().vc_counters_reset(self.h))

    def table_digest(self, kind):
        """vc_table_digest: 64-bit digest of the compiled image of the current
        snapshot (kind COUNTERS_ACL / _ROUTE / _GROUP)."""
        d = C.c_uint64()
        check(lib().vc_table_digest(self.h, kind, C.byref(d)))
        return d.value

    def counters_prometheus(self, extra_labels=None):
        """The current hit counters as Prometheus text (vc_counters_prometheus)."""
        from .prometheus import _b as pb, _call_text
        return _call_text(lib().vc_counters_prometheus, self.h,
                          None if extra_labels is None else pb(extra_labels))

    def counters_add(self, kind, out, aux=None, family=4):
        """Explicit counting pass over a device output array (torch tensor)."""
        check(lib().vc_counters_add_dev(self.h, kind, _ptr(out), _ptr(aux), family, len(out),
                                        _stream()))


def digest_acl(tcp, udp, default_allow=False):
    """vc_digest_acl over RULE_DT arrays (host only, no device)."""
    from . import workloads as W
    a, na, ka = W.as_ctypes(tcp, VcAclRule)
    b, nb, kb = W.as_ctypes(udp, VcAclRule)
    d = C.c_uint64()
    check(lib().vc_digest_acl(a, na, b, nb, 1 if default_allow else 0, C.byref(d)))
    return d.value


def digest_routes(v4, v6):
    """vc_digest_routes over NET_DT arrays in list order (host only)."""
    from . import workloads as W
    a, na, ka = W.as_ctypes(v4, VcNet)
    b, nb, kb = W.as_ctypes(v6, VcNet)
    d = C.c_uint64()
    check(lib().vc_digest_routes(a, na, b, nb, C.byref(d)))
    return d.value


def digest_upstream(groups):
    """vc_digest_upstream over (handle annotations, group annotations) pairs (host only)."""
    arr, n, keep = group_array(groups)
    d = C.c_uint64()
    check(lib().vc_digest_upstream(arr, n, C.byref(d)))
    return d.value

"""Shared edge-case generators for the CPU (image) and GPU parity tests."""
import numpy as np

import oracle_ffi as O
from vproxy_amd import workloads as W


def rule_row(netstr, lo, hi, allow):
    r = np.zeros(1, W.RULE_DT)
    r["net"] = np.frombuffer(bytes(O.net(netstr)), W.NET_DT)
    r["min_port"], r["max_port"], r["allow"] = lo, hi, 1 if allow else 0
    return r


def acl_edge_rules():
    """Rule lists exercising Network.maskMatch's cross-family cases
     and port-range edges."""
    tcp_specs = [
        ("10.0.0.0/8", 80, 80, False),
        ("::ffff:0:0/96", 0, 1000, True),       # every IPv4 input (case 3)
        ("::/80", 443, 443, False),             # every IPv4 input (case 3, m-96 < 0)
        ("::/33", 22, 22, True),
        ("2001:db8::/32", 0, 65535, False),     # 4-byte mask: first 4 bytes (case 1)
        ("[0000:0010:0000:0000:0000:0000:0000:0000]/28", 100, 200, True),
        ("127.0.0.1/32", 0, 65535, True),       # matches ::7f00:1 and ::ffff:7f00:1 (case 4)
        ("1.2.3.0/24", 500, 400, True),         # min > max: never matches
        ("::ffff:7f00:0/104", 5000, 6000, False),
        ("::7f00:0/104", 6000, 7000, True),
        ("0.0.0.0/0", 1024, 2048, True),
        ("2001:db8:1::/48", 53, 53, True),
        ("::/0", 0, 65535, True),               # never matches IPv4 input (case 2)
        ("0.0.0.0/0", 0, 65535, False),         # catch-all
        ("192.168.0.0/16", 0, 65535, True),     # shadowed by the catch-all
    ]
    udp_specs = [
        ("0.0.0.0/0", 53, 53, True),
        ("::1/128", 0, 65535, True),
        ("::/0", 0, 0, False),
        ("8.8.0.0/16", 0, 65535, False),
        ("::ffff:8.8.8.0/120", 0, 65535, True),
        ("8.8.8.8/32", 65535, 65535, True),
        ("::8.8.8.0/120", 100, 65535, True),
    ]
    tcp = np.concatenate([rule_row(*s) for s in tcp_specs])
    udp = np.concatenate([rule_row(*s) for s in udp_specs])
    return tcp, udp


def v6_edge_inputs(rng, n):
    """IPv6 sources: mapped / compat IPv4, near-misses on bytes 10-11,
    2001:db8 space, ::1, zero, random; edge ports."""
    src = rng.integers(0, 256, (n, 16), dtype=np.int64).astype(np.uint8)
    kind = rng.integers(0, 8, n)
    v4 = rng.choice(np.array([[127, 0, 0, 1], [8, 8, 8, 8], [10, 1, 2, 3], [1, 2, 3, 4],
                              [192, 168, 1, 1], [8, 8, 8, 200]], dtype=np.uint8), n)
    rand4 = rng.integers(0, 256, (n, 4), dtype=np.int64).astype(np.uint8)
    v4 = np.where((rng.random(n) < 0.5)[:, None], v4, rand4)
    for k, (b10, b11) in enumerate([(0, 0), (0xFF, 0xFF), (0, 0xFF), (0xFF, 0)]):
        sel = kind == k
        src[sel, :10] = 0
        src[sel, 10] = b10
        src[sel, 11] = b11
        src[sel, 12:] = v4[sel]
    sel = kind == 4
    src[sel, :4] = [0x20, 0x01, 0x0D, 0xB8]
    src[sel & (rng.random(n) < 0.5), 4:6] = [0, 1]
    sel = kind == 5
    src[sel] = 0
    src[sel & (rng.random(n) < 0.5), 15] = 1
    sel = kind == 6
    src[sel, 0] = 0
    src[sel, 1] = rng.integers(0, 0x20, sel.sum())
    proto = rng.choice(np.array([6, 17, 1], dtype=np.uint8), n)
    port = rng.choice(np.array([0, 22, 53, 80, 100, 443, 999, 1000, 1024, 2048, 5000, 6000, 65535],
                               dtype=np.uint16), n)
    rp = rng.random(n) < 0.3
    port[rp] = rng.integers(0, 65536, rp.sum())
    return src, proto, port


_HOSTS = ["com", "a.com", "b.a.com", "www.a.com", "x.net", "y.x.net", "*", "example.com",
          "s1.test.com", "s2.test.com", "test.com", "", "a.b.c.d.e.f", "127.0.0.1", "::1",
          "[::1]", "com.", "*.com"]
_URIS = [None, None, None, "/", "/a", "/a/b", "*", "", "/b", "/a/b/c/d"]


def hint_cases_random(rng, ng, nq):
    """Groups with overlapping hint-hosts (long member lists, suffix chains),
    handle/group annotation merging, hint-ports and hint-uris; queries with
    ports, ':port' host forms, www., IPv6 literals, nulls and URI variants."""
    groups = []
    for _ in range(ng):
        def annos():
            a = {}
            if rng.random() < 0.7:
                a["host"] = _HOSTS[int(rng.integers(0, len(_HOSTS)))]
            if rng.random() < 0.2:
                a["port"] = int(rng.choice([80, 8080, 443]))
            if rng.random() < 0.3:
                u = _URIS[int(rng.integers(0, len(_URIS)))]
                if u is not None:
                    a["uri"] = u
            return a
        groups.append((annos() if rng.random() < 0.3 else {}, annos()))
    prefixes = ["", "www.", "m.", "q.w."]
    queries = []
    for _ in range(nq):
        r = rng.random()
        if r < 0.05:
            host = None
        else:
            host = prefixes[int(rng.integers(0, 4))] + _HOSTS[int(rng.integers(0, len(_HOSTS)))]
            if rng.random() < 0.2:
                host += ":%d" % int(rng.choice([80, 8080, 1]))
            if rng.random() < 0.03:
                host = "[::1]:80"
        port = int(rng.choice([0, 0, 80, 8080, 443]))
        uri = ["/a/b/c", "/a/", "/a?x=1", "/", "/b/", "*", "/z", None, None, "/a/b"][
            int(rng.integers(0, 10))]
        queries.append((host, port, uri))
    return groups, _HOSTS, queries


def hint_cases_shapes(rng, n):
    """Groups keyed on short, long (> 48 B inline key) and deep (many-label)
    hint-hosts, and hostnames that stress the word-at-a-time fast path:
    every length mod 4, more labels than the batched probe holds, names
    long enough that a wave's 64 names overflow its LDS stage (the global
    slow path), ':port' and 'www.' forms, IPv6 literals with and without
    ports, empty labels and empty hosts."""
    def label(lo=1, hi=12):
        k = int(rng.integers(lo, hi + 1))
        return "".join(chr(97 + int(c)) for c in rng.integers(0, 26, k))
    keys = set()
    while len(keys) < 300:
        depth = int(rng.integers(1, 12))
        keys.add(".".join(label(1, 30 if rng.random() < 0.2 else 8) for _ in range(depth)))
    keys = sorted(keys)
    keys += ["*", "", "com", "a.b.c.d.e.f.g.h.i.j.k", "x" * 47, "y" * 48, "z" * 49, "w" * 200]
    groups = []
    for i, k in enumerate(keys):
        a = {"host": k}
        if rng.random() < 0.15:
            a["port"] = int(rng.choice([80, 443, 8080]))
        groups.append(({} if rng.random() < 0.8 else {"host": keys[(i + 1) % len(keys)]}, a))
    names = []
    for _ in range(n):
        r = rng.random()
        base = keys[int(rng.integers(0, len(keys)))]
        if r < 0.3:
            h = base
        elif r < 0.6:
            h = ".".join(label() for _ in range(int(rng.integers(1, 9)))) + "." + base
        elif r < 0.7:
            h = label(60, 250)                                   # long, no dots
        elif r < 0.8:
            h = ".".join(label(1, 3) for _ in range(int(rng.integers(8, 40))))
        else:
            h = rng.choice(["[::1]", "::1", "fe80::1:2", "1.2.3.4", "www.", "www", ".", "..",
                            "a..b", "", ":", "www.:80", "[::1]:8080", "::ffff:1.2.3.4",
                            "w" * 200, "x" * 47 + ".y", "." + base])
        if rng.random() < 0.25:
            h = ("www." if rng.random() < 0.5 else "") + h + ":" + str(int(rng.integers(0, 70000)))
        names.append(str(h).encode())
    return groups, names


def gen_frames(rng, n):
    """VXLAN payloads (layer 0) covering the vpacket parse chain: IPv4 and
    IPv6 over Ethernet with TCP (with valid, malformed and throwing options),
    UDP, ICMP/ICMPv6, IPv4 options, IPv6 extension headers (including the
    looping chain), ARP of every size relation, other ether types, wrong
    versions / lengths, and truncation at every offset."""
    import numpy as np

    def rb(k):
        return bytes(rng.integers(0, 256, k).astype(np.uint8))

    def tcp(opts=b""):
        pad = (-len(opts)) % 4
        opts += bytes(pad)
        doff = 20 + len(opts)
        flags = bytes([(doff // 4) << 4, int(rng.integers(0, 64))])
        return rb(4) + rb(8) + flags + rb(6) + opts + rb(int(rng.integers(0, 40)))

    def options():
        r = rng.random()
        if r < 0.3:
            return b""
        if r < 0.5:     # typical SYN options
            return bytes([2, 4, 5, 180, 1, 3, 3, 6, 1, 1, 8, 10]) + rb(8) + bytes([4, 2, 0, 0])
        if r < 0.6:
            return bytes([0]) + rb(3)                       # END first
        if r < 0.7:
            return bytes([8, int(rng.integers(0, 2))]) + rb(2)   # length 0/1: throws
        if r < 0.8:
            return bytes([2, 3, 0, 0])                      # MSS of the wrong length
        if r < 0.85:
            return bytes([3, 4, 0, 0])                      # window scale of the wrong length
        if r < 0.9:
            return bytes([9, 40]) + rb(2)                   # longer than data offset
        return rb(int(rng.integers(1, 20)))

    def ipv4(payload, proto):
        ihl = 5 if rng.random() < 0.8 else int(rng.integers(5, 8))
        hdr_opts = rb(4 * (ihl - 5))
        total = 4 * ihl + len(payload)
        if rng.random() < 0.05:
            total += int(rng.integers(-3, 4))
        ver = 4 if rng.random() < 0.95 else int(rng.integers(0, 16))
        h = bytes([(ver << 4) | ihl, 0, (total >> 8) & 255, total & 255]) + rb(4) + \
            bytes([64, proto]) + rb(2) + rb(8) + hdr_opts
        return h + payload

    def ipv6(payload, proto):
        body = payload
        nh = proto
        r = rng.random()
        if r < 0.2:                                       # one extension header
            hl = int(rng.integers(0, 12))
            nxt = proto if rng.random() < 0.85 else int(rng.choice([0, 43, 60]))
            body = bytes([nxt, hl]) + rb(6 + hl) + payload
            nh = int(rng.choice([0, 43, 44, 60]))
        elif r < 0.25:
            nh = 59
            body = b"" if rng.random() < 0.5 else rb(4)
        plen = len(body)
        if rng.random() < 0.05:
            plen = 0 if rng.random() < 0.5 else plen + 1
        ver = 6 if rng.random() < 0.95 else int(rng.integers(0, 16))
        return bytes([(ver << 4), 0, 0, 0, (plen >> 8) & 255, plen & 255, nh, 64]) + rb(32) + body

    def l4(v6):
        r = rng.random()
        if r < 0.6:
            return 6, tcp(options())
        if r < 0.8:
            return 17, rb(int(rng.integers(8, 40)))
        if r < 0.95:
            return (58 if v6 and rng.random() < 0.7 else 1), rb(int(rng.integers(4, 40)))
        return int(rng.integers(0, 256)), rb(int(rng.integers(0, 30)))

    frames = []
    for _ in range(n):
        r = rng.random()
        eth = rb(12)
        if r < 0.45:
            p, pl = l4(False)
            l3 = b"\x08\x00" + ipv4(pl, p)
        elif r < 0.75:
            p, pl = l4(True)
            l3 = b"\x86\xdd" + ipv6(pl, p)
        elif r < 0.85:
            hs, ps = int(rng.integers(0, 9)), int(rng.integers(0, 17))
            body = bytes([0, 1, 8, 0, hs, ps]) + rb(2) + rb(2 * hs + 2 * ps)
            if rng.random() < 0.3:
                body = body[:int(rng.integers(0, len(body) + 1))] + rb(int(rng.integers(0, 3)))
            l3 = b"\x08\x06" + body
        elif r < 0.9:
            l3 = rb(2) + rb(int(rng.integers(0, 60)))
        else:
            l3 = rb(int(rng.integers(0, 80)))
        frame = bytes([0x08, 0, 0, 0]) + rb(3) + b"\0" + eth + l3
        if rng.random() < 0.1:
            frame = frame[:int(rng.integers(0, len(frame) + 1))]
        frames.append(frame)
    return frames


# ---- traffic-mirror filters (vmirror/FilterConfig.java) ----
MACS = ["0a:00:27:00:00:%02x" % i for i in range(6)] + ["ff:ff:ff:ff:ff:ff", "00:00:00:00:00:00"]
MIRROR_NETS = ["10.0.0.0/8", "10.1.0.0/16", "192.168.0.0/24", "0.0.0.0/0", "10.1.2.3/32",
               "fd00::/8", "fd00:1::/32", "::/0", "::ffff:10.0.0.0/104", "::/96", "::/16",
               "::10.0.0.0/104"]
MIRROR_IPS = ["10.0.0.1", "10.1.2.3", "192.168.0.9", "8.8.8.8", "fd00::1", "fd00:1::5",
              "::ffff:10.1.2.3", "::10.1.2.3", "2001::1", "0.0.0.0"]


def gen_mirror_case(rng, nf, n, origins=("switch", "tcp-lb", "socks5")):
    """Random FilterConfig dicts over small pools (so filters hit), and n
    MirrorData-like items with every null combination.  Returns
    (filters, items) where items is a list of dicts with mac_src/mac_dst
    (str), ip_src/ip_dst (str or None), transport/app (str or None), ports."""
    def pick(xs):
        return xs[int(rng.integers(0, len(xs)))]

    filters = []
    for _ in range(nf):
        f = {"origin": pick(origins), "mirror": int(rng.integers(0, 64 if rng.random() < 0.2 else 6))}
        if rng.random() < 0.5:
            f["mac"] = pick(MACS)
            if rng.random() < 0.5:
                f["mac2"] = pick(MACS)
        if rng.random() < 0.6:
            f["network"] = pick(MIRROR_NETS)
            if rng.random() < 0.5:
                f["network2"] = pick(MIRROR_NETS)
        if rng.random() < 0.5:
            f["transportLayerProtocol"] = pick(["tcp", "udp", "sctp"])
        if rng.random() < 0.5:
            a = int(rng.integers(0, 100))
            f["port"] = [a, a + int(rng.integers(0, 50))]
            if rng.random() < 0.5:
                b = int(rng.integers(0, 100))
                f["port2"] = [b, b + int(rng.integers(0, 50))]
        if rng.random() < 0.3:
            f["applicationLayerProtocol"] = pick(["http", "dns", "h2"])
        filters.append(f)
    items = []
    for _ in range(n):
        r = rng.random()
        it = {"mac_src": pick(MACS), "mac_dst": pick(MACS), "ip_src": None, "ip_dst": None,
              "transport": None, "app": None, "port_src": int(rng.integers(0, 160)),
              "port_dst": int(rng.integers(0, 160))}
        if r > 0.15:
            it["ip_src"] = pick(MIRROR_IPS)
            it["ip_dst"] = pick(MIRROR_IPS) if rng.random() > 0.05 else None
        if r > 0.4:
            it["transport"] = pick(["tcp", "udp", "quic"])
        if r > 0.7:
            it["app"] = pick(["http", "dns", "grpc"])
        items.append(it)
    return filters, items


def mirror_columns(items, id_of, ip_parse):
    """items -> numpy vc_mirror_items columns (strings interned by id_of)."""
    import numpy as np
    n = len(items)
    mac = lambda s: bytes(int(p, 16) for p in s.split(":"))
    cols = {"mac_src": np.frombuffer(b"".join(mac(i["mac_src"]) for i in items), np.uint8).copy(),
            "mac_dst": np.frombuffer(b"".join(mac(i["mac_dst"]) for i in items), np.uint8).copy()}
    for side in ("src", "dst"):
        ln = np.zeros(n, np.uint8)
        ip = np.zeros((n, 16), np.uint8)
        for k, i in enumerate(items):
            if i["ip_" + side] is not None:
                b = ip_parse(i["ip_" + side])
                ln[k] = len(b)
                ip[k, :len(b)] = list(b)
        cols["ip_%s_len" % side] = ln
        cols["ip_" + side] = ip
    cols["transport"] = np.array([id_of(i["transport"]) for i in items], np.int32)
    cols["app"] = np.array([id_of(i["app"]) for i in items], np.int32)
    cols["port_src"] = np.array([i["port_src"] for i in items], np.int32)
    cols["port_dst"] = np.array([i["port_dst"] for i in items], np.int32)
    return cols


def mirror_frames(rng, n):
    """gen_frames VXLAN payloads with their inner MACs drawn from MACS and
    some IPv4 addresses drawn from 10.x so network filters hit."""
    frames = []
    mac = lambda s: bytes(int(p, 16) for p in s.split(":"))
    for f in gen_frames(rng, n):
        f = bytearray(f)
        if len(f) >= 20:
            f[8:14] = mac(MACS[int(rng.integers(0, len(MACS)))])
            f[14:20] = mac(MACS[int(rng.integers(0, len(MACS)))])
        if len(f) >= 42 and f[20:22] == b"\x08\x00" and rng.random() < 0.6:
            f[34:38] = bytes([10, int(rng.integers(0, 3)), 2, 3])
        frames.append(bytes(f))
    return frames


def mirror_v6_frames(rng, n):
    """IPv6 VXLAN frames whose addresses come from the mirror pools'
    families: ::ffff:a.b.c.d and ::a.b.c.d forms (matchIp's lowBitsV6V4
    case of IPv4 filter networks), fd00:: addresses and random ones."""
    out = []
    for _ in range(n):
        addr = []
        for _s in range(2):
            r = rng.random()
            v4 = bytes([10, int(rng.integers(0, 3)), 2, int(rng.integers(0, 5))])
            if r < 0.3:
                a = bytes(10) + b"\xff\xff" + v4
            elif r < 0.5:
                a = bytes(12) + v4
            elif r < 0.6:
                a = bytes(10) + bytes([0xff, 0]) + v4            # not lowBitsV6V4
            elif r < 0.8:
                a = bytes([0xfd, 0, 0, int(rng.integers(0, 2))]) + rng.bytes(12)
            else:
                a = rng.bytes(16)
            addr.append(a)
        l4 = rng.bytes(12) + bytes([5 << 4, 0x18]) + rng.bytes(6)
        ip = bytes([0x60, 0, 0, 0, 0, len(l4), 6, 64]) + addr[0] + addr[1]
        eth = bytes([10, 0, 0x27, 0, 0, 0, 10, 0, 0x27, 0, 0, 1])
        out.append(bytes([8, 0, 0, 0, 0, 0, 1, 0]) + eth + b"\x86\xdd" + ip + l4)
    return out


def http_heads_random(rng, n, hosts, uris):
    """HTTP/1 request heads (bytes) for HttpContext.connectionHint: request
    lines with and without a version, bare-LF lines, Host headers in any
    case with blanks and tabs around key and value, ':port' and 'www.'
    forms, two Host headers, Host-like keys, CR or non-ASCII bytes inside
    the uri or the Host value, keys running across lines, heads cut short
    at any byte and bodies or a second request after the empty line."""
    methods = [b"GET", b"POST", b"PUT", b"HEAD", b"OPTIONS"]
    out = []
    pick = lambda xs: xs[int(rng.integers(0, len(xs)))]
    for _ in range(n):
        eol = b"\r\n" if rng.random() < 0.9 else b"\n"
        u = pick(uris)
        u = b"" if u is None else (u.encode() if isinstance(u, str) else u)
        r = rng.random()
        if r < 0.03:
            u = u + b"\r" + b"x"
        elif r < 0.05:
            u = u + b"\xe4\xff"
        line = pick(methods) + (b"  " if rng.random() < 0.02 else b" ") + u
        line += (b" HTTP/1.1" if rng.random() < 0.85 else b"") + eol
        hdrs = []
        if rng.random() < 0.5:
            hdrs.append(b"User-Agent: curl/8.0")
        if rng.random() < 0.05:
            hdrs.append(b"Hosts: " + pick(hosts).encode())
        if rng.random() < 0.05:
            hdrs.append(b"X-Host: " + pick(hosts).encode())
        nh = 0 if rng.random() < 0.1 else (2 if rng.random() < 0.05 else 1)
        for _ in range(nh):
            key = pick([b"Host", b"host", b"HOST", b"hOsT", b" Host", b"Host\t", b"\tHOST "])
            v = pick(hosts).encode()
            if rng.random() < 0.15:
                v = b"www." + v
            if rng.random() < 0.2:
                v += b":" + str(int(rng.choice([80, 8080, 443]))).encode()
            r = rng.random()
            if r < 0.03:
                v = v[:1] + b"\r" + v[1:]
            elif r < 0.05:
                v = b"\xc3" + v
            pre = pick([b" ", b"", b"  ", b"\t", b" \t"])
            post = pick([b"", b"", b" ", b"\t", b" \r"])
            hdrs.insert(int(rng.integers(0, len(hdrs) + 1)), key + b":" + pre + v + post)
        if rng.random() < 0.02:
            hdrs.insert(0, b"Broken-Line")                  # the key runs to the next ':'
        if rng.random() < 0.3:
            hdrs.append(b"Accept: */*")
        head = line + b"".join(h + eol for h in hdrs) + eol
        r = rng.random()
        if r < 0.08:
            head = head[:int(rng.integers(0, len(head) + 1))]
        elif r < 0.12:
            head += b"GET /second HTTP/1.1" + eol + b"Host: second.example" + eol + eol
        elif r < 0.15:
            head += b"x" * int(rng.integers(1, 64))
        out.append(head)
    return out


def ip_like_strings(rng, n):
    """Strings shaped like IP literals and near misses: hex groups, "::",
    dotted quads (leading zeros, > 255), brackets, stray characters."""
    out = []
    hexd = b"0123456789abcdefABCDEF"

    def group():
        r = rng.random()
        k = int(rng.integers(1, 5)) if r < 0.9 else int(rng.choice([0, 5]))
        g = bytes(rng.choice(np.frombuffer(hexd, np.uint8), k))
        return g + b"g" if rng.random() < 0.02 else g

    def quad():
        return b".".join(str(int(rng.choice([0, 1, 10, 99, 192, 255, 256]))).encode()
                         if rng.random() < 0.97 else b"01" for _ in range(4))

    for _ in range(n):
        if rng.random() < 0.6:                  # address-shaped: 8 groups, or "::" in them
            tail4 = rng.random() < 0.25
            want = 6 if tail4 else 8
            if rng.random() < 0.5:
                gs = [group() for _ in range(want + int(rng.choice([0, 0, 0, -1, 1])))]
                s = b":".join(gs)
            else:
                k = int(rng.integers(0, want))
                a = int(rng.integers(0, k + 1))
                s = b":".join(group() for _ in range(a)) + b"::" + \
                    b":".join(group() for _ in range(k - a))
            if tail4:
                s = s + (b"" if s.endswith(b":") else b":") + quad()
            if rng.random() < 0.1:
                s = b"[" + s + b"]"
            if rng.random() < 0.05:
                s = s + b":" + str(int(rng.integers(0, 70000))).encode()
            out.append(s)
            continue
        parts = []
        for _ in range(int(rng.integers(0, 10))):
            r = rng.random()
            if r < 0.55:
                parts.append(bytes(rng.choice(np.frombuffer(hexd, np.uint8), int(rng.integers(0, 6)))))
            elif r < 0.7:
                parts.append(b"")
            elif r < 0.85:
                parts.append(b".".join(str(int(rng.choice([0, 1, 9, 10, 99, 255, 256, 7]))).encode()
                                       if rng.random() < 0.9 else b"01"
                                       for _ in range(int(rng.integers(3, 6)))))
            else:
                parts.append(bytes(rng.choice(np.frombuffer(b"gz.%x", np.uint8), int(rng.integers(1, 3)))))
        s = b":".join(parts)
        if rng.random() < 0.2:
            s = s.replace(b":", b"::", 1)
        if rng.random() < 0.15:
            s = b"[" + s + b"]"
        if rng.random() < 0.1:
            s = s + b":" + str(int(rng.integers(0, 70000))).encode()
        out.append(s)
    return out

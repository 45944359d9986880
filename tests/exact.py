"""Independent exact checkers for whole-batch parity at the headline sizes.

TEST INFRASTRUCTURE ONLY, like oracle/: nothing under vproxy_amd/ imports
this module.  The oracle (oracle/vc_oracle.c) restates the Java as the Java
runs it -- a linear scan of the rule list per item -- which is exact but
checks only a few thousand of a 16M-64M batch in test time.  The checkers
here restate the same functions by a different algorithm, one that needs a
handful of sorted-array probes per item, so a GPU test can compare EVERY
output of a headline-size batch.  Each is validated against the oracle on
random sets first (tests/test_exact_cpu.py) and shares no code with the
kernels or the table compiler.

- route_first_match_v4 / _v6: RouteTable.lookup (RouteTable.java:44-59)
  returns the first rule in list order whose network contains the address.
  A prefix of length L contains the address iff the two agree on the top L
  bits, so at each length at most one distinct network can contain it: the
  first match is the minimum list index over the lengths of the earliest
  rule whose network equals the address's top L bits.  One key array per
  length, sorted stably (so the earliest rule heads each run of equal keys),
  probed with searchsorted.  This holds for any list order -- it does not
  lean on the shortest-first / longest-prefix argument (R7).
- sg_first_match_v4 / _v6: SecurityGroup.allow (SecurityGroup.java:30-45)
  with SecurityGroupRule.match (SecurityGroupRule.java:27-29): the first rule
  of the protocol's list (TCP for 6, UDP otherwise) whose network contains
  the source and whose [minPort, maxPort] holds the port; allow is that
  rule's bit, defaultAllow when none.  Same per-length probe, then a scan of
  the (short) run of rules sharing the network for the first one whose port
  range holds the port.  IPv4 rules only; an IPv6 source reaches them through
  Network.maskMatch's cases 4/5 (Network.java:246-277): only ::a.b.c.d and
  ::ffff:a.b.c.d (Utils.lowBitsV6V4) can match, on their low 32 bits.
- hint_search_dict: Upstream.searchForGroup (Upstream.java:187-198) over
  host-only hints: Hint.ofHost / formatHost (Hint.java:17-73) and the host
  part of matchLevel (Hint.java:100-160) with the hint-port filter.  A dict
  from merged hint-host to its groups: level 3 = the host itself, level 2 =
  any "."-suffix of it (host.endsWith("." + annoHost)), level 1 = "*"; the
  strict ">" of searchForGroup makes the answer the earliest group of the
  best level.
- HintLevelChecker: searchForGroup with the whole matchLevel -- hint-uri
  levels (prefix / equal / "*", UTF-16 length, cap 1023), port filter,
  host levels -- visiting only the groups a host or uri dict lookup finds.
- CertChecker: SSLContextHolder.choose (SSLContextHolder.java:50-79,
  171-186) -- a plain-name dict and a wildcard-suffix dict, since a "*.S"
  name can only match an SNI through its suffix from the first dot.
- SourceChecker: ServerGroup's source hashing (ServerGroup.java:377-490,
  620-664) as tensor arithmetic: the sdbm hash of the signed address bytes
  per item, and per group a table of the first healthy list position at
  or after each position (the probe), so an item is two gathers.
- DnsChecker: DNSServer.handleRequest's classification (DNSServer.java:
  116-166) -- a dict restatement of Resolver.getHosts' dual-key map
  (Resolver.java:62-153), then HintChecker on the dot-stripped name, then
  the IP-literal / .vproxy.local / recursive tail.
- java_is_ipv6 / java_is_ip_literal: IP.isIpv6 / IP.isIpLiteral
  (IP.java:112-300) as validity predicates over bytes, with the parser's
  quirks (Utils.split keeps empty pieces; parseIpv6LastBits' `4 +
  colonPart` counts a failed colon part as 3), so formatHost's IPv6 branch
  and the DNS IP-literal step need no oracle call.
"""
import re

import numpy as np
import torch

CHUNK = 16 << 20


def _t(x, dev):
    if isinstance(x, torch.Tensor):
        return x.to(dev)
    return torch.from_numpy(np.ascontiguousarray(x)).to(dev)


def _u32(x):
    """any integer tensor holding uint32 bits -> int64 in [0, 2^32)"""
    return x.to(torch.int64) & 0xFFFFFFFF


def _plen_of_masks(mask_words, width):
    """prefix length of each mask (int64 words, top `width` bits), asserting
    every mask is a prefix mask (Network.validNetwork masks are)."""
    m = mask_words.cpu().numpy().astype(np.uint64)
    if width == 32:
        m = m & np.uint64(0xFFFFFFFF)
    plen = np.zeros(len(m), np.int64)
    x = m.copy()
    for _ in range(width):
        plen += (x & np.uint64(1)).astype(np.int64)
        x >>= np.uint64(1)
    full = np.uint64((1 << width) - 1)
    want = np.where(plen == 0, np.uint64(0),
                    (full << (np.uint64(width) - plen.astype(np.uint64))) & full)
    assert np.array_equal(m, want), "non-prefix mask"
    return torch.from_numpy(plen)


class _PerLength:
    """Rules grouped by prefix length: for each length L present, the rules'
    top-L-bit keys sorted stably (earliest rule first within a key), their
    list indices, and the longest run of one key."""

    def __init__(self, net, plen, width, dev):
        self.width = width
        self.levels = []
        idx = torch.arange(len(net), dtype=torch.int64)
        for L in sorted(set(plen.tolist())):
            sel = plen == L
            k = self.key(net[sel], L)
            order = torch.argsort(k, stable=True)
            k, ridx = k[order], idx[sel][order]
            run = int(torch.unique_consecutive(k, return_counts=True)[1].max())
            self.levels.append((L, k.to(dev), ridx.to(dev), run))

    def key(self, x, L):
        if L == 0:
            return torch.zeros_like(x)
        # arithmetic shift of the signed word: equal top-L bits <=> equal keys,
        # and the order is consistent on both sides of the probe
        return x >> (self.width - L)


def _first_match(levels, q, nrules, port=None, plo=None, phi=None, valid=None):
    """min list index over the lengths of a rule whose key equals q's key
    (and, with `port`, whose port range holds it); nrules when none."""
    best = torch.full(q.shape, nrules, dtype=torch.int64, device=q.device)
    for L, k, ridx, run in levels.levels:
        qk = levels.key(q, L)
        pos = torch.searchsorted(k, qk)
        for m in range(run if port is not None else 1):
            c = pos + m
            inr = c < len(k)
            c = c.clamp(max=len(k) - 1)
            ok = inr & (k[c] == qk)
            r = ridx[c]
            if port is not None:
                ok &= (plo[r] <= port) & (port <= phi[r])
            if valid is not None:
                ok &= valid
            best = torch.where(ok, torch.minimum(best, r), best)
    return best


# ---------------------------------------------------------------------------
# RouteTable.lookup
# ---------------------------------------------------------------------------
def _net_words(nets, family):
    ip = np.ascontiguousarray(nets["ip"])
    mk = np.ascontiguousarray(nets["mask"])
    if family == 4:
        assert np.all(nets["ip_len"] == 4) and np.all(nets["mask_len"] == 4)
        w = lambda a: torch.from_numpy(a[:, :4].copy().view(">u4").reshape(-1).astype(np.int64))
        return w(ip), w(mk)
    assert np.all(nets["ip_len"] == 16)
    # Network.parseMask gives 4 mask bytes up to /32: Network.maskMatch's case
    # 1 compares those bytes only, which is the same prefix test
    w = lambda a: torch.from_numpy(a[:, :8].copy().view(">i8").reshape(-1).astype(np.int64))
    lo = lambda a: a[:, 8:].copy().view(">u8").reshape(-1)
    full = np.zeros((len(mk), 16), np.uint8)
    full[:, :mk.shape[1]] = mk
    full[nets["mask_len"] == 4, 4:] = 0
    assert np.all(lo(full) == 0) and np.all(lo(ip) == 0), "IPv6 prefixes longer than /64"
    return w(ip), w(full)


class RouteChecker:
    """RouteTable.lookup (RouteTable.java:44-59) over one family's rule list
    (NET_DT rows in list order)."""

    def __init__(self, nets, family, dev):
        self.family, self.dev, self.n = family, dev, len(nets)
        width = 32 if family == 4 else 64
        net, mk = _net_words(nets, family)
        plen = _plen_of_masks(mk, width)
        self.levels = _PerLength(net, plen, width, dev)

    def __call__(self, dst):
        """dst: v4 -> uint32 bits in any integer dtype [n]; v6 -> uint8 [n, 16].
        Returns int32 list indices, -1 for null."""
        out = []
        for s in range(0, len(dst), CHUNK):
            d = _t(dst[s:s + CHUNK], self.dev)
            if self.family == 4:
                q = _u32(d)
            else:
                q = _be64(d[:, :8])
            b = _first_match(self.levels, q, self.n)
            out.append(torch.where(b == self.n, -1, b).to(torch.int32))
        return torch.cat(out) if out else torch.zeros(0, dtype=torch.int32, device=self.dev)


def _be64(b):
    """uint8 [n, 8] big-endian -> int64 [n] (two's complement bits)"""
    b = b.to(torch.int64)
    x = torch.zeros(b.shape[0], dtype=torch.int64, device=b.device)
    for i in range(8):
        x = (x << 8) | b[:, i]
    return x


# ---------------------------------------------------------------------------
# SecurityGroup.allow
# ---------------------------------------------------------------------------
class AclChecker:
    """SecurityGroup.allow (SecurityGroup.java:30-45) over IPv4 rule lists
    (workloads.RULE_DT rows in list order)."""

    def __init__(self, tcp, udp, default_allow, dev):
        self.dev, self.dflt = dev, 1 if default_allow else 0
        self.lists = []
        for rules in (tcp, udp):
            net, mk = _net_words(rules["net"], 4)
            plen = _plen_of_masks(mk, 32)
            self.lists.append(dict(
                n=len(rules), levels=_PerLength(net, plen, 32, dev),
                lo=_t(rules["min_port"].astype(np.int64), dev),
                hi=_t(rules["max_port"].astype(np.int64), dev),
                allow=_t(rules["allow"].astype(np.int64), dev)))

    def _one(self, proto, src, port, valid):
        idx = torch.full(src.shape, -1, dtype=torch.int64, device=self.dev)
        allow = torch.full(src.shape, self.dflt, dtype=torch.int64, device=self.dev)
        is_tcp = proto.to(torch.int64) == 6
        for L, sel in zip(self.lists, (is_tcp, ~is_tcp)):
            if L["n"] == 0:
                continue
            b = _first_match(L["levels"], src, L["n"], port, L["lo"], L["hi"], valid)
            hit = sel & (b < L["n"])
            bc = b.clamp(max=L["n"] - 1)
            idx = torch.where(hit, b, idx)
            allow = torch.where(hit, L["allow"][bc], allow)
        return idx.to(torch.int32), allow.to(torch.uint8)

    def v4(self, proto, src4, port):
        """proto u8, src uint32 bits, port uint16 bits -> (rule idx int32, allow u8)"""
        outs = []
        for s in range(0, len(src4), CHUNK):
            p = _t(proto[s:s + CHUNK], self.dev)
            a = _u32(_t(src4[s:s + CHUNK], self.dev))
            q = _t(port[s:s + CHUNK], self.dev).to(torch.int64) & 0xFFFF
            outs.append(self._one(p, a, q, None))
        return tuple(torch.cat(x) for x in zip(*outs))

    def v6(self, proto, src6, port):
        """IPv6 sources against the IPv4 rules: Network.maskMatch cases 4/5
        (Network.java:246-277) compare the last four bytes, then
        Utils.lowBitsV6V4(ip, 11, 10) (Utils.java:122-133) requires bytes
        0-9 zero and bytes 10-11 both 0x00 or both 0xFF."""
        outs = []
        for s in range(0, len(port), CHUNK):
            p = _t(proto[s:s + CHUNK], self.dev)
            b = _t(src6[s:s + CHUNK], self.dev).to(torch.int64)
            head0 = (b[:, :10] == 0).all(dim=1)
            b10, b11 = b[:, 10], b[:, 11]
            ok = head0 & (((b10 == 0) & (b11 == 0)) | ((b10 == 255) & (b11 == 255)))
            a = (b[:, 12] << 24) | (b[:, 13] << 16) | (b[:, 14] << 8) | b[:, 15]
            q = _t(port[s:s + CHUNK], self.dev).to(torch.int64) & 0xFFFF
            outs.append(self._one(p, a, q, ok))
        return tuple(torch.cat(x) for x in zip(*outs))


# ---------------------------------------------------------------------------
# Upstream.searchForGroup over host-only hints
# ---------------------------------------------------------------------------
_INT = re.compile(r"[+-]?[0-9]+\Z")


def _java_int(v):
    """Integer.parseInt, with Annotations' failure -> 0 (Annotations.java:45-58)"""
    if v is None:
        return 0
    if isinstance(v, int):
        return v
    if not _INT.match(v):
        return 0
    x = int(v)
    return x if -2**31 <= x < 2**31 else 0


def _anno(a, k):
    return a.get("vproxy/hint-" + k, a.get(k))


_HEX = frozenset(b"0123456789abcdefABCDEF")


def _v4_ok(s, from_idx, cap):
    """IP.parseIpv4String(s, bytes, fromIdx) succeeds (IP.java:129-155):
    three dots, four pieces of 1-3 ASCII digits, no leading zero, <= 255,
    every piece inside the byte array."""
    if s.count(b".") != 3:
        return False
    for i, p in enumerate(s.split(b".")):
        if from_idx + i >= cap or not 1 <= len(p) <= 3 or not p.isdigit():
            return False
        if (p[:1] == b"0" and len(p) > 1) or int(p) > 255:
            return False
    return True


def _colon_part(s, from_idx):
    """IP.parseIpv6ColonPart (IP.java:200-248): 2 x its pieces, or -1.
    None (Java null) and "" consume nothing."""
    if not s:
        return 0
    if from_idx < 0:
        return -1
    parts = s.split(b":")
    for i, f in enumerate(parts):
        if from_idx + 2 * i >= 16 or not 1 <= len(f) <= 4 or any(c not in _HEX for c in f):
            return -1
    return 2 * len(parts)


def _last_bits(s):
    """IP.parseIpv6LastBits (IP.java:251-269): the bytes the part after
    "::" (or the whole string) consumes, or -1; a dotted tail is an IPv4
    quad, and `4 + colonPart` turns a failed colon part before it into 3."""
    dot = s.find(b".")
    if dot == -1:
        return _colon_part(s, 16 - 2 * (s.count(b":") + 1))
    k = s.rfind(b":", 0, dot)
    if k == -1:
        return 4 if _v4_ok(s, 12, 16) else -1
    if not _v4_ok(s[k + 1:], 12, 16):
        return -1
    head = s[:k]
    return 4 + _colon_part(head, 16 - 4 - 2 * (head.count(b":") + 1))


def java_is_ipv6(s):
    """IP.isIpv6 = IP.parseIpv6String(s) != null (IP.java:158-197) on bytes."""
    if b":" not in s:
        return False                       # one piece: never 16 bytes
    if s.startswith(b"[") and s.endswith(b"]"):
        s = s[1:-1]
    if s.count(b"::") > 1:
        return False
    k = s.find(b"::")
    head, tail = (None, s) if k == -1 else (s[:k], s[k + 2:])
    a = _colon_part(head, 0)
    if a == -1:
        return False
    b = _last_bits(tail)
    if b == -1:
        return False
    return a + b < 16 if k != -1 else a + b == 16


def java_is_ip_literal(s):
    """IP.isIpLiteral (IP.java:271-300): an IPv6 string, or an IPv4 quad."""
    return java_is_ipv6(s) or _v4_ok(s, 0, 4)


class HintChecker:
    """searchForGroup for hints built by Hint.ofHost / ofHostPort."""

    def __init__(self, groups):
        self.by_host = {}          # merged hint-host bytes -> [(group index, hint-port)]
        for i, (ha, ga) in enumerate(groups):
            host = None
            port = 0
            for a in (ha or {}, ga or {}):   # Upstream.java:191: handle first
                h = _anno(a, "host")
                if host is None and h is not None:
                    host = h.encode() if isinstance(h, str) else bytes(h)
                if port == 0:
                    port = _java_int(_anno(a, "port"))
            if host is not None:
                self.by_host.setdefault(host, []).append((i, port))

    def _first(self, key, port):
        for i, p in self.by_host.get(key, ()):
            if port == 0 or p == 0 or p == port:      # Hint.java:106-108
                return i
        return -1

    @staticmethod
    def format_host(s):
        """Hint.formatHost (Hint.java:57-73): an IPv6 string or a name
        without ':' unchanged, else the part before the first ':' without
        one leading "www." (empty -> null)."""
        c = s.find(b":")
        if c == -1 or java_is_ipv6(s):
            return s
        h = s[:c]
        if h.startswith(b"www."):
            h = h[4:]
        return h if h else None

    def __call__(self, name, port=0):
        host = self.format_host(name)
        if host is None:
            return -1
        g = self._first(host, port)
        if g >= 0:
            return g                               # level 3 beats any other
        best = -1
        d = host.find(b".")
        while d != -1:                             # every "." + annoHost suffix
            g = self._first(host[d + 1:], port)
            if g >= 0 and (best < 0 or g < best):
                best = g
            d = host.find(b".", d + 1)
        if best >= 0:
            return best
        return self._first(b"*", port)

    def batch(self, blob, off, ports=None):
        blob = bytes(np.asarray(blob, np.uint8))
        off = np.asarray(off, np.int64)
        out = np.empty(len(off) - 1, np.int32)
        for i in range(len(out)):
            out[i] = self(blob[off[i]:off[i + 1]], 0 if ports is None else int(ports[i]))
        return out


# ---------------------------------------------------------------------------
# Upstream.searchForGroup over full hints (host, port, uri)
# ---------------------------------------------------------------------------
def format_uri(u):
    """Hint.formatUri (Hint.java:75-90): cut at the first '?', "/" stays,
    else one trailing '/' goes."""
    if u is None:
        return None
    q = u.find(b"?")
    if q != -1:
        u = u[:q]
    if u == b"/":
        return u
    return u[:-1] if u.endswith(b"/") else u


class HintLevelChecker:
    """Upstream.searchForGroup (Upstream.java:187-198) with the whole of
    Hint.matchLevel (Hint.java:100-160): level = hostLevel << 10 + uriLevel,
    the port filter, strict '>' over the handle list.  Only groups that can
    score above 0 are considered:
    - host candidates, whose merged hint-host equals the formatted host, one
      of its dot-suffixes or "*" (host dict): level computed exactly;
    - uri candidates, whose merged hint-uri is the uri, a prefix of it or
      "*" (uri dict, every prefix probed).  Scored as if hostLevel were 0,
      all groups of one hint-uri share one level, so only the earliest one
      the port filter lets through counts (precomputed per uri and port).
      A group that also matches the host scores >= 1024 on the host side,
      above any uri-only level (<= 1023), so the underestimate never wins.
    Any other group scores 0.  ASCII strings (UTF-16 length = byte length)."""

    def __init__(self, groups):
        self.g = []                 # merged (host, port, uri) per handle
        self.by_host, self.by_uri = {}, {}
        for i, (ha, ga) in enumerate(groups):
            host, port, uri = None, 0, None
            for a in (ha or {}, ga or {}):       # handle annotations first (Upstream.java:191)
                h, u = _anno(a, "host"), _anno(a, "uri")
                if host is None and h is not None:
                    host = h.encode() if isinstance(h, str) else bytes(h)
                if port == 0:
                    port = _java_int(_anno(a, "port"))
                if uri is None and u is not None:
                    uri = u.encode() if isinstance(u, str) else bytes(u)
            for x in (host, uri):
                assert x is None or max(x, default=0) < 0x80, "checker covers ASCII annotations"
            self.g.append((host, port, uri))
            if host is not None:
                self.by_host.setdefault(host, []).append(i)
            if uri is not None:
                # per hint-uri: (earliest handle with no hint-port, earliest
                # handle per hint-port); indices ascend, so setdefault keeps
                # the first
                e = self.by_uri.setdefault(uri, [None, {}, i])     # [2]: earliest of all
                if port == 0:
                    if e[0] is None:
                        e[0] = i
                else:
                    e[1].setdefault(port, i)

    def level(self, i, host, port, uri):
        """Hint.matchLevel of handle i (Hint.java:100-160)."""
        H, P, U = self.g[i]
        if H is None and P == 0 and U is None:
            return 0
        if port != 0 and P != 0 and port != P:
            return 0
        hl = 0
        if H is not None and host is not None:
            if host == H:
                hl = 3
            elif host.endswith(b"." + H):
                hl = 2
            elif H == b"*":
                hl = 1
        ul = 0
        if U is not None and uri is not None:
            if uri == U:
                ul = len(uri) + 1
            elif uri.startswith(U):
                ul = len(U) + 1
            elif U == b"*":
                ul = 1
        return (hl << 10) + min(ul, 1023)

    def __call__(self, name, port=0, uri=None):
        """Hint.ofHostPortUri(name, port, uri) (name / uri may be None)."""
        host = None if name is None else HintChecker.format_host(name)
        uri = format_uri(uri)
        best, lv = -1, 0

        def take(i, l):
            nonlocal best, lv
            if l > lv or (l == lv and l > 0 and i < best):
                best, lv = i, l

        if host is not None:
            cand = set(self.by_host.get(host, ()))
            d = host.find(b".")
            while d != -1:
                cand.update(self.by_host.get(host[d + 1:], ()))
                d = host.find(b".", d + 1)
            cand.update(self.by_host.get(b"*", ()))
            for i in cand:
                take(i, self.level(i, host, port, uri))
        if uri is not None:
            keys = {uri[:k] for k in range(len(uri) + 1)} | {b"*"}
            for U in keys:
                e = self.by_uri.get(U)
                if e is None:
                    continue
                if uri == U:
                    ul = len(uri) + 1
                elif uri.startswith(U):
                    ul = len(U) + 1
                else:                                   # U == "*"
                    ul = 1
                ul = min(ul, 1023)
                p0, per, first = e
                if port == 0:                           # every hint-port passes
                    take(first, ul)
                else:
                    idx = [x for x in (p0, per.get(port)) if x is not None]
                    if idx:
                        take(min(idx), ul)
        return best

    def table(self, names, uris):
        """searchForGroup(Hint.ofHostUri(name, uri)) -- port 0, what
        HttpContext.connectionHint sends (HttpContext.java:55-71) -- for
        every pair: int32 [len(names), len(uris)] (a uri may be None).  With
        port 0 no hint-port excludes a group, so level(g) = hl(g) << 10 +
        ul(g) with ul <= 1023: when the name's top host level L is > 0 the
        winner is among the groups at L -- the largest ul, then the lowest
        index -- and otherwise it is the uri-only argmax, one per uri.  The
        per-uri ul of every group is a vector, so a batch of tens of
        millions of hints is a gather from this table."""
        ng = len(self.g)
        assert ng < (1 << 20)
        furis = [format_uri(u) for u in uris]
        members = {}
        for i, (H, P, U) in enumerate(self.g):
            if U is not None:
                members.setdefault(U, []).append(i)
        members = {U: np.array(m, np.int64) for U, m in members.items()}
        ul = np.zeros((len(uris), ng), np.int64)
        for k, u in enumerate(furis):
            if u is None:
                continue
            for U, m in members.items():
                if u == U:
                    lvl = len(u) + 1
                elif u.startswith(U):
                    lvl = len(U) + 1
                elif U == b"*":
                    lvl = 1
                else:
                    continue
                ul[k, m] = min(lvl, 1023)
        uonly = np.where(ul.max(1) > 0, ul.argmax(1), -1)     # argmax: the lowest index of the max
        starts, flat = [0], []
        for name in names:
            host = HintChecker.format_host(name)
            top = []
            if host is not None:
                cand = set(self.by_host.get(host, ()))
                d = host.find(b".")
                while d != -1:
                    cand.update(self.by_host.get(host[d + 1:], ()))
                    d = host.find(b".", d + 1)
                cand.update(self.by_host.get(b"*", ()))
                lv = {i: self.level(i, host, 0, None) >> 10 for i in cand}
                L = max(lv.values(), default=0)
                if L > 0:
                    top = sorted(i for i, v in lv.items() if v == L)
            flat.extend(top)
            starts.append(len(flat))
        flat = np.array(flat, np.int64)
        starts = np.array(starts, np.int64)
        has = starts[1:] > starts[:-1]
        out = np.empty((len(names), len(uris)), np.int32)
        low = (1 << 20) - 1
        for k in range(len(uris)):
            if flat.size:
                key = (ul[k, flat] << 20) + (low - flat)
                best = np.maximum.reduceat(key, starts[:-1][has])
                out[has, k] = low - (best & low)
            out[~has, k] = uonly[k]
        return out


# ---------------------------------------------------------------------------
# DNSServer.handleRequest classification
# ---------------------------------------------------------------------------
DNS_HOSTS, DNS_GROUP, DNS_IP_LITERAL, DNS_INTERNAL, DNS_RECURSIVE = 1, 2, 3, 4, 5   # VC_DNS_*


def hosts_map(text, is_ip):
    """Resolver.getHosts (Resolver.java:62-153) restated with Python's str
    and dict: per line (\\n, \\r or \\r\\n), cut at the first '#', skip blank
    lines, split on ' ' / '\\t' and drop empty tokens; the first token must
    be an IP literal (`is_ip`: IP.parseIpString != null), and the line's
    entry index counts the lines that pass.  Each name d1 adds d1 and its
    dot-twin d2 (trailing '.' removed or added) unless either is already a
    key -- the first line naming a host wins (:130-141).  Returns {name bytes: entry index}."""
    if isinstance(text, bytes):
        text = text.decode("latin-1")
    ret, entry = {}, 0
    for line in re.split(r"\r\n|\r|\n", text):
        if "#" in line:
            line = line[:line.index("#")]
        if not line.strip(" \t\n\x0b\f\r\x1c\x1d\x1e\x1f"):    # String.isBlank (ASCII)
            continue
        toks = [s.strip("".join(chr(c) for c in range(33))) for s in re.split(r"[ \t]", line)]
        toks = [s for s in toks if s]
        if len(toks) < 2 or not is_ip(toks[0].encode("latin-1")):
            continue
        for d1 in toks[1:]:
            d2 = d1[:-1] if d1.endswith(".") else d1 + "."
            k1, k2 = d1.encode("latin-1"), d2.encode("latin-1")
            if k1 in ret or k2 in ret:
                continue
            ret[k1] = entry
            ret[k2] = entry
        entry += 1
    return ret


class DnsChecker:
    """DNSServer.handleRequest's classification of one A/AAAA/SRV qname
    (DNSServer.java:116-166): the hosts map on the raw qname (trailing dot
    included; both key forms, Resolver.java:130-141), else strip one
    trailing dot and Upstream.searchForGroup(Hint.ofHost(domain)) through
    HintChecker, else IP.isIpLiteral -> the literal's family, else
    `.vproxy.local` -> internal, else recursive.  `is_ip`: the IP-literal
    predicate (IP.java:112-300), java_is_ip_literal unless given."""

    def __init__(self, hosts_text, groups, is_ip=None):
        self.is_ip = is_ip or java_is_ip_literal
        self.hosts = hosts_map(hosts_text, self.is_ip) if hosts_text else {}
        self.hint = HintChecker(groups)

    def __call__(self, q):
        assert max(q, default=0) < 0x80, "checker covers ASCII qnames"
        v = self.hosts.get(q)
        if v is not None:
            return DNS_HOSTS, v
        d = q[:-1] if q.endswith(b".") else q
        g = self.hint(d)
        if g >= 0:
            return DNS_GROUP, g
        if self.is_ip(d):
            return DNS_IP_LITERAL, 6 if b":" in d else 4
        if d.endswith(b".vproxy.local"):
            return DNS_INTERNAL, 0
        return DNS_RECURSIVE, 0

    def batch(self, blob, off):
        blob = bytes(np.asarray(blob, np.uint8))
        off = np.asarray(off, np.int64)
        kind = np.empty(len(off) - 1, np.uint8)
        val = np.empty(len(off) - 1, np.int32)
        for i in range(len(kind)):
            kind[i], val[i] = self(blob[off[i]:off[i + 1]])
        return kind, val


# ---------------------------------------------------------------------------
# SSLContextHolder.choose (SNI -> certificate holder)
# ---------------------------------------------------------------------------
class CertChecker:
    """SSLContextHolder.choose(sni) (SSLContextHolder.java:50-79) with
    compare (:171-186): one holder -> it; none -> null (-1); a null SNI or
    no match -> the first holder; else the first holder (add() order) with
    a name equal to the SNI, or a "*.S" name where the SNI ends with ".S"
    and the rest before it is non-empty with no '.': that rest ends at the
    SNI's first dot, so one dict probe on the SNI and one on its suffix
    from the first dot cover every name."""

    def __init__(self, holders):
        self.n = len(holders)
        self.plain, self.wild = {}, {}
        for h, names in enumerate(holders):
            for nm in names:
                b = nm.encode() if isinstance(nm, str) else bytes(nm)
                if b.startswith(b"*."):
                    self.wild.setdefault(b[1:], h)        # ".S", first holder wins
                else:
                    self.plain.setdefault(b, h)

    def __call__(self, sni):
        if self.n == 1:
            return 0
        if self.n == 0:
            return -1
        if sni is None:
            return 0
        best = self.plain.get(sni, self.n)
        d = sni.find(b".")
        if d >= 1:
            best = min(best, self.wild.get(sni[d:], self.n))
        return best if best < self.n else 0

    def batch(self, blob, off, null=None):
        blob = bytes(np.asarray(blob, np.uint8))
        off = np.asarray(off, np.int64)
        out = np.empty(len(off) - 1, np.int32)
        for i in range(len(out)):
            out[i] = self(None if null is not None and null[i] else blob[off[i]:off[i + 1]])
        return out


# ---------------------------------------------------------------------------
# ServerGroup source hashing (method source)
# ---------------------------------------------------------------------------
def _signed_key(ip):
    return tuple(b - 256 if b >= 128 else b for b in ip)


class SourceChecker:
    """ServerGroup.next(source) for method source over IPv4 clients
    (ServerGroup.java:422-490): the group's sourceReset list (:620-664:
    servers with weight > 0 of the view, sorted stably by address length,
    then signed address bytes, then port), hash = Math.abs(sdbm of the
    client's signed address bytes) (:387-397, Math.abs(MIN_VALUE) taken as
    0 as the oracle does), idx = hash % size, then forward (wrapping) to the
    first healthy server; none healthy -> null (-1).  Results are indices
    into the group's own server list, as the library returns them.
    groups: list of server lists [(ip bytes, port, weight, healthy)]."""

    def __init__(self, groups, dev, view=0):
        base, size, nxt = [], [], []
        for g in groups:
            keep = [i for i, (ip, port, w, h) in enumerate(g)
                    if w > 0 and (view == 0 or (view == 4) == (len(ip) == 4))]
            order = sorted(keep, key=lambda i: (len(g[i][0]), _signed_key(g[i][0]), g[i][1]))
            base.append(len(nxt))
            size.append(len(order))
            for p in range(len(order)):       # first healthy position at or after p
                r = -1
                for q in range(len(order)):
                    c = order[(p + q) % len(order)]
                    if g[c][3]:
                        r = c
                        break
                nxt.append(r)
        T = lambda x: torch.tensor(x, dtype=torch.int64, device=dev)
        self.base, self.size, self.nxt = T(base), T(size), T(nxt if nxt else [-1])
        self.dev = dev

    @staticmethod
    def hash_v4(src):
        """Math.abs(sdbm(bytes)) of uint32 v4 keys (int64 tensor), Java int math"""
        x = _u32(src)
        h = torch.zeros_like(x)
        for sh in (24, 16, 8, 0):
            b = (x >> sh) & 0xFF
            b = torch.where(b >= 128, b - 256, b)
            h = (b + (h << 6) + (h << 16) - h) & 0xFFFFFFFF
        h = torch.where(h >= 2**31, h - 2**32, h)            # to Java int
        return torch.where(h == -2**31, torch.zeros_like(h), h.abs())

    def v4(self, grp, src):
        outs = []
        for s in range(0, len(grp), CHUNK):
            g = _t(grp[s:s + CHUNK], self.dev).long()
            h = self.hash_v4(_t(src[s:s + CHUNK], self.dev))
            sz = self.size[g]
            idx = self.base[g] + h % sz.clamp(min=1)
            outs.append(torch.where(sz > 0, self.nxt[idx.clamp(max=len(self.nxt) - 1)],
                                    torch.full_like(g, -1)).to(torch.int32))
        return torch.cat(outs)

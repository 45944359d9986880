"""DNS wire-format builder: synthetic DNS datagrams for the vc_dns_datagrams
tests and the `dnsd` benchmark (no product path uses it).

Follows the layout Formatter.format writes (base/src/main/java/vproxybase/dns/
Formatter.java:16-160): a 12-byte header, questions (name, qtype, qclass),
then answer / authority / additional resources (name, type, class, ttl,
rdlen, rdata).  Names are label sequences ending in a zero byte
(formatDomainName); `ptr` appends a compression pointer instead of the zero
byte, which Formatter never writes but Formatter.parseDomainName reads.
"""
import struct

A, CNAME, PTR, TXT, AAAA, SRV, OPT, MX, ANY = 1, 5, 12, 16, 28, 33, 41, 15, 255
IN, CH, HS, NONE_CLASS, ANY_CLASS = 1, 3, 4, 254, 255


def name(domain, ptr=None):
    """formatDomainName(domain) -- labels of the dotted name, then 0; with
    ptr, a 2-byte pointer (0xC000 | ptr) replaces the final zero byte."""
    if isinstance(domain, str):
        domain = domain.encode()
    out = b""
    for lab in [x for x in domain.split(b".") if x] if domain not in (b"", b".") else []:
        out += bytes([len(lab)]) + lab
    if ptr is None:
        return out + b"\0"
    return out + struct.pack(">H", 0xC000 | ptr)


def header(qd=1, an=0, ns=0, ar=0, ident=0x1234, response=False, opcode=0, aa=False, tc=False,
           rd=True, ra=False, rcode=0):
    """Formatter.formatHeader (Formatter.java:65-96)."""
    b2 = (0x80 if response else 0) | ((opcode & 15) << 3) | (4 if aa else 0) | \
        (2 if tc else 0) | (1 if rd else 0)
    b3 = (0x80 if ra else 0) | (rcode & 15)
    return struct.pack(">HBBHHHH", ident, b2, b3, qd, an, ns, ar)


def question(qname, qtype=A, qclass=IN):
    """Formatter.formatQuestion (Formatter.java:139-145) of a dotted qname."""
    return name(qname) + struct.pack(">HH", qtype, qclass)


def raw_question(wire_name, qtype=A, qclass=IN):
    """A question whose name is given in wire form (labels, pointers)."""
    return bytes(wire_name) + struct.pack(">HH", qtype, qclass)


def resource(rname, rtype, rdata, rclass=IN, ttl=600):
    """Formatter.formatResource (Formatter.java:147-160)."""
    n = rname if isinstance(rname, (bytes, bytearray)) else name(rname)
    return bytes(n) + struct.pack(">HHiH", rtype, rclass, ttl, len(rdata)) + bytes(rdata)


def txt(*texts):
    """TXT.toByteArray: formatString per text."""
    out = b""
    for t in texts:
        t = t.encode() if isinstance(t, str) else t
        out += bytes([len(t)]) + t
    return out


def query(questions, extra=b"", an=0, ns=0, ar=0, **hdr):
    """A query datagram: header + the given (qname, qtype[, qclass]) questions."""
    body = b"".join(question(*q) for q in questions)
    return header(qd=len(questions), an=an, ns=ns, ar=ar, **hdr) + body + extra


def opt_record(udp_size=4096):
    """An EDNS0 OPT pseudo-record (root name, type 41, class = UDP size)."""
    return b"\0" + struct.pack(">HHiH", OPT, udp_size, 0, 0)


def reference_packet(response=True):
    """The packet of TestResolver.packet (test/src/test/java/vproxy/test/
    cases/TestResolver.java:41-112): id 0xabcd, response, QUERY, aa, rd, ra,
    NoError; question www.example.com. ANY/ANY; answers A 1.2.3.4 and AAAA
    ABCD:EF01:2345:6789:ABCD:EF01:2345:6789; authority CNAME my.dns.com. ->
    dns.server.com.; additional TXT some.text.com. ["abcdefghijklmn",
    "hello world"]; every resource class IN, ttl 600."""
    h = header(qd=1, an=2, ns=1, ar=1, ident=0xABCD, response=response, opcode=0, aa=True,
               tc=False, rd=True, ra=True, rcode=0)
    body = question("www.example.com.", ANY, ANY_CLASS)
    body += resource("www.example.com.", A, bytes([1, 2, 3, 4]))
    body += resource("www.example.com.", AAAA,
                     bytes.fromhex("ABCDEF0123456789ABCDEF0123456789"))
    body += resource("my.dns.com.", CNAME, name("dns.server.com."))
    body += resource("some.text.com.", TXT, txt("abcdefghijklmn", "hello world"))
    return h + body


def random_datagram(rng, names, mutate=0.25):
    """A random query over `names` (str or bytes qnames, trailing dot):
    1-5 questions of A / AAAA / SRV (mostly) or MX / ANY / TXT, some
    compressed with a pointer into an earlier question, an optional OPT
    record or answer; `mutate` of them then get a byte flipped, truncated or
    extended -- the malformed and odd shapes the parser must agree on."""
    nq = rng.choice([1, 1, 1, 1, 2, 2, 3, 5])
    body = b""
    starts = []
    for _ in range(nq):
        qn = rng.choice(names)
        qn = qn.encode() if isinstance(qn, str) else qn
        qt = rng.choice([A, A, A, AAAA, AAAA, SRV, MX, ANY, TXT])
        at = 12 + len(body)
        if starts and rng.random() < 0.2:
            # label + pointer to an earlier question's name
            body += bytes([3]) + b"www" + struct.pack(">H", 0xC000 | rng.choice(starts))
            body += struct.pack(">HH", qt, IN)
        else:
            body += name(qn) + struct.pack(">HH", qt, rng.choice([IN, IN, IN, CH, ANY_CLASS]))
        starts.append(at)
    ar = 0
    if rng.random() < 0.3:
        body += opt_record()
        ar = 1
    an = 0
    if rng.random() < 0.1:
        body += resource(b"\xc0\x0c", rng.choice([A, AAAA, CNAME, TXT, PTR, SRV, MX]),
                         rng.choice([bytes(4), bytes(16), name("x.y."), txt("ab"), b"\x01"]))
        an = 1
    d = bytearray(header(qd=nq, an=an, ar=ar, ident=rng.randrange(65536),
                         response=rng.random() < 0.05,
                         opcode=rng.choice([0] * 20 + [1, 2, 3, 4, 5, 6, 7]),
                         rcode=rng.choice([0] * 20 + [3, 11, 12, 15])) + body)
    r = rng.random()
    if r < mutate / 3 and len(d) > 1:
        d[rng.randrange(len(d))] = rng.randrange(256)
    elif r < 2 * mutate / 3:
        d = d[:rng.randrange(len(d) + 1)]
    elif r < mutate:
        d += bytes(rng.randrange(256) for _ in range(rng.randrange(1, 16)))
    return bytes(d)

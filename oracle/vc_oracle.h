/*
 * vc_oracle.h -- CPU restatement of vproxy's classification hot path.
 *
 * TEST INFRASTRUCTURE ONLY.  This library is the parity checker for the
 * MI355X classifier (libvclassify).  Only tests/, __graft_entry__.smoke() and
 * bench.py's cpu_baseline leg may load it.  The product path never links,
 * loads or calls it.
 *
 * Every function restates one Java method of nintha/vproxy (paths relative to
 * /root/reference) with Java semantics: signed bytes, list order, strict '>'
 * tie-breaks, String.equals/endsWith/startsWith over ASCII bytes.  Strings are
 * (pointer, length) pairs; a NULL pointer is Java `null`.
 *
 * Pinned by: tests/golden/ fixtures (vectors transcribed from the reference's
 * own JUnit tests TestNetMask, TestRouteTable, TestIpParser, the behavioural
 * tests TestSocks5/TestProtocols/CI, TestPacket, and SURVEY.md Appendix B
 * quirk KATs).  ServerGroup source hashing, SSLContextHolder.choose and the
 * vmirror filters have no reference test: they are pinned by hand-derived
 * vectors (tests/test_source_cpu.py, test_certs_cpu.py, test_mirror_cpu.py).
 */
#ifndef VC_ORACLE_H
#define VC_ORACLE_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
/* ---- HTTP/1 request head -> Hint -> Upstream.searchForGroup ----
 * HttpSubContext.feed over the request line and headers (states 0-8,
 * base/.../processor/http1/HttpSubContext.java:394-534; parsing stops at
 * the end of the headers, state 9), then HttpContext.connectionHint
 * (HttpContext.java:55-71) and Upstream.searchForGroup.  *kind: 0 = no hint
 * (null), 1 = Hint.ofUri, 2 = Hint.ofHost, 3 = Hint.ofHostUri.  Returns the
 * group index, -1 for none (and for a null hint). */
enum { VO_HTTP_NONE = 0, VO_HTTP_URI = 1, VO_HTTP_HOST = 2, VO_HTTP_HOST_URI = 3 };
int vo_http_hint(const vo_group *g, int ng, const uint8_t *head, int n, int *kind);
/* theUri / theHostHeader as the parser leaves them (raw bytes, one per Java
 * char; buffers of n bytes); returns the kind bits (1 uri set, 2 host set) */
int vo_http_extract(const uint8_t *head, int n, uint8_t *uri, int *uri_len, uint8_t *host,
                    int *host_len);
void vo_http_batch(const vo_group *g, int ng, const uint8_t *blob, const uint32_t *off, int64_t n,
                   uint8_t *kind, int32_t *group, int nthreads);

#endif

/* ---- IP parsing: base/src/main/java/vfd/IP.java ---- */
int vo_parse_ipv4(const char *s, int len, uint8_t out[4]);   /* IP.java:120-127; 4 or -1 */
int vo_parse_ipv6(const char *s, int len, uint8_t out[16]);  /* IP.java:158-197; 16 or -1 */
int vo_parse_ip(const char *s, int len, uint8_t out[16]);    /* IP.java:112-117; 4/16/-1 */
int vo_is_ipv6(const char *s, int len);                      /* IP.java:294-296 */
int vo_is_ip_literal(const char *s, int len);                /* IP.java:271-300 */

/* ---- Network: base/src/main/java/vproxybase/util/Network.java ---- */
int vo_parse_mask(int m, uint8_t out[16]);                   /* :101-115; len or -1 (throws) */
int vo_mask_int(const uint8_t *mask, int mlen);              /* :135-145 */
int vo_valid_network(const uint8_t *a, int alen, const uint8_t *m, int mlen); /* :163-181 */
int vo_mask_match(const uint8_t *in, int inlen, const uint8_t *rule, int rlen,
                  const uint8_t *mask, int mlen);            /* :183-278 */

typedef struct {
    uint8_t ip[16];
    uint8_t mask[16];
    int32_t ip_len;    /* 4 or 16 */
    int32_t mask_len;  /* 4 or 16 */
} vo_net;

int vo_net_from_str(const char *s, int len, vo_net *out);     /* Network(String) :16-25; 0 ok, -1 invalid */
int vo_net_contains_ip(const vo_net *n, const uint8_t *ip, int iplen); /* :27-29 */
int vo_net_contains_net(const vo_net *a, const vo_net *b);    /* :31-36 */
int vo_net_equals(const vo_net *a, const vo_net *b);          /* :50-57 */

/* ---- SecurityGroup: core/.../component/secure/SecurityGroup{,Rule}.java ---- */
typedef struct {
    vo_net net;
    int32_t min_port, max_port;
    int32_t allow;
} vo_sg_rule;

/* SecurityGroup.allow (SecurityGroup.java:30-45) with the matched index
 * exposed: returns index into the protocol's list, or -1 for defaultAllow.
 * *verdict receives the boolean allow() would return. proto==6 -> tcp list,
 * anything else -> udp list (Java's else-branch). */
int vo_sg_allow(const vo_sg_rule *tcp, int ntcp, const vo_sg_rule *udp, int nudp,
                int default_allow, int proto, const uint8_t *ip, int iplen, int port,
                int *verdict);

/* batched, pthread-partitioned restatement (CPU baseline). src4 = big-endian
 * int (IP.ipv4Bytes2Int); out_idx per item; verdict optional. */
void vo_sg_allow_batch_v4(const vo_sg_rule *tcp, int ntcp, const vo_sg_rule *udp, int nudp,
                          int default_allow, const uint8_t *proto, const uint32_t *src4,
                          const uint16_t *port, int64_t n, int32_t *out_idx, uint8_t *out_verdict,
                          int nthreads);
void vo_sg_allow_batch_v6(const vo_sg_rule *tcp, int ntcp, const vo_sg_rule *udp, int nudp,
                          int default_allow, const uint8_t *proto, const uint8_t *src6,
                          const uint16_t *port, int64_t n, int32_t *out_idx, uint8_t *out_verdict,
                          int nthreads);

/* ---- RouteTable: core/src/main/java/vswitch/RouteTable.java ---- */
typedef struct {
    vo_net *v4; int n4, cap4;
    vo_net *v6; int n6, cap6;
} vo_route_table;

void vo_rt_init(vo_route_table *t);
void vo_rt_free(vo_route_table *t);
/* RouteTable.addRule(RouteRule) ordering part (:68-154): duplicate network ->
 * returns -1 (AlreadyExistException), else 0.  Alias/ip checks are host-side. */
int vo_rt_add(vo_route_table *t, const vo_net *n);
/* RouteTable.lookup (:44-59): family list index or -1 (null). */
int vo_rt_lookup(const vo_route_table *t, const uint8_t *ip, int iplen);
int vo_rt_lookup_list(const vo_net *list, int n, const uint8_t *ip, int iplen);
void vo_rt_lookup_batch_v4(const vo_net *v4, int n4, const uint32_t *dst4, int64_t n,
                           int32_t *out, int nthreads);
void vo_rt_lookup_batch_v6(const vo_net *v6, int n6, const uint8_t *dst6, int64_t n,
                           int32_t *out, int nthreads);

/* ---- Hint / Upstream: base/.../processor/Hint.java, core/.../svrgroup/Upstream.java ---- */
typedef struct {
    const char *host; int32_t host_len;   /* NULL = absent */
    int32_t port;                         /* 0 = absent */
    const char *uri; int32_t uri_len;     /* NULL = absent */
} vo_annos;

typedef struct {
    vo_annos handle;   /* ServerGroupHandle.annotations */
    vo_annos group;    /* ServerGroup.getAnnotations()  */
} vo_group;

typedef struct {
    const char *host; int32_t host_len;
    int32_t port;
    const char *uri; int32_t uri_len;
} vo_hint;

/* Hint.formatHost (:57-73): writes [*off,*len) sub-range of s; returns 1 if
 * non-null, 0 if the result is null. */
int vo_format_host(const char *s, int len, int *off, int *olen);
/* Hint.formatUri (:75-90): same convention. */
int vo_format_uri(const char *s, int len, int *off, int *olen);
/* Hint.of{Host,HostPort,HostUri,HostPortUri,Uri} (:17-55). host/uri may be NULL. */
vo_hint vo_hint_of(const char *host, int host_len, int port, const char *uri, int uri_len);
int vo_match_level(const vo_hint *h, const vo_annos *a, int na);   /* :100-160 */
int vo_search_for_group(const vo_group *g, int ng, const vo_hint *h); /* Upstream.java:187-198 */

/* batched, pthread-partitioned searchForGroup(Hint.ofHostPort(host, port))
 * over a packed host blob (item i = blob[off[i], off[i+1])) -- CPU baseline. */
void vo_hint_batch(const vo_group *g, int ng, const uint8_t *blob, const uint32_t *off,
                   const uint16_t *port, int64_t n, int32_t *out, int nthreads);
/* the same with uris: searchForGroup(Hint.ofHostPortUri(host, port, uri)),
 * uri i = ublob[uoff[i], uoff[i+1]) unless unull[i] (unull / port may be NULL) */
void vo_hint_uri_batch(const vo_group *g, int ng, const uint8_t *hblob, const uint32_t *hoff,
                       const uint8_t *ublob, const uint32_t *uoff, const uint8_t *unull,
                       const uint16_t *port, int64_t n, int32_t *out, int nthreads);

/* ---- DNSServer classification: core/src/main/java/vproxy/dns/DNSServer.java:116-166 ---- */
enum { VO_DNS_HOSTS = 1, VO_DNS_GROUP = 2, VO_DNS_IP_LITERAL = 3, VO_DNS_INTERNAL = 4, VO_DNS_RECURSIVE = 5 };
typedef struct {
    const char *const *keys; const int32_t *key_lens; const int32_t *values; int n;
} vo_hosts;  /* exact map, linear lookup; first key wins */
/* returns kind; *value = hosts value / group index / 4|6 for literal / 0 */
int vo_dns_classify(const vo_hosts *hosts, const vo_group *g, int ng,
                    const char *qname, int qlen, int32_t *value);

/* Resolver.getHosts (base/.../dns/Resolver.java:62-153) over the text of a
 * hosts file.  Emits map entries (key -> value) in insertion order: keys are
 * copied into keybuf (key_off/key_len), value = index of the accepted host
 * line (its IP bytes in line_ip[16*value], length line_iplen[value]).
 * Returns the entry count, or -1 if a capacity is exceeded. */
int vo_hosts_parse(const char *text, int len,
                   char *keybuf, int keybuf_cap, int32_t *key_off, int32_t *key_len,
                   int32_t *value, int cap,
                   uint8_t *line_ip, int32_t *line_iplen, int line_cap);

/* ---- ServerGroup source-hash selection:
 *      base/src/main/java/vproxybase/component/svrgroup/ServerGroup.java ---- */
typedef struct {
    uint8_t ip[16];
    int32_t ip_len;    /* 4 (IPv4 server) or 16 */
    int32_t port;
    int32_t weight;
    int32_t healthy;
} vo_server;

/* SOURCE.hash (sdbm over the signed address bytes, Math.abs, MIN_VALUE -> 0)
 * ServerGroup.java:387-397 */
int32_t vo_source_hash(const uint8_t *bytes, int len);
/* sourceReset (ServerGroup.java:626-664): the weight > 0 servers of `view`
 * (0 = all, 4 = IPv4 servers, 6 = IPv6 servers, :620-624) sorted by address
 * length, then signed address bytes, then port (stable).  Writes indices
 * into `servers` to order[] and returns how many. */
int vo_source_list(const vo_server *servers, int n, int view, int32_t *order);
/* sourceHashGet (ServerGroup.java:464-490): index into `servers` of the
 * chosen server, or -1 (null: empty list or no healthy server). */
int vo_source_select(const vo_server *servers, int n, int view, const uint8_t *src, int src_len);

/* ---- Packet header extraction: base/src/main/java/vpacket/ ----
 * VXLanPacket.from (:16-33) -> EthernetPacket.from (:14-50) -> ArpPacket /
 * Ipv4Packet (:28-101) / Ipv6Packet (:24-106) .from -> TcpPacket (:164-227) /
 * IcmpPacket (:22-33) .from.  `layer` names the class the caller starts with
 * (0 VXLAN, 1 Ethernet, 4 IPv4, 6 IPv6). */
typedef struct {
    int status;        /* 0 ok, 1 vxlan error, 2 ethernet/ARP error, 3 IP-layer error (layer 4/6),
                          4 the Java parser throws, 5 the Java parser never returns */
    int l3;            /* 0 PacketBytes, 1 ARP, 4 IPv4, 6 IPv6, 5 IP ether type kept as bytes */
    int l4;            /* 0 bytes, 1 ICMP, 58 ICMPv6, 6 TCP */
    int proto;
    uint32_t vni;
    int ether_type;
    uint8_t src[16], dst[16];   /* IPv4: first 4 bytes */
    int sport, dport;
} vo_pkt;

void vo_parse_packet(const uint8_t *p, int len, int layer, vo_pkt *out);

/* ---- Traffic-mirror filters: base/src/main/java/vmirror/ ----
 * FilterConfig (FilterConfig.java:7-21) with ids for the strings (origin,
 * transportLayerProtocol, applicationLayerProtocol; -1 = null) and the
 * MirrorConfig as an index 0..63. */
typedef struct {
    int32_t origin, mirror;
    int32_t has_mac_x, has_mac_y;
    uint8_t mac_x[6], mac_y[6];
    int32_t has_net_x, has_net_y;
    vo_net net_x, net_y;
    int32_t transport;
    int32_t has_port_x, has_port_y;
    int32_t port_x[2], port_y[2];
    int32_t app;
} vo_mirror_filter;

/* Mirror.mirror(MirrorData) filter step (Mirror.java:89-118, checkHelper
 * :133-139): bit m set when a filter of `origin` whose mirror is m matches
 * at the level picked by the null fields (ip_*_len 0 = null IP, transport /
 * app -1 = null). */
uint64_t vo_mirror_match(const vo_mirror_filter *f, int n, int origin,
                         const uint8_t *mac_src, const uint8_t *mac_dst,
                         const uint8_t *ip_src, int src_len, const uint8_t *ip_dst, int dst_len,
                         int transport, int port_src, int port_dst, int app);
/* Mirror.switchPacket (Mirror.java:73-87) on a raw VXLAN (layer 0) or
 * Ethernet (layer 1) frame; 0 when the parse rejects the frame. */
uint64_t vo_mirror_switch(const vo_mirror_filter *f, int n, int origin, const uint8_t *frame,
                          int len, int layer);

/* ---- SSLContextHolder.choose (base/src/main/java/vproxybase/util/ringbuffer/ssl/
 *      SSLContextHolder.java:51-186) ----
 * Holders 0..n_holders-1 in add() order; names[i] (length name_lens[i]) is a
 * CN or SAN dNSName of a certificate of holder[i], in the holder's own
 * certificate order.  Returns the chosen holder, or -1 (null, no holders). */
int vo_cert_choose(const char *const *names, const int32_t *name_lens, const int32_t *holder,
                   int n_names, int n_holders, const uint8_t *sni, int sni_len, int sni_null);

/* ---- batched, pthread-partitioned forms of the restatements above (the
 * GPU tests' checkers and bench.py's cpu_baseline legs); item i of a packed
 * blob = blob[off[i], off[i+1]) ---- */
void vo_dns_batch(const vo_hosts *hosts, const vo_group *g, int ng, const uint8_t *blob,
                  const uint32_t *off, int64_t n, uint8_t *kind, int32_t *value, int nthreads);
void vo_parse_batch(const uint8_t *blob, const uint32_t *off, int64_t n, int layer, vo_pkt *out,
                    int nthreads);
/* Switch.java:679-684 + L3.java:423-444 per datagram: the bare-VXLAN
 * SecurityGroup check of the IPv4 sender (UDP list, bind port), the VXLAN
 * parse, and RouteTable.lookup of the inner destination when allowed and
 * the frame parses to IPv4/IPv6 (else -1).  remote4 in IP.ipv4Bytes2Int order. */
void vo_switch_batch(const vo_sg_rule *tcp, int ntcp, const vo_sg_rule *udp, int nudp,
                     int default_allow, const uint8_t *blob, const uint32_t *off, int64_t n,
                     const uint32_t *remote4, int bind_port, const vo_net *v4, int n4,
                     const vo_net *v6, int n6, int32_t *acl, uint8_t *allow, int32_t *route,
                     int nthreads);
/* SSLContextHolder.choose per SNI (sni_null may be NULL: none null) */
void vo_cert_batch(const char *const *names, const int32_t *name_lens, const int32_t *holder,
                   int n_names, int n_holders, const uint8_t *blob, const uint32_t *off,
                   const uint8_t *sni_null, int64_t n, int32_t *out, int nthreads);
void vo_mirror_match_batch(const vo_mirror_filter *f, int nf, int origin, const uint8_t *mac_src,
                           const uint8_t *mac_dst, const uint8_t *src_len, const uint8_t *dst_len,
                           const uint8_t *ip_src, const uint8_t *ip_dst, const int32_t *transport,
                           const int32_t *port_src, const int32_t *port_dst, const int32_t *app,
                           int64_t n, uint64_t *out, int nthreads);
void vo_mirror_switch_batch(const vo_mirror_filter *f, int nf, int origin, const uint8_t *blob,
                            const uint32_t *off, int64_t n, int layer, uint64_t *out,
                            int nthreads);
/* sourceHashGet per item: group grp[i]'s servers are servers[goff[g], goff[g+1]);
 * the sourceReset order of every group is built once first (Java caches it
 * until the next reset); src4 in IP.ipv4Bytes2Int order; out = the index
 * within the group, or -1. */
void vo_source_batch(const vo_server *servers, const int32_t *goff, int n_groups, int view,
                     const int32_t *grp, const uint32_t *src4, int64_t n, int32_t *out,
                     int nthreads);

#ifdef __cplusplus
}
/* ---- HTTP/1 request head -> Hint -> Upstream.searchForGroup ----
 * HttpSubContext.feed over the request line and headers (states 0-8,
 * base/.../processor/http1/HttpSubContext.java:394-534; parsing stops at
 * the end of the headers, state 9), then HttpContext.connectionHint
 * (HttpContext.java:55-71) and Upstream.searchForGroup.  *kind: 0 = no hint
 * (null), 1 = Hint.ofUri, 2 = Hint.ofHost, 3 = Hint.ofHostUri.  Returns the
 * group index, -1 for none (and for a null hint). */
enum { VO_HTTP_NONE = 0, VO_HTTP_URI = 1, VO_HTTP_HOST = 2, VO_HTTP_HOST_URI = 3 };
int vo_http_hint(const vo_group *g, int ng, const uint8_t *head, int n, int *kind);
/* theUri / theHostHeader as the parser leaves them (raw bytes, one per Java
 * char; buffers of n bytes); returns the kind bits (1 uri set, 2 host set) */
int vo_http_extract(const uint8_t *head, int n, uint8_t *uri, int *uri_len, uint8_t *host,
                    int *host_len);
void vo_http_batch(const vo_group *g, int ng, const uint8_t *blob, const uint32_t *off, int64_t n,
                   uint8_t *kind, int32_t *group, int nthreads);

#endif

/* DNSServer's drain loop per datagram (DNSServer.java:457-500, Formatter.
 * parsePackets, handleRequest); the status codes equal vclassify.h's
 * VC_DNSD_*.  qtype/kind/value are set for the first nq questions. */
enum { VO_DNSD_ANSWER = 0, VO_DNSD_RECURSIVE = 1, VO_DNSD_RESPONSE = 2, VO_DNSD_REJECTED = 3,
       VO_DNSD_EMPTY = 4, VO_DNSD_MALFORMED = 5, VO_DNSD_HOST = 6 };
#define VO_DNSD_MAXQ 4
#define VO_DNSD_NAMECAP 128
#define VO_DNSD_MAXPTR 16
typedef struct {
    int32_t status, acl, nq;
    int32_t qtype[VO_DNSD_MAXQ], kind[VO_DNSD_MAXQ], value[VO_DNSD_MAXQ];
} vo_dnsd_out;
void vo_dns_datagram(const vo_sg_rule *tcp, int ntcp, const vo_sg_rule *udp, int nudp,
                     int default_allow, const vo_hosts *hosts, const vo_group *g, int ng,
                     const uint8_t *p, int n, const uint8_t *ip, int iplen, int port,
                     vo_dnsd_out *out);
/* remote4 in IP.ipv4Bytes2Int order; family may be NULL (all IPv4) */
void vo_dnsd_batch(const vo_sg_rule *tcp, int ntcp, const vo_sg_rule *udp, int nudp,
                   int default_allow, const vo_hosts *hosts, const vo_group *g, int ng,
                   const uint8_t *blob, const uint32_t *off, int64_t n, const uint8_t *family,
                   const uint32_t *remote4, const uint8_t *remote6, const uint16_t *remote_port,
                   vo_dnsd_out *out, int nthreads);

/* ---- HTTP/1 request head -> Hint -> Upstream.searchForGroup ----
 * HttpSubContext.feed over the request line and headers (states 0-8,
 * base/.../processor/http1/HttpSubContext.java:394-534; parsing stops at
 * the end of the headers, state 9), then HttpContext.connectionHint
 * (HttpContext.java:55-71) and Upstream.searchForGroup.  *kind: 0 = no hint
 * (null), 1 = Hint.ofUri, 2 = Hint.ofHost, 3 = Hint.ofHostUri.  Returns the
 * group index, -1 for none (and for a null hint). */
enum { VO_HTTP_NONE = 0, VO_HTTP_URI = 1, VO_HTTP_HOST = 2, VO_HTTP_HOST_URI = 3 };
int vo_http_hint(const vo_group *g, int ng, const uint8_t *head, int n, int *kind);
/* theUri / theHostHeader as the parser leaves them (raw bytes, one per Java
 * char; buffers of n bytes); returns the kind bits (1 uri set, 2 host set) */
int vo_http_extract(const uint8_t *head, int n, uint8_t *uri, int *uri_len, uint8_t *host,
                    int *host_len);
void vo_http_batch(const vo_group *g, int ng, const uint8_t *blob, const uint32_t *off, int64_t n,
                   uint8_t *kind, int32_t *group, int nthreads);

#endif

/*
 * vclassify.h -- C ABI of libvclassify, the MI355X-native batched classifier
 * behind vproxy's classification API.
 *
 * Each batched entry point replaces one Java hot-path method (paths relative
 * to the nintha/vproxy tree).  The JNI shim a maintainer would add on the Java
 * side is jni/vproxy_component_secure_GpuClassifier.c (+ jni/GpuClassifier.java,
 * walked through in INTEGRATION.md); it maps 1:1 onto these functions in the
 * style of base/src/main/c/vfd_posix_GeneralPosix.c (jlong handles, direct
 * ByteBuffers, status codes mapped to IOException/UnsupportedOperationException).
 * tests/native/abi_c.c is a plain C99 consumer of this header.
 *
 * Conventions
 *  - Plain C types only.  Every function returns an int status (VC_OK = 0,
 *    negative VC_E* on error); the message is available from vc_last_error().
 *  - Results are indices into the *live Java lists* in list order, -1 for
 *    null / "no rule" (the caller maps index -> SecurityGroupRule / RouteRule
 *    / ServerGroupHandle exactly as the Java code would have returned it).
 *  - *_dev functions take DEVICE pointers and a hipStream_t (passed as void*,
 *    NULL = HIP's null stream); they are asynchronous and ordered on it.  The
 *    plain variants take HOST pointers and are synchronous (H2D + kernel +
 *    D2H, or zero-copy over buffers registered with vc_host_register).
 *  - A batch of n = 0 items is a no-op that returns VC_OK without reading or
 *    writing any array (its pointers may be NULL); n < 0 is VC_EINVAL.
 *  - IPv4 addresses are uint32 in IP.ipv4Bytes2Int order (big-endian value,
 *    vfd/IP.java:476-478); IPv6 addresses are 16 raw bytes per item.
 *  - Strings are packed in a byte blob with uint32 offsets (n+1 entries, item
 *    i = blob[off[i], off[i+1])); an optional uint8 `null` array marks Java
 *    null items (NULL pointer = no null items).
 *  - String encoding: every Java String crosses the boundary as its UTF-8
 *    bytes (String.getBytes(UTF_8); an unpaired surrogate, which that call
 *    would replace by '?', must be sent as its 3-byte WTF-8 form).  That
 *    covers annotations (hint-host / hint-uri), hosts-file keys, Host / SNI /
 *    URI hint strings and certificate names.  equals / startsWith / endsWith
 *    on these bytes agree with Java's on the strings, and the one length Java
 *    scores -- Hint.matchLevel's uriLevel = uri.length() + 1
 *    (base/src/main/java/vproxybase/processor/Hint.java:146-150) -- is taken
 *    in UTF-16 units of the annotation, so non-ASCII URIs score as in Java.
 *    The exception is DNS: qnames are the wire bytes Formatter.parseDomainName
 *    reads (base/.../dns/Formatter.java:225-257 appends (char) b per byte b,
 *    and the Java byte -> char cast sign-extends): a qname byte 0xE9 is the
 *    char U+FFE9 and matches the annotation bytes EF BF A9, as in Java.  vc_compile_hosts_text reads the
 *    hosts file as UTF-8, as Resolver.getHosts' InputStreamReader does with a
 *    UTF-8 default charset.
 *  - Rule tables are compiled into immutable snapshots and published
 *    atomically; concurrent classify calls keep using the snapshot they
 *    started with (threads: SURVEY.md §8(b) "Threading").
 */
#ifndef VCLASSIFY_H
#define VCLASSIFY_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define VC_OK         0
#define VC_EINVAL    -1   /* IllegalArgumentException (bad network, mask, size) */
#define VC_EEXIST    -2   /* AlreadyExistException */
#define VC_ENOTFOUND -3   /* NotFoundException */
#define VC_EXEXC     -4   /* XException (RouteTable validation) */
#define VC_EDEVICE   -5   /* HIP runtime / device error */
#define VC_ENOMEM    -6
#define VC_ESTATE    -7   /* nothing compiled yet for this classifier */

#define VC_PROTO_TCP  6   /* vproxybase.connection.Protocol.TCP */
#define VC_PROTO_UDP 17   /* Protocol.UDP (any non-6 value selects the UDP list) */

typedef struct vc_ctx vc_ctx;

const char *vc_version(void);
/* Thread-local message of the last failing call on this thread. */
const char *vc_last_error(void);

/* One classifier instance on one GPU (device ordinal).  Fails with
 * VC_EDEVICE when no MI355X (gfx950) device is usable: there is no CPU path. */
int vc_create(int device, vc_ctx **out);
void vc_destroy(vc_ctx *ctx);

/* ------------------------------------------------------------------------ */
/* Snapshot pins (SURVEY.md §8(b) "Threading").  The reference's readers    */
/* never wait for a writer: SecurityGroup and Upstream swap copy-on-write    */
/* lists (core/src/main/java/vproxy/component/secure/SecurityGroup.java:     */
/* 56-103, core/.../svrgroup/Upstream.java:146-157).  Every vc_compile_*    */
/* (and vc_servers_set_health) publishes an immutable snapshot under a new  */
/* generation; a caller that maps result indices back to its own lists pins */
/* the snapshots its lists describe, binds the pin to the thread that runs  */
/* the batch, and maps through those lists -- no lock across the compile.   */
/* ------------------------------------------------------------------------ */
#define VC_SNAP_ACL       0   /* vc_compile_acl (SecurityGroup) */
#define VC_SNAP_ROUTE     1   /* vc_compile_routes (RouteTable) */
#define VC_SNAP_UPSTREAM  2   /* vc_compile_upstream (Upstream) */
#define VC_SNAP_HOSTS     3   /* vc_compile_hosts[_text] (Resolver.getHosts) */
#define VC_SNAP_SERVERS   4   /* vc_compile_servers / vc_servers_set_health */
#define VC_SNAP_CERTS     5   /* vc_compile_certs */
#define VC_SNAP_MIRROR    6   /* vc_compile_mirror */
#define VC_SNAP_VNI       7   /* vc_compile_vni_routes (Switch.tables) */
#define VC_SNAP_ALL       0xFF
typedef struct vc_pin vc_pin;
/* Pins the snapshots of the kinds in the bit set `kinds` (1 << VC_SNAP_*)
 * that are current now.  The pin keeps them (and their device tables)
 * alive until vc_pin_release; it never blocks a compile, and a compile
 * never waits for it. */
int vc_pin_acquire(vc_ctx *ctx, uint32_t kinds, vc_pin **out);
/* Calls on ctx from the calling thread use pin's snapshots for the kinds
 * it pinned (the current ones for the others) until the next bind; NULL
 * unbinds.  A pin may be bound on several threads at once. */
int vc_pin_bind(vc_ctx *ctx, const vc_pin *pin);
/* The generation of a pinned snapshot: every publish on a context takes
 * the next number (from 1, shared by all kinds); 0 = nothing compiled. */
int vc_pin_generation(const vc_pin *pin, int kind, uint64_t *gen);
/* Unbinds it from the calling thread if bound there (binding a released
 * pin on another thread is the caller's error). */
void vc_pin_release(vc_pin *pin);
/* The generation of the current snapshot of `kind` (0 = none). */
int vc_generation(vc_ctx *ctx, int kind, uint64_t *gen);

/* ------------------------------------------------------------------------ */
/* Network value: base/src/main/java/vproxybase/util/Network.java            */
/* ------------------------------------------------------------------------ */
typedef struct vc_net {
    uint8_t ip[16];     /* Network.ip, first ip_len bytes used */
    uint8_t mask[16];   /* Network.mask = parseMask(m): 4 bytes if m <= 32 else 16 */
    int32_t ip_len;     /* 4 or 16 */
    int32_t mask_len;   /* 4 or 16 */
} vc_net;

/* new Network(String) (Network.java:16-25): "a.b.c.d/m" or "v6/m";
 * VC_EINVAL when validNetworkStr fails. */
int vc_net_parse(const char *s, vc_net *out);
/* new Network(ip, Network.parseMask(prefix)) with validNetwork enforced
 * (NetworkHandle.get, app/.../param/NetworkHandle.java:21-30). */
int vc_net_from_prefix(const uint8_t *ip, int ip_len, int prefix, vc_net *out);
/* Network.contains(IP) -> Network.maskMatch (Network.java:27-29,183-278). */
int vc_net_contains_ip(const vc_net *net, const uint8_t *ip, int ip_len);
/* IP.parseIpString (vfd/IP.java:112-117): returns 4, 16 or VC_EINVAL. */
int vc_ip_parse(const char *s, uint8_t out[16]);

/* ------------------------------------------------------------------------ */
/* SecurityGroup: core/src/main/java/vproxy/component/secure/SecurityGroup.java */
/* ------------------------------------------------------------------------ */
typedef struct vc_acl_rule {
    vc_net net;          /* SecurityGroupRule.network */
    int32_t min_port;    /* SecurityGroupRule.minPort */
    int32_t max_port;    /* SecurityGroupRule.maxPort */
    int32_t allow;       /* SecurityGroupRule.allow */
} vc_acl_rule;

/* Compile SecurityGroup{tcpRules, udpRules, defaultAllow} (list order =
 * priority) into the GPU ACL image and publish it. */
int vc_compile_acl(vc_ctx *ctx, const vc_acl_rule *tcp, int n_tcp,
                   const vc_acl_rule *udp, int n_udp, int default_allow);

/* Batched SecurityGroup.allow(Protocol, IP, int) (SecurityGroup.java:30-45).
 * out_idx[i] = index of the first matching rule in the protocol's list, or
 * -1 when defaultAllow decided; out_allow[i] (optional) = the boolean allow()
 * returns.  proto: VC_PROTO_TCP selects tcpRules, anything else udpRules. */
int vc_acl_classify_v4_dev(vc_ctx *ctx, const uint8_t *proto, const uint32_t *src4,
                           const uint16_t *port, int64_t n, int32_t *out_idx,
                           uint8_t *out_allow, void *stream);
int vc_acl_classify_v6_dev(vc_ctx *ctx, const uint8_t *proto, const uint8_t *src6,
                           const uint16_t *port, int64_t n, int32_t *out_idx,
                           uint8_t *out_allow, void *stream);
int vc_acl_classify_v4(vc_ctx *ctx, const uint8_t *proto, const uint32_t *src4,
                       const uint16_t *port, int64_t n, int32_t *out_idx, uint8_t *out_allow);
int vc_acl_classify_v6(vc_ctx *ctx, const uint8_t *proto, const uint8_t *src6,
                       const uint16_t *port, int64_t n, int32_t *out_idx, uint8_t *out_allow);

/* ------------------------------------------------------------------------ */
/* RouteTable: core/src/main/java/vswitch/RouteTable.java                    */
/* ------------------------------------------------------------------------ */
/* Compile rulesV4 / rulesV6 (list order = priority: lookup returns the first
 * matching rule, RouteTable.java:44-59) into stride tries and publish. */
int vc_compile_routes(vc_ctx *ctx, const vc_net *v4, int n4, const vc_net *v6, int n6);
/* Batched RouteTable.lookup(IP): out[i] = index in rulesV4 (v4 call) or
 * rulesV6 (v6 call), -1 for null. */
int vc_route_lookup_v4_dev(vc_ctx *ctx, const uint32_t *dst4, int64_t n, int32_t *out,
                           void *stream);
int vc_route_lookup_v6_dev(vc_ctx *ctx, const uint8_t *dst6, int64_t n, int32_t *out,
                           void *stream);
int vc_route_lookup_v4(vc_ctx *ctx, const uint32_t *dst4, int64_t n, int32_t *out);
int vc_route_lookup_v6(vc_ctx *ctx, const uint8_t *dst6, int64_t n, int32_t *out);

/* Switch.tables (Switch.java:560-566): one RouteTable per VNI, for the
 * switch entry points (vc_switch_classify[_dev]).  Table t has VNI vni[t]
 * (24-bit, distinct) and rules v4[v4_off[t] .. v4_off[t + 1]) and
 * v6[v6_off[t] .. v6_off[t + 1]) in list order (CSR offsets, n_tables + 1
 * entries each).  n_tables == 0 removes the per-VNI tables. */
#define VC_SWITCH_NO_TABLE (-2)
int vc_compile_vni_routes(vc_ctx *ctx, const int32_t *vni, const vc_net *v4,
                          const int32_t *v4_off, const vc_net *v6, const int32_t *v6_off,
                          int n_tables);

/* ------------------------------------------------------------------------ */
/* Upstream hint matching: core/.../svrgroup/Upstream.java + Hint.java       */
/* ------------------------------------------------------------------------ */
typedef struct vc_annos {      /* vproxybase.util.Annotations hint fields */
    const char *host; int32_t host_len;   /* vproxy/hint-host, NULL = absent */
    int32_t port;                         /* vproxy/hint-port, 0 = absent */
    const char *uri; int32_t uri_len;     /* vproxy/hint-uri, NULL = absent */
} vc_annos;

typedef struct vc_group_annos {  /* one ServerGroupHandle, in Upstream list order */
    vc_annos handle;             /* ServerGroupHandle.getAnnotations() */
    vc_annos group;              /* handle.group.getAnnotations() */
} vc_group_annos;

/* Compile Upstream.serverGroupHandles (list order) for searchForGroup. */
int vc_compile_upstream(vc_ctx *ctx, const vc_group_annos *groups, int n);

/* Batched Upstream.searchForGroup(Hint.ofHostPortUri(host, port, uri))
 * (Upstream.java:187-198, Hint.java:17-160): raw host/uri strings are
 * formatted on the device exactly as Hint.formatHost/formatUri do.
 * host_null / uri_blob / uri_off / uri_null may be NULL.  out_group[i] =
 * handle index or -1 (null). */
int vc_hint_search_dev(vc_ctx *ctx, const uint8_t *host_blob, const uint32_t *host_off,
                       const uint8_t *host_null, const uint16_t *port,
                       const uint8_t *uri_blob, const uint32_t *uri_off, const uint8_t *uri_null,
                       int64_t n, int32_t *out_group, void *stream);
int vc_hint_search(vc_ctx *ctx, const uint8_t *host_blob, const uint32_t *host_off,
                   const uint8_t *host_null, const uint16_t *port,
                   const uint8_t *uri_blob, const uint32_t *uri_off, const uint8_t *uri_null,
                   int64_t n, int32_t *out_group);

/* ------------------------------------------------------------------------ */
/* DNSServer classification: core/src/main/java/vproxy/dns/DNSServer.java:116-166 */
/* ------------------------------------------------------------------------ */
#define VC_DNS_HOSTS       1  /* hosts.get(qname) hit: value = hosts value */
#define VC_DNS_GROUP       2  /* rrsets.searchForGroup(Hint.ofHost(domain)): value = handle index */
#define VC_DNS_IP_LITERAL  3  /* IP.isIpLiteral(domain): value = 4 or 6 (IP.from type) */
#define VC_DNS_INTERNAL    4  /* domain.endsWith(".vproxy.local") */
#define VC_DNS_RECURSIVE   5  /* falls through to runRecursive */

/* The hosts map (Resolver.getHosts result, exact keys incl. trailing-dot
 * variants).  The rrsets Upstream is the one given to vc_compile_upstream. */
int vc_compile_hosts(vc_ctx *ctx, const char *const *keys, const int32_t *key_lens,
                     const int32_t *values, int n);
/* Resolver.getHosts over hosts-file text (Resolver.java:62-153), then
 * vc_compile_hosts; value = index of the accepted host line. */
int vc_compile_hosts_text(vc_ctx *ctx, const char *text, int64_t len);
int vc_dns_classify_dev(vc_ctx *ctx, const uint8_t *qblob, const uint32_t *qoff, int64_t n,
                        uint8_t *out_kind, int32_t *out_value, void *stream);
int vc_dns_classify(vc_ctx *ctx, const uint8_t *qblob, const uint32_t *qoff, int64_t n,
                    uint8_t *out_kind, int32_t *out_value);

/* ------------------------------------------------------------------------ */
/* The upstream group of an HTTP/1 request (HttpLB's frontend): for request
 * head i = blob[off[i], off[i+1]), HttpSubContext's request-line and header
 * states (HttpSubContext.java:394-534, parsing stops at the empty line that
 * ends the headers), HttpContext.connectionHint (HttpContext.java:55-71:
 * theUri and the last Host header's trimmed value; Hint.ofUri / ofHost /
 * ofHostUri) and Upstream.searchForGroup on the compiled Upstream.
 * out_group = handle index, -1 for no group and for a null hint; out_kind
 * (optional) = VC_HTTP_* of the hint.  Heads are bytes as they came off the
 * socket; the _dev form needs blob_bytes >= off[n] (it sizes the scratch
 * that heads with CR or non-ASCII bytes in their uri / Host are rewritten
 * into). */
/* ------------------------------------------------------------------------ */
#define VC_HTTP_NONE      0  /* no uri and no Host header: the hint is null */
#define VC_HTTP_URI       1  /* Hint.ofUri(theUri) */
#define VC_HTTP_HOST      2  /* Hint.ofHost(theHostHeader) */
#define VC_HTTP_HOST_URI  3  /* Hint.ofHostUri(theHostHeader, theUri) */
#define VC_HTTP_BAD_SPAN  0xFF  /* _dev only: off[i + 1] > blob_bytes, not classified (group -1) */
int vc_http_hint_dev(vc_ctx *ctx, const uint8_t *blob, int64_t blob_bytes, const uint32_t *off,
                     int64_t n, int32_t *out_group, uint8_t *out_kind, void *stream);
int vc_http_hint(vc_ctx *ctx, const uint8_t *blob, const uint32_t *off, int64_t n,
                 int32_t *out_group, uint8_t *out_kind);

/* DNSServer's drain loop per datagram (DNSServer.java:457-500): for UDP
 * payload i = blob[off[i], off[i+1]) from the remote address (family 4/6,
 * remote4 in IP.ipv4Bytes2Int order or 16 remote6 bytes, 16-byte aligned)
 * and port: securityGroup.allow(Protocol.UDP, remote, remote port) on the
 * compiled SecurityGroup's UDP list; `read == 0`; Formatter.parsePackets
 * (Formatter.java:162-372: header, questions, resources, the A / AAAA /
 * CNAME / PTR / TXT / SRV rdata checks); then p.isResponse, the opcode and
 * handleRequest's classification of each question in order (the kinds of
 * vc_dns_classify) until one sends the packet to runRecursive.  The
 * answers themselves (server choice, records) stay with the caller. */
#define VC_DNSD_ANSWER     0  /* handleRequest answers every question locally */
#define VC_DNSD_RECURSIVE  1  /* runRecursive(p, remote): opcode != QUERY (nq = 0), a
                                 qtype other than A / AAAA / SRV, or a name no table
                                 knows (the last evaluated question) */
#define VC_DNSD_RESPONSE   2  /* p.isResponse: logged and skipped */
#define VC_DNSD_REJECTED   3  /* securityGroup.allow false: skipped */
#define VC_DNSD_EMPTY      4  /* read == 0: the loop returns */
#define VC_DNSD_MALFORMED  5  /* parsePackets threw InvalidDNSPacketException: the loop returns */
#define VC_DNSD_HOST       6  /* outside this entry point's shapes, run the Java path: a
                                 second packet in the datagram, more than VC_DNSD_MAXQ
                                 questions, a qname over 128 chars, a chain of more than
                                 16 compression pointers (nq = 0) */
#define VC_DNSD_MAXQ       4
typedef struct {
    uint8_t *status;          /* VC_DNSD_* (required) */
    int32_t *acl;             /* matched UDP rule index, -1 = default (optional) */
    uint8_t *nq;              /* questions evaluated (optional) */
    uint16_t *qtype;          /* [n][VC_DNSD_MAXQ] (optional) */
    uint8_t *kind;            /* [n][VC_DNSD_MAXQ] VC_DNS_* of question q < nq, 0 for the
                                 other slots (required) */
    int32_t *value;           /* [n][VC_DNSD_MAXQ] its value (required) */
} vc_dnsd_out;
/* With counters on (vc_counters_enable), a call counts the matched UDP rule
 * of every datagram (when out->acl is given) and the group of every question
 * classified VC_DNS_GROUP. */
int vc_dns_datagrams_dev(vc_ctx *ctx, const uint8_t *blob, const uint32_t *off, int64_t n,
                         const uint8_t *remote_family, const uint32_t *remote4,
                         const uint8_t *remote6, const uint16_t *remote_port,
                         const vc_dnsd_out *out, void *stream);
int vc_dns_datagrams(vc_ctx *ctx, const uint8_t *blob, const uint32_t *off, int64_t n,
                     const uint8_t *remote_family, const uint32_t *remote4,
                     const uint8_t *remote6, const uint16_t *remote_port,
                     const vc_dnsd_out *out);

/* ------------------------------------------------------------------------ */
/* TLS certificate choice by SNI (SSLContextHolder.java:47-186)             */
/* ------------------------------------------------------------------------ */
/* Replaces SSLContextHolder.add(ctx, certs) for a whole holder list: holder
 * h (add() order, 0..n_holders-1) lists the names of its certificates --
 * each certificate's subject CN (if any) and its SAN dNSNames (type 2) --
 * as names[i] with holder[i] == h; order within a holder is irrelevant.  A
 * name "*.S" is a wildcard (compare(), :171-186).  Names are raw bytes,
 * compared case-sensitively as Java's String.equals/endsWith do. */
int vc_compile_certs(vc_ctx *ctx, const char *const *names, const int32_t *name_lens,
                     const int32_t *holder, int n_names, int n_holders);
/* SSLContextHolder.choose(sni) per SNI (:51-63): the holder index; 0 (the
 * default first holder) for one holder, a null SNI (sni_null[i] != 0) or no
 * match; -1 (null) when there are no holders.  SNIs as blob + uint32
 * offsets (n + 1 entries); sni_null may be NULL.  Device pointers. */
int vc_cert_choose_dev(vc_ctx *ctx, const uint8_t *sni_blob, const uint32_t *sni_off,
                       const uint8_t *sni_null, int64_t n, int32_t *out_holder, void *stream);
int vc_cert_choose(vc_ctx *ctx, const uint8_t *sni_blob, const uint32_t *sni_off,
                   const uint8_t *sni_null, int64_t n, int32_t *out_holder);

/* ------------------------------------------------------------------------ */
/* Combined per-packet pipeline: ACL -> route -> host      */
/* ------------------------------------------------------------------------ */
/* For each IPv4 packet: out_acl = SecurityGroup.allow index on (proto, src,
 * dport), out_route = RouteTable.lookup(dst) index, out_group =
 * pool_group[host_id] (the per-pass classified hostname pool of n_pool
 * entries from vc_hint_search_dev; host_id >= n_pool, e.g. 0xFFFFFFFF for
 * "no hostname", -> -1).  out_allow optional. */
int vc_pipeline_v4_dev(vc_ctx *ctx, const uint8_t *proto, const uint32_t *src4,
                       const uint32_t *dst4, const uint16_t *dport, const uint32_t *host_id,
                       const int32_t *pool_group, int64_t n_pool, int64_t n, int32_t *out_acl,
                       int32_t *out_route, int32_t *out_group, uint8_t *out_allow, void *stream);
/* Same, plus an optional hipEvent_t recorded on `stream` right after the
 * classify kernel, before the hit-counter passes that follow it when
 * counters are enabled (the kernel counts the ACL and the route/group
 * buckets itself; the passes finish the large counter spaces). */
int vc_pipeline_v4_dev_ex(vc_ctx *ctx, const uint8_t *proto, const uint32_t *src4,
                          const uint32_t *dst4, const uint16_t *dport, const uint32_t *host_id,
                          const int32_t *pool_group, int64_t n_pool, int64_t n, int32_t *out_acl,
                          int32_t *out_route, int32_t *out_group, uint8_t *out_allow, void *stream,
                          void *kernel_done_event);

/* The general pipeline: IPv4 and IPv6 packets in one batch, as the vswitch
 * drain loop (core/src/main/java/vswitch/Switch.java:744-776) hands them to
 * L3.route (core/src/main/java/vswitch/stack/L3.java:423-444).  Every array
 * has n entries in packet order (the layout vc_parse_packets writes); the
 * fields a packet's family does not use are ignored. */
typedef struct vc_packets {
    const uint8_t *family;        /* 4 or 6 per packet: whether the packet's IP objects are
                                     IPv4 or IPv6 instances -- RouteTable.lookup's `instanceof
                                     IPv4` dispatch (RouteTable.java:44-58), so an IPv4-mapped
                                     ::ffff:a.b.c.d address is family 6 and goes to rulesV6 and
                                     the v6 ACL projection.  NULL = every packet IPv4 */
    const uint8_t *proto;         /* VC_PROTO_TCP selects tcpRules */
    const uint32_t *src4, *dst4;  /* IPv4 packets, IP.ipv4Bytes2Int order */
    const uint8_t *src6, *dst6;   /* IPv6 packets, 16 bytes each, 16-byte aligned; may be NULL
                                     only when family is NULL */
    const uint16_t *dport;        /* SecurityGroup.allow's port */
    const uint32_t *host_id;      /* index into the classified hostname pool (pool_group, from
                                     vc_hint_search); NULL = no hostname stage (group -1, the
                                     group counters untouched) */
} vc_packets;

typedef struct vc_pipeline_out {
    int32_t *acl;                 /* SecurityGroup.allow: first matching rule index, -1 = default */
    int32_t *route;               /* RouteTable.lookup: index in rulesV4 (family 4) or rulesV6
                                     (family 6), -1 = null */
    int32_t *group;               /* pool_group[host_id]; -1 for host_id >= n_pool */
    uint8_t *allow;               /* optional: the boolean SecurityGroup.allow returns */
} vc_pipeline_out;

/* Device pointers, asynchronous on `stream`.  With counters enabled the
 * classify kernel counts the ACL hits and the route/group buckets itself;
 * the passes that finish the large counter spaces run on `count_stream`
 * (ordered after the kernel) when it is not NULL -- so a caller's next batch
 * can overlap them -- else on `stream`.  kernel_done_event (a hipEvent_t,
 * optional) is recorded on `stream` right after the classify kernel. */
int vc_pipeline_dev(vc_ctx *ctx, const vc_packets *in, int64_t n, const int32_t *pool_group,
                    int64_t n_pool, const vc_pipeline_out *out, void *stream, void *count_stream,
                    void *kernel_done_event);
/* vc_pipeline_dev with the IPv6 addresses compacted: src6 / dst6 hold n6
 * rows, row k the addresses of the batch's k-th family-6 packet (packet
 * order); family is required.  An IPv6 packet's addresses then share cache
 * lines with the next IPv6 packets' instead of sitting in rows no IPv4
 * packet reads.  The arrays must be aligned as the vector kernels load them:
 * src4 / dst4 / host_id and the int32 outputs 16 bytes, family / proto /
 * allow 4 bytes, dport 8 bytes, src6 / dst6 16 bytes.  n6 must be the
 * number of family-6 packets: with fewer rows the IPv6 packets past them
 * get unspecified results (no memory outside the rows is read). */
int vc_pipeline_c6_dev(vc_ctx *ctx, const vc_packets *in, int64_t n, int64_t n6,
                       const int32_t *pool_group, int64_t n_pool, const vc_pipeline_out *out,
                       void *stream, void *count_stream, void *kernel_done_event);
/* Host pointers (every array in `in` and `out`, and pool_group), synchronous.
 * Zero-copy for an IPv4-only batch (no family array) whose every array is
 * inside a vc_host_register'ed buffer (the kernel reads and writes across
 * PCIe directly); otherwise the batch is staged through device memory in
 * chunks on two streams (a mixed batch's scattered 16-byte IPv6 reads ran at
 * 7 GB/s zero-copy).  All chunks classify against the snapshots current when
 * the call started. */
int vc_pipeline(vc_ctx *ctx, const vc_packets *in, int64_t n, const int32_t *pool_group,
                int64_t n_pool, const vc_pipeline_out *out);
/* vc_pipeline with compact IPv6 rows (as vc_pipeline_c6_dev: src6 / dst6
 * hold n6 rows, row k the k-th family-6 packet's addresses; family
 * required).  Zero-copy when every array is registered and aligned as
 * vc_pipeline_c6_dev asks (the rows are read coalesced); otherwise staged
 * in chunks, each chunk's rows found by counting its family-6 packets, and
 * only the n6 rows cross PCIe instead of n.  Both paths first count the
 * family array's IPv6 packets and return VC_EINVAL, before any output is
 * written, when that count is not n6. */
int vc_pipeline_c6(vc_ctx *ctx, const vc_packets *in, int64_t n, int64_t n6,
                   const int32_t *pool_group, int64_t n_pool, const vc_pipeline_out *out);

/* ------------------------------------------------------------------------ */
/* Server choice after the group match, method == source:                    */
/* base/src/main/java/vproxybase/component/svrgroup/ServerGroup.java         */
/* ------------------------------------------------------------------------ */
typedef struct {
    uint8_t ip[16];     /* server address bytes (IPv4: first 4) */
    int32_t ip_len;     /* 4 (IPv4 server) or 16 */
    int32_t port;
    int32_t weight;     /* ServerHandle.weight; <= 0 never chosen (:628) */
    int32_t healthy;    /* ServerHandle.healthy */
} vc_server;

/* The servers of every group of the compiled Upstream, each group's list in
 * ServerGroup.getServerHandles() order: group g owns servers[group_off[g] ..
 * group_off[g + 1]).  Builds the three source-hash lists of each group
 * (sourceReset, ServerGroup.java:620-664: weight > 0, sorted by address
 * length, signed address bytes, port; all / IPv4-only / IPv6-only). */
int vc_compile_servers(vc_ctx *ctx, const vc_server *servers, const int32_t *group_off,
                       int n_groups);
/* Health-check result changed: healthy[i] for every server (same indexing
 * as vc_compile_servers).  Publishes a new snapshot (copy-on-write): batches
 * issued afterwards see it, a batch already in flight -- every chunk of a
 * chunked host call included -- keeps the health it started with.  The call
 * rebuilds the lists' per-position answers on the host (O(servers)) and
 * uploads them, so a classify call's probe is one table read. */
int vc_servers_set_health(vc_ctx *ctx, const uint8_t *healthy, int64_t n_servers);
#define VC_SOURCE_ALL   0   /* ServerGroup.next(source)      :422-434 */
#define VC_SOURCE_IPV4  4   /* ServerGroup.nextIPv4(source)  :436-448 */
#define VC_SOURCE_IPV6  6   /* ServerGroup.nextIPv6(source)  :450-462 */
/* sourceHashGet per item (ServerGroup.java:464-490): group[i] (e.g. the
 * searchForGroup result; -1 or out of range -> -1) and the client address;
 * out_server[i] = index into that group's server list, or -1 for null. */
int vc_source_select_v4_dev(vc_ctx *ctx, const int32_t *group, const uint32_t *src4, int64_t n,
                            int view, int32_t *out_server, void *stream);
int vc_source_select_v6_dev(vc_ctx *ctx, const int32_t *group, const uint8_t *src6, int64_t n,
                            int view, int32_t *out_server, void *stream);
int vc_source_select_v4(vc_ctx *ctx, const int32_t *group, const uint32_t *src4, int64_t n,
                        int view, int32_t *out_server);
int vc_source_select_v6(vc_ctx *ctx, const int32_t *group, const uint8_t *src6, int64_t n,
                        int view, int32_t *out_server);

/* ------------------------------------------------------------------------ */
/* Header extraction from raw frames: the vswitch's  */
/* parse chain base/src/main/java/vpacket/: VXLanPacket.from (:16-33) ->     */
/* EthernetPacket.from (:14-50) -> ArpPacket / Ipv4Packet (:28-101) /         */
/* Ipv6Packet (:24-106) .from -> TcpPacket (:164-227) / IcmpPacket .from.    */
/* ------------------------------------------------------------------------ */
#define VC_LAYER_VXLAN  0   /* frames are VXLAN UDP payloads (Switch.java:679-690) */
#define VC_LAYER_ETHER  1
#define VC_LAYER_IPV4   4
#define VC_LAYER_IPV6   6

#define VC_PKT_OK          0   /* `from` returned null */
#define VC_PKT_ERR_VXLAN   1   /* VXLAN header too short */
#define VC_PKT_ERR_ETHER   2   /* Ethernet too short, or an ARP error */
#define VC_PKT_ERR_IP      3   /* IP/TCP/ICMP error (layer VC_LAYER_IPV4/6 only; under
                                  Ethernet the IP payload is kept as bytes: VC_L3_BAD_IP) */
#define VC_PKT_EXCEPTION   4   /* the Java parser throws (a TCP option of length 0 or 1) */
#define VC_PKT_LOOP        5   /* the Java parser never returns (IPv6 extension header whose
                                  next header is an extension header, Ipv6Packet.java:63-78) */

#define VC_L3_OTHER   0   /* PacketBytes */
#define VC_L3_ARP     1
#define VC_L3_IPV4    4
#define VC_L3_BAD_IP  5   /* IP ether type whose parse failed (EthernetPacket.java:36-45) */
#define VC_L3_IPV6    6

#define VC_L4_BYTES   0   /* PacketBytes (UDP included, as in the reference) */
#define VC_L4_ICMP    1
#define VC_L4_TCP     6
#define VC_L4_ICMPV6  58

#define VC_TCPOPT_END  0
#define VC_TCPOPT_NOP  1
#define VC_TCPOPT_MSS  2
#define VC_TCPOPT_WS   3

/* Per-frame outputs (SoA); any pointer may be NULL.  Fields a frame does
 * not have are 0.  src4/dst4 feed the ACL / route / pipeline entry points
 * directly (IP.ipv4Bytes2Int order). */
typedef struct {
    uint8_t *status;       /* VC_PKT_* */
    uint8_t *l3;           /* VC_L3_* */
    uint8_t *l4;           /* VC_L4_* */
    uint8_t *proto;        /* IPv4 protocol / IPv6 final next header */
    uint32_t *vni;         /* VXLAN vni */
    uint16_t *ether_type;
    uint32_t *src4, *dst4; /* IPv4 addresses */
    uint8_t *src6, *dst6;  /* IPv6 addresses, 16 bytes per frame */
    uint16_t *sport, *dport;   /* TCP ports */
} vc_pkt_out;

/* frames: blob + uint32 offsets (n + 1 entries).  Device pointers in `out`. */
int vc_parse_packets_dev(vc_ctx *ctx, const uint8_t *blob, const uint32_t *off, int64_t n,
                         int layer, const vc_pkt_out *out, void *stream);
/* Host pointers (blob, off and every array in `out`). */
int vc_parse_packets(vc_ctx *ctx, const uint8_t *blob, const uint32_t *off, int64_t n, int layer,
                     const vc_pkt_out *out);

/* Switch.PacketHandler.readable's per-datagram classification in one pass
 * (core/src/main/java/vswitch/Switch.java:679-700,744-776): for datagram i
 * from sender remote[i],
 *   out_allow[i] / out_acl[i] = bareVXLanAccess.allow(Protocol.UDP, remote,
 *       bind_port) -- the compiled SecurityGroup's UDP list (index, -1 =
 *       defaultAllow decided);
 *   `out` = VXLanPacket.from(payload) etc., as vc_parse_packets;
 *   out_route[i] = ctx.table.routeTable.lookup(inner dst) (L3.java:423-444),
 *       where ctx.table is the switch's Table of the packet's VNI
 *       (Switch.java:560-566 tables.get(vni)): an index in that table's
 *       rulesV4 (inner IPv4) or rulesV6 (inner IPv6); -1 when none matches,
 *       the datagram is denied, or it does not parse into an IP packet;
 *       VC_SWITCH_NO_TABLE when the datagram parsed and was allowed but its
 *       VNI has no table (inputVXLan drops it).  The per-VNI tables come
 *       from vc_compile_vni_routes; a context without them routes every
 *       packet through the single table of vc_compile_routes (a one-network
 *       switch).
 * Precondition: the batch holds only datagrams for which
 * VProxyEncryptedPacket.from failed (Switch.java:648-679): user-iface
 * traffic is decrypted and routed by the Java path first, since its
 * bareVXLanAccess check and bare-VXLAN parse never run in the reference.
 * The switch's further per-packet decisions (remote-switch ifaces, MAC
 * checks, synthetic IPs, hop limit) stay with the caller.  remote_family:
 * 4/6 per datagram (NULL = all IPv4); remote4 / remote6 (16-byte aligned)
 * as in vc_packets.  Any vc_pkt_out pointer and out_acl / out_allow may be
 * NULL; out_route is required.  Device pointers.
 * bind_port is constant for a switch, so the library keeps the UDP list's
 * IPv4 rules at that port as a small merged table: the first call with a
 * new bind_port on a compiled SecurityGroup builds it (a host build and a
 * small synchronous copy on the calling thread), and every later
 * vc_compile_acl builds it ahead for each bind_port used so far. */
int vc_switch_classify_dev(vc_ctx *ctx, const uint8_t *blob, const uint32_t *off, int64_t n,
                           int layer, const uint8_t *remote_family, const uint32_t *remote4,
                           const uint8_t *remote6, int bind_port, const vc_pkt_out *out,
                           int32_t *out_acl, uint8_t *out_allow, int32_t *out_route, void *stream);
/* Host pointers (every array), synchronous. */
int vc_switch_classify(vc_ctx *ctx, const uint8_t *blob, const uint32_t *off, int64_t n, int layer,
                       const uint8_t *remote_family, const uint32_t *remote4,
                       const uint8_t *remote6, int bind_port, const vc_pkt_out *out,
                       int32_t *out_acl, uint8_t *out_allow, int32_t *out_route);

/* ------------------------------------------------------------------------ */
/* Traffic-mirror filters (vmirror/FilterConfig.java:27-94, Mirror.java)   */
/* ------------------------------------------------------------------------ */
/* One FilterConfig as Mirror.parseAndLoadFilter builds it (Mirror.java:545-601).
 * Strings (origin, transport and application protocol names) are passed as
 * ids from an interning the caller keeps: equal strings <-> equal ids. */
typedef struct vc_mirror_filter {
    int32_t origin;                 /* OriginConfig.origin id */
    int32_t mirror;                 /* the origin's MirrorConfig (tap) as an index, 0..63 */
    int32_t has_mac_x, has_mac_y;   /* "mac", "mac2" */
    uint8_t mac_x[6], mac_y[6];
    int32_t has_net_x, has_net_y;   /* "network", "network2" */
    vc_net net_x, net_y;
    int32_t transport;              /* "transportLayerProtocol" id, -1 = null */
    int32_t has_port_x, has_port_y; /* "port", "port2": [min, max] */
    int32_t port_x[2], port_y[2];
    int32_t app;                    /* "applicationLayerProtocol" id, -1 = null */
} vc_mirror_filter;
/* Replaces the filter list Mirror.loadConfig publishes (Mirror.java:506-543).
 * VC_EINVAL: mirror outside 0..63, a port range with min > max, or a
 * network whose address / mask is not 4 or 16 bytes. */
int vc_compile_mirror(vc_ctx *ctx, const vc_mirror_filter *filters, int n);

/* MirrorData fields per item (MirrorData.java:13-26), SoA.  Any array may
 * be NULL: MACs then read as 00:00:00:00:00:00 / ff:ff:ff:ff:ff:ff (the
 * MirrorData defaults), a NULL length array makes every IP null, NULL id
 * arrays make every protocol null, NULL ports read 0. */
typedef struct vc_mirror_items {
    const uint8_t *mac_src, *mac_dst;         /* 6 bytes per item */
    const uint8_t *ip_src_len, *ip_dst_len;   /* 0 = null, 4 or 16 */
    const uint8_t *ip_src, *ip_dst;           /* 16 bytes per item (IPv4 in the first 4) */
    const int32_t *transport;                 /* id, -1 = null */
    const int32_t *port_src, *port_dst;
    const int32_t *app;                       /* id, -1 = null */
} vc_mirror_items;
/* Mirror.mirror(MirrorData) filter step (Mirror.java:89-118): per item the
 * set of mirrors (bit m = MirrorConfig m) whose filters of `origin` match,
 * at the level the item's null fields select (ether / ip / transport /
 * application).  Device pointers (every array in `items` and out); ip_src /
 * ip_dst 16-byte aligned, mac_src / mac_dst 2-byte aligned (VC_EINVAL
 * otherwise; the host form stages any alignment). */
int vc_mirror_match_dev(vc_ctx *ctx, int32_t origin, const vc_mirror_items *items, int64_t n,
                        uint64_t *out_mirrors, void *stream);
int vc_mirror_match(vc_ctx *ctx, int32_t origin, const vc_mirror_items *items, int64_t n,
                    uint64_t *out_mirrors);
/* Mirror.switchPacket (Mirror.java:73-87) on raw frames (layer VC_LAYER_VXLAN
 * or VC_LAYER_ETHER): parse as vc_parse_packets, then matchIp on IPv4/IPv6
 * packets and matchEthernet on the rest; 0 for frames the parse rejects. */
int vc_mirror_switch_dev(vc_ctx *ctx, int32_t origin, const uint8_t *blob, const uint32_t *off,
                         int64_t n, int layer, uint64_t *out_mirrors, void *stream);
int vc_mirror_switch(vc_ctx *ctx, int32_t origin, const uint8_t *blob, const uint32_t *off,
                     int64_t n, int layer, uint64_t *out_mirrors);

/* ------------------------------------------------------------------------ */
/* Host buffers                                                             */
/* ------------------------------------------------------------------------ */
/* Page-lock and map a caller buffer (e.g. a Java direct ByteBuffer, once per
 * buffer, SURVEY.md §8(b) "Buffers").  When every buffer of a plain ACL /
 * route / source call is registered, the kernel reads and writes them across
 * PCIe directly (zero-copy, both directions at once); otherwise the call
 * copies through device staging in chunks. */
int vc_host_register(void *p, int64_t bytes);
int vc_host_unregister(void *p);

/* ------------------------------------------------------------------------ */
/* Per-rule hit counters (no reference counterpart)          */
/* ------------------------------------------------------------------------ */
#define VC_COUNTERS_ACL    0  /* [tcp rules][udp rules][tcp default][udp default] */
#define VC_COUNTERS_ROUTE  1  /* [v4 rules][v6 rules][v4 null][v6 null] */
#define VC_COUNTERS_GROUP  2  /* [handles][null] */
/* When enabled, every classify call adds its hits into device-resident uint64
 * counters of the current snapshot (reset when a table is recompiled). */
int vc_counters_enable(vc_ctx *ctx, int on);
/* Device pointer + length of a counter array (for an RCCL all-reduce). */
int vc_counters_device(vc_ctx *ctx, int kind, uint64_t **dev_ptr, int64_t *n);
int vc_counters_read(vc_ctx *ctx, int kind, uint64_t *host, int64_t n);
int vc_counters_reset(vc_ctx *ctx);
/* Replicated tables (no reference counterpart): a 64-bit
 * digest of the compiled image of the current snapshot, kind VC_COUNTERS_ACL
 * (SecurityGroup), _ROUTE (RouteTable) or _GROUP (Upstream).  Ranks that
 * sum hit counters check first that they compiled identical tables; equal
 * rule lists give equal digests on any host.  The vc_digest_* forms build
 * the same images in host memory only (no device, no context). */
int vc_table_digest(vc_ctx *ctx, int kind, uint64_t *digest);
int vc_digest_acl(const vc_acl_rule *tcp, int n_tcp, const vc_acl_rule *udp, int n_udp,
                  int default_allow, uint64_t *digest);
int vc_digest_routes(const vc_net *v4, int n4, const vc_net *v6, int n6, uint64_t *digest);
int vc_digest_upstream(const vc_group_annos *groups, int n, uint64_t *digest);
/* Add the hits of an already-computed output array to the counters of the
 * current snapshot (what vc_counters_enable does automatically after each
 * classify call; exposed so callers can schedule the counting pass):
 *   VC_COUNTERS_ACL   out = out_idx,   aux = proto (required)
 *   VC_COUNTERS_ROUTE out = route out, family = 4 or 6, aux = NULL
 *   VC_COUNTERS_GROUP out = group out (hint / pipeline), aux = NULL; or
 *                     out = DNS out_value with aux = DNS out_kind. */
int vc_counters_add_dev(vc_ctx *ctx, int kind, const int32_t *out, const uint8_t *aux, int family,
                        int64_t n, void *stream);

/* ------------------------------------------------------------------------ */
/* Prometheus text exposition                       */
/* ------------------------------------------------------------------------ */
/* Text functions write NUL-terminated text into (buf, cap) and set *len to
 * its length; VC_ENOMEM (and *len = the length needed) when cap <= *len.    */
#define VC_METRIC_COUNTER 0   /* prometheus/Counter.java */
#define VC_METRIC_GAUGE   1   /* prometheus/Gauge.java */
typedef struct vc_metric {
    const char *metric;
    int32_t type;                    /* VC_METRIC_* */
    int32_t n_labels;                /* a repeated key: the later value wins */
    const char *const *label_keys;
    const char *const *label_values; /* raw; quoted as Metric's constructor does */
    int64_t value;
} vc_metric;
/* Metrics.toString (prometheus/Metrics.java:27-64): metrics given in
 * creation order, help messages as registerHelpMessage (later wins). */
int vc_prometheus_format(const vc_metric *metrics, int32_t n, const char *const *help_metric,
                         const char *const *help_text, int32_t n_help, char *buf, int64_t cap,
                         int64_t *len);
/* The hit counters of the VC_COUNTERS_* layouts above (host arrays; NULL
 * skips a kind) as security_group_rule_hit_count{protocol,rule},
 * route_table_rule_hit_count{family,rule} and
 * upstream_server_group_hit_count{group}, each added through the rules of
 * GlobalInspection.addMetric (GlobalInspection.java:118-125) with
 * `extra_labels` parsed as getExtraLabels (GlobalInspection.java:95-116):
 * "k1=v1,k2=v2"; VC_EINVAL for a piece without '='. */
int vc_prometheus_hits(const uint64_t *acl, int n_tcp, int n_udp, const uint64_t *route, int n4,
                       int n6, const uint64_t *group, int n_groups, const char *extra_labels,
                       char *buf, int64_t cap, int64_t *len);
/* Same over the context's current device counters (synchronises). */
int vc_counters_prometheus(vc_ctx *ctx, const char *extra_labels, char *buf, int64_t cap,
                           int64_t *len);

/* ------------------------------------------------------------------------ */
/* Control-plane mirrors (host only, no GPU): the reference's list-ordering  */
/* and validation rules, so a caller can keep the exact Java list order.    */
/* ------------------------------------------------------------------------ */
typedef struct vc_secgroup vc_secgroup;
/* new SecurityGroup(alias, defaultAllow) (SecurityGroup.java:21-24) */
int vc_secgroup_new(const char *alias, int default_allow, vc_secgroup **out);
void vc_secgroup_free(vc_secgroup *sg);
int vc_secgroup_set_default(vc_secgroup *sg, int default_allow);
/* SecurityGroup.addRule (SecurityGroup.java:56-83): VC_EEXIST on duplicate
 * alias or duplicate (network, protocol, minPort, maxPort). */
int vc_secgroup_add_rule(vc_secgroup *sg, const char *alias, const vc_net *net, int proto,
                         int min_port, int max_port, int allow);
/* SecurityGroup.removeRule (SecurityGroup.java:85-103): VC_ENOTFOUND. */
int vc_secgroup_remove_rule(vc_secgroup *sg, const char *alias);
/* Rule counts and list export in list order (proto = VC_PROTO_TCP / UDP). */
int vc_secgroup_rules(const vc_secgroup *sg, int proto, vc_acl_rule *out, int cap);
int vc_secgroup_compile(vc_ctx *ctx, const vc_secgroup *sg);

typedef struct vc_routetable vc_routetable;
/* new RouteTable() (RouteTable.java:25-28) when v4net == NULL, else
 * new RouteTable(Table) seeding "default"/"default-v6" (RouteTable.java:30-42). */
int vc_routetable_new(const vc_net *v4net, const vc_net *v6net, int vni, vc_routetable **out);
void vc_routetable_free(vc_routetable *rt);
/* RouteTable.addRule (RouteTable.java:68-154) incl. the insertion-order
 * heuristic.  via_ip NULL -> RouteRule(alias, net, toVni); else
 * RouteRule(alias, net, ip) (via_len 4/16).  VC_EEXIST / VC_EXEXC as Java. */
int vc_routetable_add_rule(vc_routetable *rt, const char *alias, const vc_net *net, int to_vni,
                           const uint8_t *via_ip, int via_len);
/* Bulk insert of vni rules in the given order.  Exact same final lists as
 * repeated vc_routetable_add_rule; O(n log n) when every insert is no
 * shorter than the rules already present, otherwise
 * falls back to the per-rule heuristic. Aliases are "<prefix><i>".
 * Returns 1 when the bulk path ran, 0 for the per-rule path, <0 on error. */
int vc_routetable_add_rules(vc_routetable *rt, const char *alias_prefix, const vc_net *nets,
                            int n, int to_vni);
/* RouteTable.delRule (RouteTable.java:156-172) */
int vc_routetable_del_rule(vc_routetable *rt, const char *alias);
/* family 4 -> rulesV4, 6 -> rulesV6; returns count (writes up to cap). */
int vc_routetable_rules(const vc_routetable *rt, int family, vc_net *out, int cap);
int vc_routetable_compile(vc_ctx *ctx, const vc_routetable *rt);
/* The switch's tables: each RouteTable under the VNI it was created with
 * (vc_routetable_new), as vc_compile_vni_routes. */
int vc_routetables_compile_vni(vc_ctx *ctx, const vc_routetable *const *tables, int n);

#ifdef __cplusplus
}
#endif
#endif /* VCLASSIFY_H */

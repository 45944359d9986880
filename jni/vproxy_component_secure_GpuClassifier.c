/*
 * vproxy_component_secure_GpuClassifier.c -- the JNI shim a vproxy
 * maintainer adds next to base/src/main/c/vfd_posix_GeneralPosix.c, over the
 * plain C ABI of libvclassify (include/vclassify.h).  Java side:
 * jni/GpuClassifier.java (package vproxy.component.secure).
 *
 * Conventions follow the reference's vfdposix library:
 *   - native handles cross as jlong (vfd_posix_GeneralPosix.c:76-83);
 *   - batches are direct ByteBuffers resolved with GetDirectBufferAddress,
 *     zero-copy (vfd_posix_GeneralPosix.c:639-657); a caller registers each
 *     long-lived buffer once with registerBuffer (vc_host_register) so the
 *     GPU reads and writes it across PCIe directly;
 *   - every buffer is checked against the bytes the batch needs
 *     (GetDirectBufferCapacity) before the library sees it;
 *   - a failing call throws (exception.h:10-31): VC_EEXIST ->
 *     AlreadyExistException, VC_ENOTFOUND -> NotFoundException, VC_EXEXC ->
 *     XException, VC_EINVAL -> IllegalArgumentException, VC_ESTATE (nothing
 *     compiled yet) -> IllegalStateException, anything else (VC_EDEVICE,
 *     VC_ENOMEM) -> IOException, each with vc_last_error() as the message.
 *     GpuContext (jni/GpuContext.java) keys its fallback on the last two:
 *     IllegalStateException answers that one batch with the Java
 *     classifiers, IOException marks the context dead;
 *   - offsets buffers are not trusted: they must be non-decreasing from a
 *     non-negative first entry, so every item's bytes lie inside the span
 *     the blob's capacity is checked against (the GPU reads them at those
 *     offsets, on registered buffers straight from host memory).
 *
 * Built only where a JDK is present (jni/Makefile checks JAVA_HOME): this
 * image has no JDK, so tests/native/abi_c.c runs the same call sequence
 * from plain C99 instead.
 */
#include <jni.h>
#include <stdint.h>
#include <stdlib.h>

#include "vclassify.h"

static int jni_throw(JNIEnv *env, int rc) {
    const char *cls;
    jclass c;
    if (rc >= 0) return 0;
    cls = rc == VC_EEXIST    ? "vproxybase/util/exception/AlreadyExistException"
        : rc == VC_ENOTFOUND ? "vproxybase/util/exception/NotFoundException"
        : rc == VC_EXEXC     ? "vproxybase/util/exception/XException"
        : rc == VC_EINVAL    ? "java/lang/IllegalArgumentException"
        : rc == VC_ESTATE    ? "java/lang/IllegalStateException"
        : "java/io/IOException";
    c = (*env)->FindClass(env, cls);
    if (c) (*env)->ThrowNew(env, c, vc_last_error());
    return 1;
}

static void *addr(JNIEnv *env, jobject buf) {
    return buf ? (*env)->GetDirectBufferAddress(env, buf) : NULL;
}

/* Throws IllegalArgumentException(msg) once per call and sets *bad. */
static void refuse(JNIEnv *env, const char *msg, int *bad) {
    jclass c;
    if (*bad) return;
    *bad = 1;
    c = (*env)->FindClass(env, "java/lang/IllegalArgumentException");
    if (c) (*env)->ThrowNew(env, c, msg);
}

/* The address of direct buffer b when it holds at least `need` bytes (a
 * NULL buffer gives NULL: the argument is optional); otherwise throws
 * IllegalArgumentException once and sets *bad, so a short buffer never lets
 * the library read or write past it into JVM memory. */
static void *buf(JNIEnv *env, jobject b, int64_t need, int *bad) {
    jlong cap;
    if (*bad || !b) return NULL;
    cap = (*env)->GetDirectBufferCapacity(env, b);
    if (need >= 0 && cap >= 0 && (int64_t) cap >= need) return (*env)->GetDirectBufferAddress(env, b);
    refuse(env, "direct buffer smaller than the batch needs", bad);
    return NULL;
}

/* buf() for an argument the shim reads itself: a NULL buffer is refused
 * too when the batch needs bytes from it. */
static void *req(JNIEnv *env, jobject b, int64_t need, int *bad) {
    if (!*bad && !b && need > 0) refuse(env, "required direct buffer is null", bad);
    return buf(env, b, need, bad);
}

/* An offsets buffer of n + 1 ints (NULL allowed unless `required`):
 * off[0] >= 0 and off[i] <= off[i + 1], so item i's bytes
 * [off[i], off[i + 1]) lie inside [0, off[n]), the span end_of() sizes the
 * blob's capacity check by. */
static const int32_t *offsets(JNIEnv *env, jobject b, jint n, int required, int *bad) {
    const int32_t *o = required ? req(env, b, ((int64_t) n + 1) * 4, bad)
                                : buf(env, b, ((int64_t) n + 1) * 4, bad);
    jint i;
    if (!o) return NULL;
    if (o[0] < 0) {
        refuse(env, "offsets must start at a non-negative value", bad);
        return NULL;
    }
    for (i = 0; i < n; ++i)
        if (o[i + 1] < o[i]) {
            refuse(env, "offsets must be non-decreasing", bad);
            return NULL;
        }
    return o;
}

/* off[n] of a validated offsets buffer (0 if absent) */
static int64_t end_of(const int32_t *off, jint n) {
    return off && n >= 0 ? (int64_t) off[n] : 0;
}

#define CTX(h) ((vc_ctx *) (intptr_t) (h))

JNIEXPORT jlong JNICALL Java_vproxy_component_secure_GpuClassifier_create
  (JNIEnv *env, jclass self, jint device) {
    vc_ctx *ctx = NULL;
    (void) self;
    if (jni_throw(env, vc_create(device, &ctx))) return 0;
    return (jlong) (intptr_t) ctx;
}

JNIEXPORT void JNICALL Java_vproxy_component_secure_GpuClassifier_destroy
  (JNIEnv *env, jclass self, jlong ctx) {
    (void) env; (void) self;
    vc_destroy(CTX(ctx));
}

/* Snapshot pins: GpuContext's views (vc_pin_*).  A pin crosses as a jlong
 * like the context handle. */
JNIEXPORT jlong JNICALL Java_vproxy_component_secure_GpuClassifier_pinAcquire
  (JNIEnv *env, jclass self, jlong ctx, jint kinds) {
    vc_pin *pin = NULL;
    (void) self;
    if (jni_throw(env, vc_pin_acquire(CTX(ctx), (uint32_t) kinds, &pin))) return 0;
    return (jlong) (intptr_t) pin;
}

JNIEXPORT void JNICALL Java_vproxy_component_secure_GpuClassifier_bindPin
  (JNIEnv *env, jclass self, jlong ctx, jlong pin) {
    (void) self;
    jni_throw(env, vc_pin_bind(CTX(ctx), (const vc_pin *) (intptr_t) pin));
}

JNIEXPORT jlong JNICALL Java_vproxy_component_secure_GpuClassifier_pinGeneration
  (JNIEnv *env, jclass self, jlong pin, jint kind) {
    uint64_t g = 0;
    (void) self;
    if (jni_throw(env, vc_pin_generation((const vc_pin *) (intptr_t) pin, kind, &g))) return 0;
    return (jlong) g;
}

JNIEXPORT void JNICALL Java_vproxy_component_secure_GpuClassifier_pinRelease
  (JNIEnv *env, jclass self, jlong pin) {
    (void) env; (void) self;
    vc_pin_release((vc_pin *) (intptr_t) pin);
}

JNIEXPORT void JNICALL Java_vproxy_component_secure_GpuClassifier_registerBuffer
  (JNIEnv *env, jclass self, jobject b) {
    (void) self;
    jni_throw(env, vc_host_register(addr(env, b), (int64_t) (*env)->GetDirectBufferCapacity(env, b)));
}

JNIEXPORT void JNICALL Java_vproxy_component_secure_GpuClassifier_unregisterBuffer
  (JNIEnv *env, jclass self, jobject b) {
    (void) self;
    jni_throw(env, vc_host_unregister(addr(env, b)));
}

/* SecurityGroup: packed vc_acl_rule[] (52 B each) per protocol list, in list order */
JNIEXPORT void JNICALL Java_vproxy_component_secure_GpuClassifier_compileAcl
  (JNIEnv *env, jclass self, jlong ctx, jobject tcp, jint nTcp, jobject udp, jint nUdp,
   jboolean defaultAllow) {
    int bad = 0;
    const vc_acl_rule *t = buf(env, tcp, (int64_t) nTcp * (int64_t) sizeof(vc_acl_rule), &bad);
    const vc_acl_rule *u = buf(env, udp, (int64_t) nUdp * (int64_t) sizeof(vc_acl_rule), &bad);
    (void) self;
    if (bad) return;
    jni_throw(env, vc_compile_acl(CTX(ctx), t, nTcp, u, nUdp, defaultAllow ? 1 : 0));
}

/* SecurityGroup.allow(Protocol, IP, int) over n IPv4 / IPv6 items */
static void classify_acl(JNIEnv *env, jlong ctx, int fam, jobject proto, jobject src, jobject port,
                         jint n, jobject outIdx, jobject outAllow) {
    int bad = 0;
    const int64_t m = n;
    const uint8_t *p = buf(env, proto, m, &bad);
    const void *s = buf(env, src, m * (fam == 4 ? 4 : 16), &bad);
    const uint16_t *q = buf(env, port, m * 2, &bad);
    int32_t *oi = buf(env, outIdx, m * 4, &bad);
    uint8_t *oa = buf(env, outAllow, m, &bad);
    if (bad) return;
    jni_throw(env, fam == 4 ? vc_acl_classify_v4(CTX(ctx), p, s, q, n, oi, oa)
                            : vc_acl_classify_v6(CTX(ctx), p, s, q, n, oi, oa));
}

JNIEXPORT void JNICALL Java_vproxy_component_secure_GpuClassifier_classifyAclV4
  (JNIEnv *env, jclass self, jlong ctx, jobject proto, jobject src4, jobject port, jint n,
   jobject outIdx, jobject outAllow) {
    (void) self;
    classify_acl(env, ctx, 4, proto, src4, port, n, outIdx, outAllow);
}

JNIEXPORT void JNICALL Java_vproxy_component_secure_GpuClassifier_classifyAclV6
  (JNIEnv *env, jclass self, jlong ctx, jobject proto, jobject src6, jobject port, jint n,
   jobject outIdx, jobject outAllow) {
    (void) self;
    classify_acl(env, ctx, 6, proto, src6, port, n, outIdx, outAllow);
}

/* RouteTable: packed vc_net[] (40 B each) of rulesV4 and rulesV6, list order */
JNIEXPORT void JNICALL Java_vproxy_component_secure_GpuClassifier_compileRoutes
  (JNIEnv *env, jclass self, jlong ctx, jobject v4, jint n4, jobject v6, jint n6) {
    int bad = 0;
    const vc_net *a = buf(env, v4, (int64_t) n4 * (int64_t) sizeof(vc_net), &bad);
    const vc_net *b = buf(env, v6, (int64_t) n6 * (int64_t) sizeof(vc_net), &bad);
    (void) self;
    if (bad) return;
    jni_throw(env, vc_compile_routes(CTX(ctx), a, n4, b, n6));
}

/* Switch.tables: vni[n] ints; v4 / v6 packed vc_net[] of every table in
 * turn, split by the n + 1 int offsets v4Off / v6Off */
JNIEXPORT void JNICALL Java_vproxy_component_secure_GpuClassifier_compileVniRoutes
  (JNIEnv *env, jclass self, jlong ctx, jobject vni, jobject v4, jobject v4Off, jobject v6,
   jobject v6Off, jint n) {
    int bad = 0;
    const int32_t *k = buf(env, vni, (int64_t) n * 4, &bad);
    const int32_t *o4 = offsets(env, v4Off, n, 0, &bad);
    const int32_t *o6 = offsets(env, v6Off, n, 0, &bad);
    const vc_net *a = bad ? NULL : buf(env, v4, end_of(o4, n) * (int64_t) sizeof(vc_net), &bad);
    const vc_net *b = bad ? NULL : buf(env, v6, end_of(o6, n) * (int64_t) sizeof(vc_net), &bad);
    (void) self;
    if (bad) return;
    jni_throw(env, vc_compile_vni_routes(CTX(ctx), k, a, o4, b, o6, n));
}

static void lookup_route(JNIEnv *env, jlong ctx, int fam, jobject dst, jint n, jobject out) {
    int bad = 0;
    const void *d = buf(env, dst, (int64_t) n * (fam == 4 ? 4 : 16), &bad);
    int32_t *o = buf(env, out, (int64_t) n * 4, &bad);
    if (bad) return;
    jni_throw(env, fam == 4 ? vc_route_lookup_v4(CTX(ctx), d, n, o)
                            : vc_route_lookup_v6(CTX(ctx), d, n, o));
}

JNIEXPORT void JNICALL Java_vproxy_component_secure_GpuClassifier_lookupRouteV4
  (JNIEnv *env, jclass self, jlong ctx, jobject dst4, jint n, jobject out) {
    (void) self;
    lookup_route(env, ctx, 4, dst4, n, out);
}

JNIEXPORT void JNICALL Java_vproxy_component_secure_GpuClassifier_lookupRouteV6
  (JNIEnv *env, jclass self, jlong ctx, jobject dst6, jint n, jobject out) {
    (void) self;
    lookup_route(env, ctx, 6, dst6, n, out);
}

/* Upstream: packed vc_group_annos[] whose string slots hold offsets into
 * `strings` (-1 = null).  The offsets are rebased into pointers in a copy,
 * so the caller's buffer stays reusable for the next compile. */
JNIEXPORT void JNICALL Java_vproxy_component_secure_GpuClassifier_compileUpstream
  (JNIEnv *env, jclass self, jlong ctx, jobject groups, jint n, jobject strings) {
    int bad = 0;
    const vc_group_annos *g = req(env, groups, (int64_t) n * (int64_t) sizeof(vc_group_annos), &bad);
    const char *base = addr(env, strings);
    const int64_t cap = strings ? (int64_t) (*env)->GetDirectBufferCapacity(env, strings) : 0;
    vc_group_annos *c;
    jint i;
    (void) self;
    if (bad) return;
    c = malloc(sizeof(vc_group_annos) * (size_t) (n > 0 ? n : 1));
    if (!c) {
        jni_throw(env, VC_ENOMEM);
        return;
    }
    for (i = 0; i < n; ++i) {
        const vc_annos *src[2] = {&g[i].handle, &g[i].group};
        vc_annos *dst[2] = {&c[i].handle, &c[i].group};
        int k;
        for (k = 0; k < 2; ++k) {
            const intptr_t h = (intptr_t) src[k]->host, u = (intptr_t) src[k]->uri;
            *dst[k] = *src[k];
            if ((h >= 0 && (!base || src[k]->host_len < 0 || h + src[k]->host_len > cap)) ||
                (u >= 0 && (!base || src[k]->uri_len < 0 || u + src[k]->uri_len > cap)))
                bad = 1;
            dst[k]->host = h < 0 ? NULL : base + h;
            dst[k]->uri = u < 0 ? NULL : base + u;
        }
    }
    if (bad) {
        jclass e = (*env)->FindClass(env, "java/lang/IllegalArgumentException");
        if (e) (*env)->ThrowNew(env, e, "annotation string outside the strings buffer");
    } else {
        jni_throw(env, vc_compile_upstream(CTX(ctx), c, n));
    }
    free(c);
}

/* Upstream.searchForGroup(Hint.ofHostPortUri(host, port, uri)): UTF-8 blobs +
 * int offsets (n + 1), null flags, ports */
JNIEXPORT void JNICALL Java_vproxy_component_secure_GpuClassifier_searchHints
  (JNIEnv *env, jclass self, jlong ctx, jobject hostBlob, jobject hostOff, jobject hostNull,
   jobject port, jobject uriBlob, jobject uriOff, jobject uriNull, jint n, jobject outGroup) {
    int bad = 0;
    const int64_t m = n;
    const int32_t *ho = offsets(env, hostOff, n, hostBlob != NULL, &bad);
    const int32_t *uo = offsets(env, uriOff, n, uriBlob != NULL, &bad);
    const uint8_t *hb = bad ? NULL : buf(env, hostBlob, end_of(ho, n), &bad);
    const uint8_t *ub = bad ? NULL : buf(env, uriBlob, end_of(uo, n), &bad);
    const uint8_t *hn = buf(env, hostNull, m, &bad);
    const uint16_t *p = buf(env, port, m * 2, &bad);
    const uint8_t *un = buf(env, uriNull, m, &bad);
    int32_t *o = buf(env, outGroup, m * 4, &bad);
    (void) self;
    if (bad) return;
    jni_throw(env, vc_hint_search(CTX(ctx), hb, (const uint32_t *) ho, hn, p, ub,
                                 (const uint32_t *) uo, un, n, o));
}

/* DNSServer: the hosts file text (Resolver.getHosts), then qname wire bytes */
JNIEXPORT void JNICALL Java_vproxy_component_secure_GpuClassifier_compileHostsText
  (JNIEnv *env, jclass self, jlong ctx, jobject text, jint len) {
    int bad = 0;
    const char *t = buf(env, text, len, &bad);
    (void) self;
    if (bad) return;
    jni_throw(env, vc_compile_hosts_text(CTX(ctx), t, len));
}

JNIEXPORT void JNICALL Java_vproxy_component_secure_GpuClassifier_classifyDns
  (JNIEnv *env, jclass self, jlong ctx, jobject qBlob, jobject qOff, jint n, jobject outKind,
   jobject outValue) {
    int bad = 0;
    const int32_t *o = offsets(env, qOff, n, 1, &bad);
    const uint8_t *b = bad ? NULL : req(env, qBlob, end_of(o, n), &bad);
    uint8_t *k = buf(env, outKind, n, &bad);
    int32_t *v = buf(env, outValue, (int64_t) n * 4, &bad);
    (void) self;
    if (bad) return;
    jni_throw(env, vc_dns_classify(CTX(ctx), b, (const uint32_t *) o, n, k, v));
}

/* HttpContext.connectionHint + Upstream.searchForGroup for the first read
 * of each new HTTP/1 connection (blob + n + 1 int offsets) */
JNIEXPORT void JNICALL Java_vproxy_component_secure_GpuClassifier_httpHint
  (JNIEnv *env, jclass self, jlong ctx, jobject heads, jobject off, jint n, jobject outGroup,
   jobject outKind) {
    int bad = 0;
    const int32_t *o = offsets(env, off, n, 1, &bad);
    const uint8_t *b = bad ? NULL : req(env, heads, end_of(o, n), &bad);
    int32_t *g = buf(env, outGroup, (int64_t) n * 4, &bad);
    uint8_t *k = buf(env, outKind, n, &bad);
    (void) self;
    if (bad) return;
    jni_throw(env, vc_http_hint(CTX(ctx), b, (const uint32_t *) o, n, g, k));
}

/* The vswitch drain loop's batch: ACL + route (+ pool group) per packet,
 * IPv4 and IPv6 together (vc_packets / vc_pipeline_out field order) */
JNIEXPORT void JNICALL Java_vproxy_component_secure_GpuClassifier_pipeline
  (JNIEnv *env, jclass self, jlong ctx, jobject family, jobject proto, jobject src4,
   jobject dst4, jobject src6, jobject dst6, jobject dport, jobject hostId, jobject poolGroup,
   jint nPool, jint n, jobject outAcl, jobject outRoute, jobject outGroup, jobject outAllow) {
    int bad = 0;
    const int64_t m = n;
    vc_packets in;
    vc_pipeline_out out;
    const int32_t *pool;
    (void) self;
    in.family = buf(env, family, m, &bad);
    in.proto = buf(env, proto, m, &bad);
    in.src4 = buf(env, src4, m * 4, &bad);
    in.dst4 = buf(env, dst4, m * 4, &bad);
    in.src6 = buf(env, src6, m * 16, &bad);
    in.dst6 = buf(env, dst6, m * 16, &bad);
    in.dport = buf(env, dport, m * 2, &bad);
    in.host_id = buf(env, hostId, m * 4, &bad);
    pool = buf(env, poolGroup, (int64_t) nPool * 4, &bad);
    out.acl = buf(env, outAcl, m * 4, &bad);
    out.route = buf(env, outRoute, m * 4, &bad);
    out.group = buf(env, outGroup, m * 4, &bad);
    out.allow = buf(env, outAllow, m, &bad);
    if (bad) return;
    jni_throw(env, vc_pipeline(CTX(ctx), &in, n, pool, nPool, &out));
}

/* pipeline with compact IPv6 rows: src6 / dst6 hold n6 rows, row k the k-th
 * family-6 packet's addresses (vc_pipeline_c6).  The drain loop fills them
 * as it meets IPv6 packets, so a batch that is mostly IPv4 moves 16 bytes
 * per IPv6 packet per address instead of 16 per packet, and runs zero-copy
 * over registered buffers. */
JNIEXPORT void JNICALL Java_vproxy_component_secure_GpuClassifier_pipelineCompact6
  (JNIEnv *env, jclass self, jlong ctx, jobject family, jobject proto, jobject src4,
   jobject dst4, jobject src6, jobject dst6, jint n6, jobject dport, jobject hostId,
   jobject poolGroup, jint nPool, jint n, jobject outAcl, jobject outRoute, jobject outGroup,
   jobject outAllow) {
    int bad = 0;
    const int64_t m = n, r = n6;
    vc_packets in;
    vc_pipeline_out out;
    const int32_t *pool;
    (void) self;
    if (n6 < 0) refuse(env, "negative IPv6 row count", &bad);
    in.family = req(env, family, m, &bad);
    in.proto = buf(env, proto, m, &bad);
    in.src4 = buf(env, src4, m * 4, &bad);
    in.dst4 = buf(env, dst4, m * 4, &bad);
    in.src6 = buf(env, src6, r * 16, &bad);
    in.dst6 = buf(env, dst6, r * 16, &bad);
    in.dport = buf(env, dport, m * 2, &bad);
    in.host_id = buf(env, hostId, m * 4, &bad);
    pool = buf(env, poolGroup, (int64_t) nPool * 4, &bad);
    out.acl = buf(env, outAcl, m * 4, &bad);
    out.route = buf(env, outRoute, m * 4, &bad);
    out.group = buf(env, outGroup, m * 4, &bad);
    out.allow = buf(env, outAllow, m, &bad);
    if (bad) return;
    jni_throw(env, vc_pipeline_c6(CTX(ctx), &in, n, n6, pool, nPool, &out));
}

/* ServerGroup source hashing */
JNIEXPORT void JNICALL Java_vproxy_component_secure_GpuClassifier_compileServers
  (JNIEnv *env, jclass self, jlong ctx, jobject servers, jobject groupOff, jint nGroups) {
    int bad = 0;
    const int32_t *o = offsets(env, groupOff, nGroups, 0, &bad);
    const vc_server *s = bad ? NULL
                             : buf(env, servers, end_of(o, nGroups) * (int64_t) sizeof(vc_server), &bad);
    (void) self;
    if (bad) return;
    jni_throw(env, vc_compile_servers(CTX(ctx), s, o, nGroups));
}

JNIEXPORT void JNICALL Java_vproxy_component_secure_GpuClassifier_setServerHealth
  (JNIEnv *env, jclass self, jlong ctx, jobject healthy, jint nServers) {
    int bad = 0;
    const uint8_t *h = buf(env, healthy, nServers, &bad);
    (void) self;
    if (bad) return;
    jni_throw(env, vc_servers_set_health(CTX(ctx), h, nServers));
}

JNIEXPORT void JNICALL Java_vproxy_component_secure_GpuClassifier_selectSourceV4
  (JNIEnv *env, jclass self, jlong ctx, jobject group, jobject src4, jint n, jint view,
   jobject outServer) {
    int bad = 0;
    const int32_t *g = buf(env, group, (int64_t) n * 4, &bad);
    const uint32_t *s = buf(env, src4, (int64_t) n * 4, &bad);
    int32_t *o = buf(env, outServer, (int64_t) n * 4, &bad);
    (void) self;
    if (bad) return;
    jni_throw(env, vc_source_select_v4(CTX(ctx), g, s, n, view, o));
}

/* The 12 vc_pkt_out buffers of `out` (null array or element = skip), each
 * checked against its field width */
static void pkt_out(JNIEnv *env, jobjectArray out, jint n, vc_pkt_out *o, int *bad) {
    static const int width[12] = {1, 1, 1, 1, 4, 2, 4, 4, 16, 16, 2, 2};
    void *f[12];
    int i;
    for (i = 0; i < 12; ++i)
        f[i] = out ? buf(env, (*env)->GetObjectArrayElement(env, out, i), (int64_t) n * width[i], bad)
                   : NULL;
    o->status = f[0]; o->l3 = f[1]; o->l4 = f[2]; o->proto = f[3]; o->vni = f[4];
    o->ether_type = f[5]; o->src4 = f[6]; o->dst4 = f[7]; o->src6 = f[8]; o->dst6 = f[9];
    o->sport = f[10]; o->dport = f[11];
}

/* Header extraction: `out` holds one direct buffer per vc_pkt_out field (null = skip) */
JNIEXPORT void JNICALL Java_vproxy_component_secure_GpuClassifier_parsePackets
  (JNIEnv *env, jclass self, jlong ctx, jobject blob, jobject off, jint n, jint layer,
   jobjectArray out) {
    int bad = 0;
    vc_pkt_out o;
    const int32_t *of = offsets(env, off, n, 1, &bad);
    const uint8_t *b = bad ? NULL : req(env, blob, end_of(of, n), &bad);
    (void) self;
    pkt_out(env, out, n, &o, &bad);
    if (bad) return;
    jni_throw(env, vc_parse_packets(CTX(ctx), b, (const uint32_t *) of, n, layer, &o));
}

/* Precondition (include/vclassify.h): only datagrams VProxyEncryptedPacket.from
 * rejected (Switch.java:648-679) */
JNIEXPORT void JNICALL Java_vproxy_component_secure_GpuClassifier_switchClassify
  (JNIEnv *env, jclass self, jlong ctx, jobject blob, jobject off, jint n, jint layer,
   jobject remoteFamily, jobject remote4, jobject remote6, jint bindPort, jobjectArray out,
   jobject outAcl, jobject outAllow, jobject outRoute) {
    int bad = 0;
    const int64_t m = n;
    vc_pkt_out o;
    const int32_t *of = offsets(env, off, n, 1, &bad);
    const uint8_t *b = bad ? NULL : req(env, blob, end_of(of, n), &bad);
    const uint8_t *rf = buf(env, remoteFamily, m, &bad);
    const uint32_t *r4 = buf(env, remote4, m * 4, &bad);
    const uint8_t *r6 = buf(env, remote6, m * 16, &bad);
    int32_t *oa = buf(env, outAcl, m * 4, &bad);
    uint8_t *ol = buf(env, outAllow, m, &bad);
    int32_t *orr = buf(env, outRoute, m * 4, &bad);
    (void) self;
    pkt_out(env, out, n, &o, &bad);
    if (bad) return;
    jni_throw(env, vc_switch_classify(CTX(ctx), b, (const uint32_t *) of, n, layer, rf, r4, r6,
                                      bindPort, &o, oa, ol, orr));
}

/* DNSServer's drain loop per datagram (DNSServer.java:457-500): out = status,
 * acl, nq, qtype, kind, value (vc_dnsd_out order; acl / nq / qtype may be null) */
JNIEXPORT void JNICALL Java_vproxy_component_secure_GpuClassifier_dnsDatagrams
  (JNIEnv *env, jclass self, jlong ctx, jobject blob, jobject off, jint n,
   jobject remoteFamily, jobject remote4, jobject remote6, jobject remotePort,
   jobjectArray out) {
    static const int width[6] = {1, 4, 1, 2 * VC_DNSD_MAXQ, VC_DNSD_MAXQ, 4 * VC_DNSD_MAXQ};
    int bad = 0;
    const int64_t m = n;
    vc_dnsd_out o;
    void *f[6];
    int i;
    const int32_t *of = offsets(env, off, n, 1, &bad);
    const uint8_t *b = bad ? NULL : req(env, blob, end_of(of, n), &bad);
    const uint8_t *rf = buf(env, remoteFamily, m, &bad);
    const uint32_t *r4 = buf(env, remote4, m * 4, &bad);
    const uint8_t *r6 = buf(env, remote6, m * 16, &bad);
    const uint16_t *rp = buf(env, remotePort, m * 2, &bad);
    (void) self;
    for (i = 0; i < 6; ++i)
        f[i] = out ? buf(env, (*env)->GetObjectArrayElement(env, out, i), m * width[i], &bad) : NULL;
    if (bad) return;
    o.status = f[0]; o.acl = f[1]; o.nq = f[2]; o.qtype = f[3]; o.kind = f[4]; o.value = f[5];
    jni_throw(env, vc_dns_datagrams(CTX(ctx), b, (const uint32_t *) of, n, rf, r4, r6, rp, &o));
}

/* SSLContextHolder: certificate names (UTF-8 blob + offsets) and holder per name */
JNIEXPORT void JNICALL Java_vproxy_component_secure_GpuClassifier_compileCerts
  (JNIEnv *env, jclass self, jlong ctx, jobject names, jobject off, jobject holder,
   jint nNames, jint nHolders) {
    int bad = 0;
    const int32_t *o = offsets(env, off, nNames, 1, &bad);
    const char *blob = bad ? NULL : req(env, names, end_of(o, nNames), &bad);
    const int32_t *h = req(env, holder, (int64_t) nNames * 4, &bad);
    const char **ptrs;
    int32_t *lens;
    jint i;
    (void) self;
    if (bad) return;
    ptrs = malloc(sizeof(char *) * (size_t) (nNames > 0 ? nNames : 1));
    lens = malloc(sizeof(int32_t) * (size_t) (nNames > 0 ? nNames : 1));
    if (!ptrs || !lens) {
        free(ptrs);
        free(lens);
        jni_throw(env, VC_ENOMEM);
        return;
    }
    for (i = 0; i < nNames; ++i) {
        ptrs[i] = blob + o[i];
        lens[i] = o[i + 1] - o[i];
    }
    jni_throw(env, vc_compile_certs(CTX(ctx), ptrs, lens, h, nNames, nHolders));
    free(ptrs);
    free(lens);
}

JNIEXPORT void JNICALL Java_vproxy_component_secure_GpuClassifier_chooseCerts
  (JNIEnv *env, jclass self, jlong ctx, jobject sni, jobject off, jobject isNull, jint n,
   jobject outHolder) {
    int bad = 0;
    const int32_t *o = offsets(env, off, n, 1, &bad);
    const uint8_t *s = bad ? NULL : req(env, sni, end_of(o, n), &bad);
    const uint8_t *z = buf(env, isNull, n, &bad);
    int32_t *h = buf(env, outHolder, (int64_t) n * 4, &bad);
    (void) self;
    if (bad) return;
    jni_throw(env, vc_cert_choose(CTX(ctx), s, (const uint32_t *) o, z, n, h));
}

/* Mirror filters: packed vc_mirror_filter[] (strings interned to ids in Java) */
JNIEXPORT void JNICALL Java_vproxy_component_secure_GpuClassifier_compileMirror
  (JNIEnv *env, jclass self, jlong ctx, jobject filters, jint n) {
    int bad = 0;
    const vc_mirror_filter *f = buf(env, filters, (int64_t) n * (int64_t) sizeof(vc_mirror_filter), &bad);
    (void) self;
    if (bad) return;
    jni_throw(env, vc_compile_mirror(CTX(ctx), f, n));
}

JNIEXPORT void JNICALL Java_vproxy_component_secure_GpuClassifier_mirrorSwitch
  (JNIEnv *env, jclass self, jlong ctx, jint origin, jobject blob, jobject off, jint n,
   jint layer, jobject outMirrors) {
    int bad = 0;
    const int32_t *o = offsets(env, off, n, 1, &bad);
    const uint8_t *b = bad ? NULL : req(env, blob, end_of(o, n), &bad);
    uint64_t *m = buf(env, outMirrors, (int64_t) n * 8, &bad);
    (void) self;
    if (bad) return;
    jni_throw(env, vc_mirror_switch(CTX(ctx), origin, b, (const uint32_t *) o, n, layer, m));
}

/* Per-rule hit counters as Prometheus text (GlobalInspection's /metrics) */
JNIEXPORT void JNICALL Java_vproxy_component_secure_GpuClassifier_enableCounters
  (JNIEnv *env, jclass self, jlong ctx, jboolean on) {
    (void) self;
    jni_throw(env, vc_counters_enable(CTX(ctx), on ? 1 : 0));
}

JNIEXPORT jstring JNICALL Java_vproxy_component_secure_GpuClassifier_countersPrometheus
  (JNIEnv *env, jclass self, jlong ctx, jstring extra) {
    const char *x = extra ? (*env)->GetStringUTFChars(env, extra, NULL) : NULL;
    int64_t len = 0;
    char *text = NULL;
    jstring s = NULL;
    int rc = vc_counters_prometheus(CTX(ctx), x, NULL, 0, &len);   /* size query */
    (void) self;
    if (rc == VC_ENOMEM) {
        text = malloc((size_t) len + 1);
        rc = text ? vc_counters_prometheus(CTX(ctx), x, text, len + 1, &len) : VC_ENOMEM;
    }
    if (x) (*env)->ReleaseStringUTFChars(env, extra, x);
    if (!jni_throw(env, rc) && text) s = (*env)->NewStringUTF(env, text);
    free(text);
    return s;
}

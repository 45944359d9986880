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
 *   - a failing call throws (exception.h:10-31): VC_EEXIST ->
 *     AlreadyExistException, VC_ENOTFOUND -> NotFoundException, VC_EXEXC ->
 *     XException, VC_EINVAL -> IllegalArgumentException, anything else ->
 *     IOException, each with vc_last_error() as the message.
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
        : "java/io/IOException";
    c = (*env)->FindClass(env, cls);
    if (c) (*env)->ThrowNew(env, c, vc_last_error());
    return 1;
}

static void *addr(JNIEnv *env, jobject buf) {
    return buf ? (*env)->GetDirectBufferAddress(env, buf) : NULL;
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

JNIEXPORT void JNICALL Java_vproxy_component_secure_GpuClassifier_registerBuffer
  (JNIEnv *env, jclass self, jobject buf) {
    (void) self;
    jni_throw(env, vc_host_register(addr(env, buf), (int64_t) (*env)->GetDirectBufferCapacity(env, buf)));
}

JNIEXPORT void JNICALL Java_vproxy_component_secure_GpuClassifier_unregisterBuffer
  (JNIEnv *env, jclass self, jobject buf) {
    (void) self;
    jni_throw(env, vc_host_unregister(addr(env, buf)));
}

/* SecurityGroup: packed vc_acl_rule[] (52 B each) per protocol list, in list order */
JNIEXPORT void JNICALL Java_vproxy_component_secure_GpuClassifier_compileAcl
  (JNIEnv *env, jclass self, jlong ctx, jobject tcp, jint nTcp, jobject udp, jint nUdp,
   jboolean defaultAllow) {
    (void) self;
    jni_throw(env, vc_compile_acl(CTX(ctx), addr(env, tcp), nTcp, addr(env, udp), nUdp,
                                 defaultAllow ? 1 : 0));
}

/* SecurityGroup.allow(Protocol, IP, int) over n IPv4 / IPv6 items */
JNIEXPORT void JNICALL Java_vproxy_component_secure_GpuClassifier_classifyAclV4
  (JNIEnv *env, jclass self, jlong ctx, jobject proto, jobject src4, jobject port, jint n,
   jobject outIdx, jobject outAllow) {
    (void) self;
    jni_throw(env, vc_acl_classify_v4(CTX(ctx), addr(env, proto), addr(env, src4), addr(env, port),
                                     n, addr(env, outIdx), addr(env, outAllow)));
}

JNIEXPORT void JNICALL Java_vproxy_component_secure_GpuClassifier_classifyAclV6
  (JNIEnv *env, jclass self, jlong ctx, jobject proto, jobject src6, jobject port, jint n,
   jobject outIdx, jobject outAllow) {
    (void) self;
    jni_throw(env, vc_acl_classify_v6(CTX(ctx), addr(env, proto), addr(env, src6), addr(env, port),
                                     n, addr(env, outIdx), addr(env, outAllow)));
}

/* RouteTable: packed vc_net[] (40 B each) of rulesV4 and rulesV6, list order */
JNIEXPORT void JNICALL Java_vproxy_component_secure_GpuClassifier_compileRoutes
  (JNIEnv *env, jclass self, jlong ctx, jobject v4, jint n4, jobject v6, jint n6) {
    (void) self;
    jni_throw(env, vc_compile_routes(CTX(ctx), addr(env, v4), n4, addr(env, v6), n6));
}

JNIEXPORT void JNICALL Java_vproxy_component_secure_GpuClassifier_lookupRouteV4
  (JNIEnv *env, jclass self, jlong ctx, jobject dst4, jint n, jobject out) {
    (void) self;
    jni_throw(env, vc_route_lookup_v4(CTX(ctx), addr(env, dst4), n, addr(env, out)));
}

JNIEXPORT void JNICALL Java_vproxy_component_secure_GpuClassifier_lookupRouteV6
  (JNIEnv *env, jclass self, jlong ctx, jobject dst6, jint n, jobject out) {
    (void) self;
    jni_throw(env, vc_route_lookup_v6(CTX(ctx), addr(env, dst6), n, addr(env, out)));
}

/* Upstream: packed vc_group_annos[] whose string pointers point into `strings`
 * (the Java side writes offsets; they are rebased here) */
JNIEXPORT void JNICALL Java_vproxy_component_secure_GpuClassifier_compileUpstream
  (JNIEnv *env, jclass self, jlong ctx, jobject groups, jint n, jobject strings) {
    vc_group_annos *g = addr(env, groups);
    const char *base = addr(env, strings);
    jint i;
    (void) self;
    for (i = 0; g && i < n; ++i) {            /* offsets (or -1 for null) -> pointers */
        vc_annos *a[2] = {&g[i].handle, &g[i].group};
        int k;
        for (k = 0; k < 2; ++k) {
            a[k]->host = (intptr_t) a[k]->host < 0 ? NULL : base + (intptr_t) a[k]->host;
            a[k]->uri = (intptr_t) a[k]->uri < 0 ? NULL : base + (intptr_t) a[k]->uri;
        }
    }
    jni_throw(env, vc_compile_upstream(CTX(ctx), g, n));
}

/* Upstream.searchForGroup(Hint.ofHostPortUri(host, port, uri)): UTF-8 blobs +
 * int offsets (n + 1), null flags, ports */
JNIEXPORT void JNICALL Java_vproxy_component_secure_GpuClassifier_searchHints
  (JNIEnv *env, jclass self, jlong ctx, jobject hostBlob, jobject hostOff, jobject hostNull,
   jobject port, jobject uriBlob, jobject uriOff, jobject uriNull, jint n, jobject outGroup) {
    (void) self;
    jni_throw(env, vc_hint_search(CTX(ctx), addr(env, hostBlob), addr(env, hostOff),
                                 addr(env, hostNull), addr(env, port), addr(env, uriBlob),
                                 addr(env, uriOff), addr(env, uriNull), n, addr(env, outGroup)));
}

/* DNSServer: the hosts file text (Resolver.getHosts), then qname wire bytes */
JNIEXPORT void JNICALL Java_vproxy_component_secure_GpuClassifier_compileHostsText
  (JNIEnv *env, jclass self, jlong ctx, jobject text, jint len) {
    (void) self;
    jni_throw(env, vc_compile_hosts_text(CTX(ctx), addr(env, text), len));
}

JNIEXPORT void JNICALL Java_vproxy_component_secure_GpuClassifier_classifyDns
  (JNIEnv *env, jclass self, jlong ctx, jobject qBlob, jobject qOff, jint n, jobject outKind,
   jobject outValue) {
    (void) self;
    jni_throw(env, vc_dns_classify(CTX(ctx), addr(env, qBlob), addr(env, qOff), n,
                                  addr(env, outKind), addr(env, outValue)));
}

/* The vswitch drain loop's batch: ACL + route (+ pool group) per packet,
 * IPv4 and IPv6 together (vc_packets / vc_pipeline_out field order) */
JNIEXPORT void JNICALL Java_vproxy_component_secure_GpuClassifier_pipeline
  (JNIEnv *env, jclass self, jlong ctx, jobject family, jobject proto, jobject src4,
   jobject dst4, jobject src6, jobject dst6, jobject dport, jobject hostId, jobject poolGroup,
   jint nPool, jint n, jobject outAcl, jobject outRoute, jobject outGroup, jobject outAllow) {
    vc_packets in;
    vc_pipeline_out out;
    (void) self;
    in.family = addr(env, family);
    in.proto = addr(env, proto);
    in.src4 = addr(env, src4);
    in.dst4 = addr(env, dst4);
    in.src6 = addr(env, src6);
    in.dst6 = addr(env, dst6);
    in.dport = addr(env, dport);
    in.host_id = addr(env, hostId);
    out.acl = addr(env, outAcl);
    out.route = addr(env, outRoute);
    out.group = addr(env, outGroup);
    out.allow = addr(env, outAllow);
    jni_throw(env, vc_pipeline(CTX(ctx), &in, n, addr(env, poolGroup), nPool, &out));
}

/* ServerGroup source hashing */
JNIEXPORT void JNICALL Java_vproxy_component_secure_GpuClassifier_compileServers
  (JNIEnv *env, jclass self, jlong ctx, jobject servers, jobject groupOff, jint nGroups) {
    (void) self;
    jni_throw(env, vc_compile_servers(CTX(ctx), addr(env, servers), addr(env, groupOff), nGroups));
}

JNIEXPORT void JNICALL Java_vproxy_component_secure_GpuClassifier_setServerHealth
  (JNIEnv *env, jclass self, jlong ctx, jobject healthy, jint nServers) {
    (void) self;
    jni_throw(env, vc_servers_set_health(CTX(ctx), addr(env, healthy), nServers));
}

JNIEXPORT void JNICALL Java_vproxy_component_secure_GpuClassifier_selectSourceV4
  (JNIEnv *env, jclass self, jlong ctx, jobject group, jobject src4, jint n, jint view,
   jobject outServer) {
    (void) self;
    jni_throw(env, vc_source_select_v4(CTX(ctx), addr(env, group), addr(env, src4), n, view,
                                      addr(env, outServer)));
}

/* Header extraction: `out` holds one direct buffer per vc_pkt_out field (null = skip) */
JNIEXPORT void JNICALL Java_vproxy_component_secure_GpuClassifier_parsePackets
  (JNIEnv *env, jclass self, jlong ctx, jobject blob, jobject off, jint n, jint layer,
   jobjectArray out) {
    vc_pkt_out o;
    void *f[12];
    int i;
    (void) self;
    for (i = 0; i < 12; ++i)
        f[i] = addr(env, (*env)->GetObjectArrayElement(env, out, i));
    o.status = f[0]; o.l3 = f[1]; o.l4 = f[2]; o.proto = f[3]; o.vni = f[4];
    o.ether_type = f[5]; o.src4 = f[6]; o.dst4 = f[7]; o.src6 = f[8]; o.dst6 = f[9];
    o.sport = f[10]; o.dport = f[11];
    jni_throw(env, vc_parse_packets(CTX(ctx), addr(env, blob), addr(env, off), n, layer, &o));
}

JNIEXPORT void JNICALL Java_vproxy_component_secure_GpuClassifier_switchClassify
  (JNIEnv *env, jclass self, jlong ctx, jobject blob, jobject off, jint n, jint layer,
   jobject remoteFamily, jobject remote4, jobject remote6, jint bindPort, jobjectArray out,
   jobject outAcl, jobject outAllow, jobject outRoute) {
    vc_pkt_out o;
    void *f[12];
    int i;
    (void) self;
    for (i = 0; i < 12; ++i)
        f[i] = out ? addr(env, (*env)->GetObjectArrayElement(env, out, i)) : NULL;
    o.status = f[0]; o.l3 = f[1]; o.l4 = f[2]; o.proto = f[3]; o.vni = f[4];
    o.ether_type = f[5]; o.src4 = f[6]; o.dst4 = f[7]; o.src6 = f[8]; o.dst6 = f[9];
    o.sport = f[10]; o.dport = f[11];
    jni_throw(env, vc_switch_classify(CTX(ctx), addr(env, blob), addr(env, off), n, layer,
                                      addr(env, remoteFamily), addr(env, remote4),
                                      addr(env, remote6), bindPort, &o, addr(env, outAcl),
                                      addr(env, outAllow), addr(env, outRoute)));
}

/* DNSServer's drain loop per datagram (DNSServer.java:457-500): out = status,
 * acl, nq, qtype, kind, value (vc_dnsd_out order; acl / nq / qtype may be null) */
JNIEXPORT void JNICALL Java_vproxy_component_secure_GpuClassifier_dnsDatagrams
  (JNIEnv *env, jclass self, jlong ctx, jobject blob, jobject off, jint n,
   jobject remoteFamily, jobject remote4, jobject remote6, jobject remotePort,
   jobjectArray out) {
    vc_dnsd_out o;
    void *f[6];
    int i;
    (void) self;
    for (i = 0; i < 6; ++i)
        f[i] = out ? addr(env, (*env)->GetObjectArrayElement(env, out, i)) : NULL;
    o.status = f[0]; o.acl = f[1]; o.nq = f[2]; o.qtype = f[3]; o.kind = f[4]; o.value = f[5];
    jni_throw(env, vc_dns_datagrams(CTX(ctx), addr(env, blob), addr(env, off), n,
                                    addr(env, remoteFamily), addr(env, remote4),
                                    addr(env, remote6), addr(env, remotePort), &o));
}

/* SSLContextHolder: certificate names (UTF-8 blob + offsets) and holder per name */
JNIEXPORT void JNICALL Java_vproxy_component_secure_GpuClassifier_compileCerts
  (JNIEnv *env, jclass self, jlong ctx, jobject names, jobject off, jobject holder,
   jint nNames, jint nHolders) {
    const char *blob = addr(env, names);
    const int32_t *o = addr(env, off);
    const char **ptrs = malloc(sizeof(char *) * (size_t) (nNames > 0 ? nNames : 1));
    int32_t *lens = malloc(sizeof(int32_t) * (size_t) (nNames > 0 ? nNames : 1));
    jint i;
    (void) self;
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
    jni_throw(env, vc_compile_certs(CTX(ctx), ptrs, lens, addr(env, holder), nNames, nHolders));
    free(ptrs);
    free(lens);
}

JNIEXPORT void JNICALL Java_vproxy_component_secure_GpuClassifier_chooseCerts
  (JNIEnv *env, jclass self, jlong ctx, jobject sni, jobject off, jobject isNull, jint n,
   jobject outHolder) {
    (void) self;
    jni_throw(env, vc_cert_choose(CTX(ctx), addr(env, sni), addr(env, off), addr(env, isNull), n,
                                 addr(env, outHolder)));
}

/* Mirror filters: packed vc_mirror_filter[] (strings interned to ids in Java) */
JNIEXPORT void JNICALL Java_vproxy_component_secure_GpuClassifier_compileMirror
  (JNIEnv *env, jclass self, jlong ctx, jobject filters, jint n) {
    (void) self;
    jni_throw(env, vc_compile_mirror(CTX(ctx), addr(env, filters), n));
}

JNIEXPORT void JNICALL Java_vproxy_component_secure_GpuClassifier_mirrorSwitch
  (JNIEnv *env, jclass self, jlong ctx, jint origin, jobject blob, jobject off, jint n,
   jint layer, jobject outMirrors) {
    (void) self;
    jni_throw(env, vc_mirror_switch(CTX(ctx), origin, addr(env, blob), addr(env, off), n, layer,
                                   addr(env, outMirrors)));
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
    char *buf = NULL;
    jstring s = NULL;
    int rc = vc_counters_prometheus(CTX(ctx), x, NULL, 0, &len);   /* size query */
    (void) self;
    if (rc == VC_ENOMEM) {
        buf = malloc((size_t) len + 1);
        rc = buf ? vc_counters_prometheus(CTX(ctx), x, buf, len + 1, &len) : VC_ENOMEM;
    }
    if (x) (*env)->ReleaseStringUTFChars(env, extra, x);
    if (!jni_throw(env, rc) && buf) s = (*env)->NewStringUTF(env, buf);
    free(buf);
    return s;
}

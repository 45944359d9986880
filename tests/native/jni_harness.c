/*
 * jni_harness.c -- runs the JNI shim (jni/vproxy_component_secure_GpuClassifier.c)
 * under a fake JNIEnv (test infrastructure only; built against
 * tests/native/jni_spec/jni.h).  Direct ByteBuffers are {address, capacity}
 * objects; ThrowNew records the exception class and message.
 *
 *   jni_harness cpu  -- no GPU: create throws IOException; a buffer shorter
 *                       than the batch throws IllegalArgumentException
 *                       before the library is called; an annotation string
 *                       outside the strings buffer is refused; a null
 *                       required buffer and offsets that are negative or
 *                       decrease are refused; injected statuses map to the
 *                       exceptions GpuContext keys its fallback on
 *                       (VC_EDEVICE / VC_ENOMEM -> IOException, VC_ESTATE ->
 *                       IllegalStateException).
 *   jni_harness gpu  -- through the shim vs the C ABI directly: ACL, routes,
 *                       per-VNI routes + switch, and compileUpstream twice
 *                       on one groups buffer (rebased in a copy, so the
 *                       second compile reads the same offsets).
 * Prints "JNI OK" and exits 0 when every check holds.
 */
#define _GNU_SOURCE
#include <dlfcn.h>
#include <jni.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "vclassify.h"

struct _jobject {
    void *p;
    jlong cap;
};

static char thrown_cls[128], thrown_msg[512];
static int n_thrown;

static jclass fake_find_class(JNIEnv *env, const char *name) {
    static struct _jobject c[8];
    static int k;
    (void) env;
    c[k & 7].p = (void *) name;
    return &c[k++ & 7];
}
static jint fake_throw_new(JNIEnv *env, jclass clazz, const char *msg) {
    (void) env;
    snprintf(thrown_cls, sizeof thrown_cls, "%s", (const char *) clazz->p);
    snprintf(thrown_msg, sizeof thrown_msg, "%s", msg ? msg : "");
    ++n_thrown;
    return 0;
}
static void *fake_addr(JNIEnv *env, jobject b) {
    (void) env;
    return b ? b->p : NULL;
}
static jlong fake_cap(JNIEnv *env, jobject b) {
    (void) env;
    return b ? b->cap : -1;
}
static jobject fake_elem(JNIEnv *env, jobjectArray a, jsize i) {
    (void) env;
    return ((jobject *) a->p)[i];
}
static const char *fake_utf(JNIEnv *env, jstring s, jboolean *c) {
    (void) env; (void) c;
    return (const char *) s->p;
}
static void fake_release(JNIEnv *env, jstring s, const char *x) {
    (void) env; (void) s; (void) x;
}
static jstring fake_new_utf(JNIEnv *env, const char *u) {
    static struct _jobject o;
    (void) env;
    o.p = (void *) u;
    return &o;
}

static struct JNINativeInterface_ table;
static JNIEnv env_obj = &table;
static JNIEnv *env = &env_obj;

/* the shim's exports */
#define J(name) Java_vproxy_component_secure_GpuClassifier_##name
jlong J(create)(JNIEnv *, jclass, jint);
void J(destroy)(JNIEnv *, jclass, jlong);
void J(compileAcl)(JNIEnv *, jclass, jlong, jobject, jint, jobject, jint, jboolean);
void J(classifyAclV4)(JNIEnv *, jclass, jlong, jobject, jobject, jobject, jint, jobject, jobject);
void J(compileRoutes)(JNIEnv *, jclass, jlong, jobject, jint, jobject, jint);
void J(lookupRouteV4)(JNIEnv *, jclass, jlong, jobject, jint, jobject);
void J(compileVniRoutes)(JNIEnv *, jclass, jlong, jobject, jobject, jobject, jobject, jobject, jint);
void J(compileUpstream)(JNIEnv *, jclass, jlong, jobject, jint, jobject);
void J(searchHints)(JNIEnv *, jclass, jlong, jobject, jobject, jobject, jobject, jobject, jobject,
                    jobject, jint, jobject);
jlong J(pinAcquire)(JNIEnv *, jclass, jlong, jint);
void J(bindPin)(JNIEnv *, jclass, jlong, jlong);
jlong J(pinGeneration)(JNIEnv *, jclass, jlong, jint);
void J(pinRelease)(JNIEnv *, jclass, jlong);
void J(switchClassify)(JNIEnv *, jclass, jlong, jobject, jobject, jint, jint, jobject, jobject,
                       jobject, jint, jobjectArray, jobject, jobject, jobject);

void J(compileCerts)(JNIEnv *, jclass, jlong, jobject, jobject, jobject, jint, jint);
void J(classifyDns)(JNIEnv *, jclass, jlong, jobject, jobject, jint, jobject, jobject);
void J(httpHint)(JNIEnv *, jclass, jlong, jobject, jobject, jint, jobject, jobject);
void J(pipelineCompact6)(JNIEnv *, jclass, jlong, jobject, jobject, jobject, jobject, jobject,
                        jobject, jint, jobject, jobject, jobject, jint, jint, jobject, jobject,
                        jobject, jobject);
void J(compileServers)(JNIEnv *, jclass, jlong, jobject, jobject, jint);
void J(setServerHealth)(JNIEnv *, jclass, jlong, jobject, jint);
void J(selectSourceV4)(JNIEnv *, jclass, jlong, jobject, jobject, jint, jint, jobject);

/* Fault injection.  The executable's definitions of these entry points
 * preempt libvclassify's for the shim linked into it: with inject_rc set
 * they return that status as the library would after a device error (or
 * before anything is compiled), otherwise they forward to the library. */
static int inject_rc;
typedef int (*acl_fn)(vc_ctx *, const uint8_t *, const uint32_t *, const uint16_t *, int64_t,
                      int32_t *, uint8_t *);
int vc_acl_classify_v4(vc_ctx *ctx, const uint8_t *proto, const uint32_t *src4,
                       const uint16_t *port, int64_t n, int32_t *out_idx, uint8_t *out_allow) {
    static acl_fn real;
    if (inject_rc) return inject_rc;
    if (!real) *(void **) &real = dlsym(RTLD_NEXT, "vc_acl_classify_v4");
    return real(ctx, proto, src4, port, n, out_idx, out_allow);
}
typedef int (*route_fn)(vc_ctx *, const uint32_t *, int64_t, int32_t *);
int vc_route_lookup_v4(vc_ctx *ctx, const uint32_t *dst4, int64_t n, int32_t *out) {
    static route_fn real;
    if (inject_rc) return inject_rc;
    if (!real) *(void **) &real = dlsym(RTLD_NEXT, "vc_route_lookup_v4");
    return real(ctx, dst4, n, out);
}

static struct _jobject B(void *p, jlong cap) {
    struct _jobject o;
    o.p = p;
    o.cap = cap;
    return o;
}

static int fails;
#define CHECK(c, what) do { if (!(c)) { fprintf(stderr, "FAIL %s (%s: %s)\n", what, thrown_cls, thrown_msg); ++fails; } n_thrown = 0; thrown_cls[0] = thrown_msg[0] = 0; } while (0)

static void expect_throw(const char *cls, const char *msg_part, const char *what) {
    CHECK(n_thrown == 1 && strcmp(thrown_cls, cls) == 0 && strstr(thrown_msg, msg_part), what);
    n_thrown = 0;
    thrown_cls[0] = thrown_msg[0] = 0;
}

static void net4(vc_net *n, uint32_t ip, int len) {
    int k;
    memset(n, 0, sizeof *n);
    n->ip_len = n->mask_len = 4;
    for (k = 0; k < 4; ++k) {
        const int bits = len - 8 * k;
        n->ip[k] = (uint8_t) (ip >> (24 - 8 * k));
        n->mask[k] = (uint8_t) (bits >= 8 ? 0xFF : bits <= 0 ? 0 : (0xFF << (8 - bits)) & 0xFF);
        n->ip[k] &= n->mask[k];
    }
}

static void cpu_mode(void) {
    uint8_t proto[8] = {6, 6, 17, 17, 6, 6, 6, 6};
    uint32_t src[8] = {0};
    uint16_t port[8] = {0};
    int32_t out[8];
    struct _jobject bp = B(proto, 8), bs = B(src, 31), bq = B(port, 16), bo = B(out, 32);
    vc_group_annos g;
    char strings[8] = "a.com";
    struct _jobject bg = B(&g, sizeof g), bstr = B(strings, 5);
    (void) J(create)(env, NULL, 0);
    expect_throw("java/io/IOException", "", "create without a GPU throws IOException");
    /* snapshot pins: a null context or pin is refused, release of 0 is a no-op */
    {
        const jlong pin = J(pinAcquire)(env, NULL, 0, 0xFF);
        expect_throw("java/lang/IllegalArgumentException", "null", "pinAcquire on a null context");
        CHECK(pin == 0, "pinAcquire on a null context returns 0");
        J(bindPin)(env, NULL, 0, 0);
        expect_throw("java/lang/IllegalArgumentException", "null", "bindPin on a null context");
        const jlong gen = J(pinGeneration)(env, NULL, 0, 1);
        expect_throw("java/lang/IllegalArgumentException", "null", "pinGeneration of a null pin");
        CHECK(gen == 0, "pinGeneration of a null pin returns 0");
    }
    J(pinRelease)(env, NULL, 0);
    CHECK(n_thrown == 0, "pinRelease(0) is a no-op");
    /* 8 items need 32 bytes of src4: a 31-byte buffer is refused before any vc_ call */
    J(classifyAclV4)(env, NULL, 0, &bp, &bs, &bq, 8, &bo, NULL);
    expect_throw("java/lang/IllegalArgumentException", "smaller than the batch",
                 "short src4 buffer");
    bs.cap = 32;
    bo.cap = 31;
    J(classifyAclV4)(env, NULL, 0, &bp, &bs, &bq, 8, &bo, NULL);
    expect_throw("java/lang/IllegalArgumentException", "smaller than the batch",
                 "short output buffer");
    J(classifyAclV4)(env, NULL, 0, &bp, &bs, &bq, -1, &bo, NULL);
    expect_throw("java/lang/IllegalArgumentException", "smaller than the batch", "negative n");
    /* an annotation whose string runs past the strings buffer */
    memset(&g, 0, sizeof g);
    g.handle.host = (const char *) (intptr_t) 2;
    g.handle.host_len = 4;
    g.handle.uri = (const char *) (intptr_t) -1;
    g.group.host = (const char *) (intptr_t) -1;
    g.group.uri = (const char *) (intptr_t) -1;
    J(compileUpstream)(env, NULL, 0, &bg, 1, &bstr);
    expect_throw("java/lang/IllegalArgumentException", "outside the strings buffer",
                 "annotation string past the buffer");
    CHECK((intptr_t) g.handle.host == 2, "the caller's groups buffer is left as it was");
    /* a null groups buffer with n > 0: refused, never dereferenced */
    J(compileUpstream)(env, NULL, 0, NULL, 1, &bstr);
    expect_throw("java/lang/IllegalArgumentException", "required", "null groups buffer");
    /* an annotation offset with no strings buffer at all */
    g.handle.host = (const char *) (intptr_t) 0;
    g.handle.host_len = 0;
    J(compileUpstream)(env, NULL, 0, &bg, 1, NULL);
    expect_throw("java/lang/IllegalArgumentException", "outside the strings buffer",
                 "annotation offset without a strings buffer");
    {   /* certificate names: offsets that decrease or start negative, a null
         * offsets buffer -- each refused before any pointer is formed */
        char names[8] = "abcde";
        int32_t bad_off[3] = {0, 100000, 5}, neg_off[3] = {-4, 0, 5}, holder[2] = {0, 0};
        struct _jobject bn = B(names, 5), bo1 = B(bad_off, 12), bo2 = B(neg_off, 12),
                        bh = B(holder, 8);
        J(compileCerts)(env, NULL, 0, &bn, &bo1, &bh, 2, 1);
        expect_throw("java/lang/IllegalArgumentException", "non-decreasing", "decreasing offsets");
        J(compileCerts)(env, NULL, 0, &bn, &bo2, &bh, 2, 1);
        expect_throw("java/lang/IllegalArgumentException", "non-negative", "negative offset");
        J(compileCerts)(env, NULL, 0, &bn, NULL, &bh, 2, 1);
        expect_throw("java/lang/IllegalArgumentException", "required", "null offsets");
        J(compileCerts)(env, NULL, 0, &bn, &bo1, NULL, 2, 1);
        expect_throw("java/lang/IllegalArgumentException", "", "null holder buffer");
    }
    {   /* a batch call whose offsets decrease: refused before the library */
        uint8_t q[16] = {0}, kind[2];
        int32_t qoff[3] = {0, 9, 4}, val[2];
        struct _jobject bq2 = B(q, 16), bo3 = B(qoff, 12), bk = B(kind, 2), bv = B(val, 8);
        J(classifyDns)(env, NULL, 0, &bq2, &bo3, 2, &bk, &bv);
        expect_throw("java/lang/IllegalArgumentException", "non-decreasing", "dns offsets");
    }
    {   /* compact IPv6 rows: family required, n6 rows of src6 / dst6 */
        uint8_t fam[8] = {4, 6, 4, 4, 6, 4, 4, 4}, rows[32] = {0};
        int32_t r[8], g2[8];
        struct _jobject bf = B(fam, 8), b6 = B(rows, 32), b6s = B(rows, 31), br2 = B(r, 32),
                        bg2 = B(g2, 32);
        J(pipelineCompact6)(env, NULL, 0, NULL, &bp, &bs, &bs, &b6, &b6, 2, &bq, NULL, NULL, 0, 8,
                            &bo, &br2, &bg2, NULL);
        expect_throw("java/lang/IllegalArgumentException", "required", "compact rows, null family");
        J(pipelineCompact6)(env, NULL, 0, &bf, &bp, &bs, &bs, &b6s, &b6, 2, &bq, NULL, NULL, 0, 8,
                            &bo, &br2, &bg2, NULL);
        expect_throw("java/lang/IllegalArgumentException", "smaller than the batch",
                     "compact rows, short src6");
        J(pipelineCompact6)(env, NULL, 0, &bf, &bp, &bs, &bs, &b6, &b6, -1, &bq, NULL, NULL, 0, 8,
                            &bo, &br2, &bg2, NULL);
        expect_throw("java/lang/IllegalArgumentException", "negative", "compact rows, n6 < 0");
    }
    /* the statuses GpuContext keys its fallback on (jni/GpuContext.java) */
    bs.cap = 32;
    bo.cap = 32;
    inject_rc = VC_EDEVICE;
    J(classifyAclV4)(env, NULL, 0, &bp, &bs, &bq, 8, &bo, NULL);
    expect_throw("java/io/IOException", "", "VC_EDEVICE -> IOException (context dead)");
    inject_rc = VC_ENOMEM;
    J(lookupRouteV4)(env, NULL, 0, &bs, 8, &bo);
    expect_throw("java/io/IOException", "", "VC_ENOMEM -> IOException");
    inject_rc = VC_ESTATE;
    J(classifyAclV4)(env, NULL, 0, &bp, &bs, &bq, 8, &bo, NULL);
    expect_throw("java/lang/IllegalStateException", "", "VC_ESTATE -> IllegalStateException");
    inject_rc = VC_EINVAL;
    J(lookupRouteV4)(env, NULL, 0, &bs, 8, &bo);
    expect_throw("java/lang/IllegalArgumentException", "", "VC_EINVAL -> IllegalArgumentException");
    inject_rc = 0;
}

static uint32_t rnd_state = 12345;
static uint32_t rnd(void) {
    rnd_state = rnd_state * 1103515245u + 12345u;
    return (rnd_state >> 8) ^ (rnd_state << 13);
}

static void gpu_mode(void) {
    enum { NR = 300, N = 50000, NV = 4 };
    static vc_acl_rule tcp[NR], udp[NR];
    static uint8_t proto[N];
    static uint32_t src[N], dst[N];
    static uint16_t port[N];
    static int32_t o1[N], o2[N];
    static uint8_t a1[N], a2[N];
    static vc_net routes[NR];
    jlong h;
    vc_ctx *ctx = NULL;
    int i;
    struct _jobject bt = B(tcp, sizeof tcp), bu = B(udp, sizeof udp), bp = B(proto, N),
                    bs = B(src, 4 * N), bq = B(port, 2 * N), bo = B(o1, 4 * N), ba = B(a1, N),
                    br = B(routes, sizeof routes), bd = B(dst, 4 * N);
    h = J(create)(env, NULL, 0);
    CHECK(h && !n_thrown, "create");
    CHECK(vc_create(0, &ctx) == VC_OK, "vc_create");
    for (i = 0; i < NR; ++i) {
        net4(&tcp[i].net, rnd(), 8 + (int) (rnd() % 17));
        tcp[i].min_port = (int32_t) (rnd() % 1000);
        tcp[i].max_port = tcp[i].min_port + (int32_t) (rnd() % 30000);
        tcp[i].allow = (int32_t) (rnd() & 1);
        net4(&routes[i], rnd(), 4 + (int) (rnd() % 21));
    }
    for (i = 0; i < NR; ++i) {
        udp[i] = tcp[(i * 7) % NR];
        udp[i].allow ^= 1;
    }
    for (i = 0; i < N; ++i) {
        proto[i] = (rnd() & 1) ? 6 : 17;
        src[i] = (i & 3) ? (uint32_t) ((tcp[rnd() % NR].net.ip[0] << 24) | (rnd() & 0xFFFFFF)) : rnd();
        port[i] = (uint16_t) (rnd() % 40000);
        dst[i] = (uint32_t) ((routes[rnd() % NR].ip[0] << 24) | (rnd() & 0xFFFFFF));
    }
    J(compileAcl)(env, NULL, h, &bt, NR, &bu, NR, 0);
    CHECK(!n_thrown, "compileAcl");
    J(classifyAclV4)(env, NULL, h, &bp, &bs, &bq, N, &bo, &ba);
    CHECK(!n_thrown, "classifyAclV4");
    CHECK(vc_compile_acl(ctx, tcp, NR, udp, NR, 0) == VC_OK, "vc_compile_acl");
    CHECK(vc_acl_classify_v4(ctx, proto, src, port, N, o2, a2) == VC_OK, "vc_acl_classify_v4");
    CHECK(memcmp(o1, o2, sizeof o1) == 0 && memcmp(a1, a2, sizeof a1) == 0,
          "ACL through the shim == the C ABI");
    J(compileRoutes)(env, NULL, h, &br, NR, NULL, 0);
    CHECK(!n_thrown, "compileRoutes");
    J(lookupRouteV4)(env, NULL, h, &bd, N, &bo);
    CHECK(vc_compile_routes(ctx, routes, NR, NULL, 0) == VC_OK, "vc_compile_routes");
    CHECK(vc_route_lookup_v4(ctx, dst, N, o2) == VC_OK, "vc_route_lookup_v4");
    CHECK(memcmp(o1, o2, sizeof o1) == 0, "routes through the shim == the C ABI");
    {   /* the mixed pipeline with compact IPv6 rows through the shim == the
         * sparse form through the C ABI (every 5th packet IPv6) */
        static uint8_t fam[N], s6[N][16], d6[N][16], c6s[N][16], c6d[N][16];
        static int32_t g1[N], g2[N], q1[N], q2[N];
        vc_packets in;
        vc_pipeline_out out;
        int n6 = 0;
        struct _jobject bf = B(fam, N), bcs = B(c6s, 16 * N), bcd = B(c6d, 16 * N),
                        bq1 = B(q1, 4 * N), bg1 = B(g1, 4 * N);
        for (i = 0; i < N; ++i) {
            int k;
            fam[i] = i % 5 == 2 ? 6 : 4;
            for (k = 0; k < 16; ++k) {
                s6[i][k] = (uint8_t) rnd();
                d6[i][k] = (uint8_t) rnd();
            }
            if (i % 3 == 0) memset(s6[i], 0, 12);          /* ::a.b.c.d against v4 rules */
            if (fam[i] == 6) {
                memcpy(c6s[n6], s6[i], 16);
                memcpy(c6d[n6], d6[i], 16);
                ++n6;
            }
        }
        J(pipelineCompact6)(env, NULL, h, &bf, &bp, &bs, &bd, &bcs, &bcd, n6, &bq, NULL, NULL, 0,
                            N, &bo, &bq1, &bg1, &ba);
        CHECK(!n_thrown, "pipelineCompact6");
        memset(&in, 0, sizeof in);
        in.family = fam;
        in.proto = proto;
        in.src4 = src;
        in.dst4 = dst;
        in.src6 = &s6[0][0];
        in.dst6 = &d6[0][0];
        in.dport = port;
        out.acl = o2;
        out.route = q2;
        out.group = g2;
        out.allow = a2;
        CHECK(vc_pipeline(ctx, &in, N, NULL, 0, &out) == VC_OK, "vc_pipeline");
        CHECK(memcmp(o1, o2, sizeof o1) == 0 && memcmp(q1, q2, sizeof q1) == 0 &&
              memcmp(a1, a2, sizeof a1) == 0 && memcmp(g1, g2, sizeof g1) == 0,
              "compact-row pipeline through the shim == the sparse form through the C ABI");
    }
    {   /* per-VNI tables through the shim: the VNI-10 table is routes[0..150) */
        int32_t vni[2] = {10, 20}, off4[3] = {0, 150, NR}, off6[3] = {0, 0, 0};
        struct _jobject bv = B(vni, 8), b4o = B(off4, 12), b6o = B(off6, 12);
        J(compileVniRoutes)(env, NULL, h, &bv, &br, &b4o, NULL, &b6o, 2);
        CHECK(!n_thrown, "compileVniRoutes");
        b4o.cap = 11;
        J(compileVniRoutes)(env, NULL, h, &bv, &br, &b4o, NULL, &b6o, 2);
        expect_throw("java/lang/IllegalArgumentException", "smaller than the batch",
                     "short vni offsets");
    }
    {   /* compileUpstream twice from one groups buffer of offsets */
        static vc_group_annos g[3], gd[3];
        static const char strings[] = "a.example.com" "b.example.com" "/api";
        static const char *names[6] = {"a.example.com", "x.b.example.com", "b.example.com",
                                       "nope.org", "a.example.com", "www.b.example.com"};
        static uint8_t blob[128];
        static uint32_t off[7];
        static uint16_t hp[6];
        static int32_t r1[6], r2[6], r3[6];
        struct _jobject bg = B(g, sizeof g), bst = B((void *) strings, sizeof strings - 1),
                        bb = B(blob, sizeof blob), bof = B(off, sizeof off), bhp = B(hp, sizeof hp),
                        bres = B(r1, sizeof r1);
        int k, pos = 0;
        for (k = 0; k < 3; ++k) {
            vc_annos *a[2] = {&g[k].handle, &g[k].group};
            int j;
            for (j = 0; j < 2; ++j) {
                a[j]->host = (const char *) (intptr_t) -1;
                a[j]->uri = (const char *) (intptr_t) -1;
                a[j]->host_len = a[j]->uri_len = 0;
                a[j]->port = 0;
            }
        }
        g[0].handle.host = (const char *) (intptr_t) 0;
        g[0].handle.host_len = 13;
        g[1].group.host = (const char *) (intptr_t) 13;
        g[1].group.host_len = 13;
        g[2].handle.host = (const char *) (intptr_t) 13;
        g[2].handle.host_len = 13;
        g[2].handle.uri = (const char *) (intptr_t) 26;
        g[2].handle.uri_len = 4;
        for (k = 0; k < 6; ++k) {
            off[k] = (uint32_t) pos;
            memcpy(blob + pos, names[k], strlen(names[k]));
            pos += (int) strlen(names[k]);
        }
        off[6] = (uint32_t) pos;
        J(compileUpstream)(env, NULL, h, &bg, 3, &bst);
        CHECK(!n_thrown, "compileUpstream");
        J(searchHints)(env, NULL, h, &bb, &bof, NULL, &bhp, NULL, NULL, NULL, 6, &bres);
        CHECK(!n_thrown, "searchHints");
        bres.p = r3;
        J(compileUpstream)(env, NULL, h, &bg, 3, &bst);         /* same buffer again */
        CHECK(!n_thrown, "second compileUpstream from the same buffer");
        J(searchHints)(env, NULL, h, &bb, &bof, NULL, &bhp, NULL, NULL, NULL, 6, &bres);
        for (k = 0; k < 3; ++k) {
            vc_annos *s[2] = {&g[k].handle, &g[k].group}, *d[2] = {&gd[k].handle, &gd[k].group};
            int j;
            for (j = 0; j < 2; ++j) {
                *d[j] = *s[j];
                d[j]->host = (intptr_t) s[j]->host < 0 ? NULL : strings + (intptr_t) s[j]->host;
                d[j]->uri = (intptr_t) s[j]->uri < 0 ? NULL : strings + (intptr_t) s[j]->uri;
            }
        }
        CHECK(vc_compile_upstream(ctx, gd, 3) == VC_OK, "vc_compile_upstream");
        CHECK(vc_hint_search(ctx, blob, off, NULL, hp, NULL, NULL, NULL, 6, r2) == VC_OK,
              "vc_hint_search");
        CHECK(memcmp(r1, r2, sizeof r1) == 0 && memcmp(r3, r2, sizeof r2) == 0,
              "hints through the shim (twice) == the C ABI");
        CHECK(r2[0] == 0 && r2[3] == -1, "a.example.com -> group 0, nope.org -> null");
        {   /* HTTP/1 request heads through the shim == the C ABI (same Upstream) */
            static const char *heads[4] = {
                "GET /x HTTP/1.1\r\nHost: a.example.com\r\n\r\n",
                "GET /y HTTP/1.1\r\nHost: www.a.example.com:80\r\nAccept: x\r\n\r\n",
                "GET /z HTTP/1.1\r\nhost: nope.org\r\n\r\n", "GET"};
            static uint8_t hb[256], k1[4], k2[4];
            static int32_t ho[5], g1[4], g2[4];
            struct _jobject bhb = B(hb, sizeof hb), bho = B(ho, sizeof ho), bg1 = B(g1, sizeof g1),
                            bk1 = B(k1, sizeof k1);
            int q = 0;
            for (k = 0; k < 4; ++k) {
                ho[k] = q;
                memcpy(hb + q, heads[k], strlen(heads[k]));
                q += (int) strlen(heads[k]);
            }
            ho[4] = q;
            J(httpHint)(env, NULL, h, &bhb, &bho, 4, &bg1, &bk1);
            CHECK(!n_thrown, "httpHint");
            CHECK(vc_http_hint(ctx, hb, (const uint32_t *) ho, 4, g2, k2) == VC_OK, "vc_http_hint");
            CHECK(memcmp(g1, g2, sizeof g1) == 0 && memcmp(k1, k2, sizeof k1) == 0,
                  "HTTP heads through the shim == the C ABI");
            CHECK(g2[0] == 0 && g2[2] == -1 && k2[0] == 3 && k2[3] == 0,
                  "Host a.example.com -> group 0, nope.org -> null, a bare method -> no hint");
        }
    }
    {   /* source hashing through the shim: compile, health update, select ==
         * the C ABI; a short health buffer is refused */
        enum { NG = 40, NS = 200 };
        static vc_server sv[NS];
        static int32_t goff[NG + 1], grp[N], s1[N], s2[N];
        static uint8_t hl[NS];
        struct _jobject bsv = B(sv, sizeof sv), bgo = B(goff, sizeof goff), bgr = B(grp, 4 * N),
                        bsr = B(src, 4 * N), bh = B(hl, NS), bout = B(s1, 4 * N);
        for (i = 0; i < NS; ++i) {
            const uint32_t a = rnd();
            memset(&sv[i], 0, sizeof sv[i]);
            sv[i].ip[0] = (uint8_t) (a >> 24);
            sv[i].ip[1] = (uint8_t) (a >> 16);
            sv[i].ip[2] = (uint8_t) (a >> 8);
            sv[i].ip[3] = (uint8_t) a;
            sv[i].ip_len = 4;
            sv[i].port = 80;
            sv[i].weight = 1;
            sv[i].healthy = 1;
            hl[i] = (uint8_t) (rnd() % 3 != 0);
        }
        for (i = 0; i <= NG; ++i) goff[i] = i * NS / NG;
        for (i = 0; i < N; ++i) grp[i] = (int32_t) (rnd() % NG);
        J(compileServers)(env, NULL, h, &bsv, &bgo, NG);
        CHECK(!n_thrown, "compileServers");
        J(setServerHealth)(env, NULL, h, &bh, NS);
        CHECK(!n_thrown, "setServerHealth");
        J(selectSourceV4)(env, NULL, h, &bgr, &bsr, N, 0, &bout);
        CHECK(!n_thrown, "selectSourceV4");
        CHECK(vc_compile_servers(ctx, sv, goff, NG) == VC_OK, "vc_compile_servers");
        CHECK(vc_servers_set_health(ctx, hl, NS) == VC_OK, "vc_servers_set_health");
        CHECK(vc_source_select_v4(ctx, grp, src, N, 0, s2) == VC_OK, "vc_source_select_v4");
        CHECK(memcmp(s1, s2, sizeof s1) == 0, "source hashing through the shim == the C ABI");
        bh.cap = NS - 1;
        J(setServerHealth)(env, NULL, h, &bh, NS);
        expect_throw("java/lang/IllegalArgumentException", "smaller than the batch",
                     "short health buffer");
    }
    J(destroy)(env, NULL, h);
    vc_destroy(ctx);
}

int main(int argc, char **argv) {
    table.FindClass = fake_find_class;
    table.ThrowNew = fake_throw_new;
    table.GetDirectBufferAddress = fake_addr;
    table.GetDirectBufferCapacity = fake_cap;
    table.GetObjectArrayElement = fake_elem;
    table.GetStringUTFChars = fake_utf;
    table.ReleaseStringUTFChars = fake_release;
    table.NewStringUTF = fake_new_utf;
    if (argc > 1 && strcmp(argv[1], "gpu") == 0)
        gpu_mode();
    else
        cpu_mode();
    if (fails) return 1;
    printf("JNI OK\n");
    return 0;
}

/*
 * pin_loop.c -- C replay of jni/GpuContext.java's view protocol (test
 * infrastructure only), run through the JNI shim's natives under a
 * thread-safe fake JNIEnv.
 *
 * GpuContext (round 6) never holds a lock across a native compile: a View is
 * {native pin, the lists its indices refer to, a reference count}; batch()
 * retains the current view with a compare-and-set, binds its pin around the
 * native call (bindPin), releases it, and maps the outputs through the
 * view's lists; publish() compiles under a monitor only compiles take, pins
 * what it published (pinAcquire), swaps the view and releases the old one
 * (its pin goes when its last batch ends).  Mode 1 replays the round-5
 * GpuContext instead: a read-write lock, the compile and the list swap
 * under the write side, each batch's call and mapping under the read side.
 *
 * pin_loop_run: event-loop threads classify route batches (RouteTable.lookup,
 * lookupRouteV4 on registered direct buffers) while the control thread
 * recompiles the route table `recompiles` times, alternating two tables.
 * Each batch's outputs must equal the lookups of its view's table (the
 * "lists" a view carries is the table id; the expected outputs per table are
 * computed first with the C ABI directly), and the pin must report the
 * generation the view recorded at publish.  Latencies per batch are split
 * into the quiet phase (before the first recompile) and the recompile phase.
 */
#define _GNU_SOURCE
#include <jni.h>
#include <pthread.h>
#include <stdatomic.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>

#include "vclassify.h"

struct _jobject {
    void *p;
    jlong cap;
};

/* ---- fake JNIEnv: per-thread exception state -------------------------- */
static _Thread_local char t_cls[128], t_msg[512];
static _Thread_local int t_thrown;
static _Thread_local struct _jobject t_class;

static jclass fake_find_class(JNIEnv *e, const char *name) {
    (void) e;
    t_class.p = (void *) name;
    return &t_class;
}
static jint fake_throw_new(JNIEnv *e, jclass c, const char *msg) {
    (void) e;
    snprintf(t_cls, sizeof t_cls, "%s", (const char *) c->p);
    snprintf(t_msg, sizeof t_msg, "%s", msg ? msg : "");
    ++t_thrown;
    return 0;
}
static void *fake_addr(JNIEnv *e, jobject b) {
    (void) e;
    return b ? b->p : NULL;
}
static jlong fake_cap(JNIEnv *e, jobject b) {
    (void) e;
    return b ? b->cap : -1;
}
static struct JNINativeInterface_ table;
static JNIEnv env_obj = &table;
static JNIEnv *env = &env_obj;

#define J(name) Java_vproxy_component_secure_GpuClassifier_##name
jlong J(create)(JNIEnv *, jclass, jint);
void J(destroy)(JNIEnv *, jclass, jlong);
void J(registerBuffer)(JNIEnv *, jclass, jobject);
void J(unregisterBuffer)(JNIEnv *, jclass, jobject);
void J(compileRoutes)(JNIEnv *, jclass, jlong, jobject, jint, jobject, jint);
void J(lookupRouteV4)(JNIEnv *, jclass, jlong, jobject, jint, jobject);
jlong J(pinAcquire)(JNIEnv *, jclass, jlong, jint);
void J(bindPin)(JNIEnv *, jclass, jlong, jlong);
jlong J(pinGeneration)(JNIEnv *, jclass, jlong, jint);
void J(pinRelease)(JNIEnv *, jclass, jlong);

#define SNAP_ALL 0xFF
#define SNAP_ROUTE 1

typedef struct {
    int threads;      /* event-loop threads */
    int batch;        /* lookups per batch */
    int think_us;     /* an event loop's other work between batches */
    int quiet_ms;     /* quiet phase before the first recompile */
    int tail_ms;      /* batches after the last recompile */
    int recompiles;
    int mode;         /* 0 = views + pins (GpuContext), 1 = read-write lock (round 5) */
} pin_loop_cfg;

typedef struct {
    int64_t batches_quiet, batches_during, batches_after;
    double p50_quiet, p99_quiet, max_quiet;     /* ms */
    double p50_during, p99_during, max_during;
    double compile_ms_mean, compile_ms_max;
    int64_t mismatches;       /* batches whose outputs differ from their view's table */
    int64_t gen_mismatches;   /* pinGeneration != the view's recorded generation */
    int64_t errors;           /* exceptions thrown by a native */
    int64_t views_used;       /* distinct views batches ran on */
    int64_t table_batches[2]; /* batches per table id */
    int64_t retries;          /* retain() that lost a race with a swap */
    int64_t differ;           /* keys whose expected outputs differ between the tables */
    int64_t slow_quiet, slow_during;   /* batches over 10 ms */
} pin_loop_stats;

/* ---- the View (GpuContext.View) ---------------------------------------- */
typedef struct View {
    jlong pin;
    int table;          /* the "lists": which table's indices these are */
    uint64_t gen;       /* generation pinned at publish */
    int serial;         /* publish count */
    atomic_int refs;    /* 1 for being current, 1 per batch on it */
} View;

static _Atomic(View *) current;
static pthread_rwlock_t rw = PTHREAD_RWLOCK_INITIALIZER;     /* mode 1 */
static int r_table;                                         /* mode 1: the swapped "lists" */
static atomic_int stop_flag;
static atomic_long phase_start_ns, phase_end_ns;            /* recompile phase */
static jlong g_ctx;
static const int32_t *g_exp[2];
static const uint32_t *g_keys;
static int64_t g_nkeys;
static pin_loop_cfg g_cfg;
static atomic_long g_err, g_mis, g_gmis, g_retry;

static int64_t now_ns(void) {
    struct timespec ts;
    clock_gettime(CLOCK_MONOTONIC, &ts);
    return (int64_t) ts.tv_sec * 1000000000 + ts.tv_nsec;
}

static int retain(View *v) {
    int r = atomic_load(&v->refs);
    while (r != 0)
        if (atomic_compare_exchange_weak(&v->refs, &r, r + 1)) return 1;
    return 0;
}

/* A View's memory stays until the run ends, as Java's garbage collector
 * keeps an object a batch still references: a batch may read `current` just
 * before a swap and the old view's last release, and then finds refs == 0
 * (retain fails, it reads `current` again).  The pin goes at refs == 0. */
static View *all_views[4097];
static int n_views;

static View *new_view(void) {
    View *v = calloc(1, sizeof *v);
    all_views[n_views++] = v;
    return v;
}

static void release(View *v) {
    if (atomic_fetch_sub(&v->refs, 1) == 1) J(pinRelease)(env, NULL, v->pin);
}

static int threw(void) {
    if (!t_thrown) return 0;
    fprintf(stderr, "native threw %s: %s\n", t_cls, t_msg);
    t_thrown = 0;
    atomic_fetch_add(&g_err, 1);
    return 1;
}

typedef struct {
    int id;
    int64_t *lat_ns;      /* per batch */
    int64_t *start_ns;
    int *table;
    int *serial;
    int64_t n;
    int64_t cap;
} Loop;

static void *event_loop(void *arg) {
    Loop *L = arg;
    const int b = g_cfg.batch;
    uint32_t *in = NULL;
    int32_t *out = NULL;
    struct _jobject bi, bo;
    int64_t pos = (int64_t) L->id * 7919 * b % g_nkeys;
    if (posix_memalign((void **) &in, 4096, (size_t) b * 4) ||
        posix_memalign((void **) &out, 4096, (size_t) b * 4)) {
        atomic_fetch_add(&g_err, 1);
        return NULL;
    }
    bi.p = in;
    bi.cap = (jlong) b * 4;
    bo.p = out;
    bo.cap = (jlong) b * 4;
    /* the drain-loop batchers register their buffers once (zero-copy calls) */
    J(registerBuffer)(env, NULL, &bi);
    J(registerBuffer)(env, NULL, &bo);
    threw();
    while (!atomic_load(&stop_flag) && L->n < L->cap) {
        int64_t k;
        int tab, serial = -1, bad = 0;
        if (pos + b > g_nkeys) pos = 0;
        memcpy(in, g_keys + pos, (size_t) b * 4);
        const int64_t t0 = now_ns();
        if (g_cfg.mode == 0) {
            View *v;
            for (;;) {
                v = atomic_load(&current);
                if (retain(v)) break;
                atomic_fetch_add(&g_retry, 1);
            }
            J(bindPin)(env, NULL, g_ctx, v->pin);
            J(lookupRouteV4)(env, NULL, g_ctx, &bi, b, &bo);
            J(bindPin)(env, NULL, g_ctx, 0);
            if (threw()) bad = 1;
            else if ((uint64_t) J(pinGeneration)(env, NULL, v->pin, SNAP_ROUTE) != v->gen)
                atomic_fetch_add(&g_gmis, 1);
            tab = v->table;
            serial = v->serial;
            release(v);                 /* the outputs are in our buffer */
        } else {
            pthread_rwlock_rdlock(&rw);
            J(lookupRouteV4)(env, NULL, g_ctx, &bi, b, &bo);
            if (threw()) bad = 1;
            tab = r_table;
        }
        /* map: every output through the view's lists */
        if (!bad)
            for (k = 0; k < b; ++k)
                if (out[k] != g_exp[tab][pos + k]) {
                    atomic_fetch_add(&g_mis, 1);
                    break;
                }
        if (g_cfg.mode == 1) pthread_rwlock_unlock(&rw);
        const int64_t t1 = now_ns();
        L->start_ns[L->n] = t0;
        L->lat_ns[L->n] = t1 - t0;
        L->table[L->n] = tab;
        L->serial[L->n] = serial;
        ++L->n;
        pos += b;
        if (g_cfg.think_us > 0) {
            struct timespec ts = {0, (long) g_cfg.think_us * 1000};
            nanosleep(&ts, NULL);
        }
    }
    J(unregisterBuffer)(env, NULL, &bi);
    J(unregisterBuffer)(env, NULL, &bo);
    threw();
    free(in);
    free(out);
    return NULL;
}

static int cmp_i64(const void *a, const void *b) {
    const int64_t x = *(const int64_t *) a, y = *(const int64_t *) b;
    return x < y ? -1 : x > y;
}

static void pct(int64_t *v, int64_t n, double *p50, double *p99, double *mx) {
    if (n == 0) {
        *p50 = *p99 = *mx = 0;
        return;
    }
    qsort(v, (size_t) n, sizeof *v, cmp_i64);
    *p50 = v[n / 2] / 1e6;
    *p99 = v[(int64_t) ((n - 1) * 0.99)] / 1e6;
    *mx = v[n - 1] / 1e6;
}

static void sleep_ms(int ms) {
    struct timespec ts = {ms / 1000, (long) (ms % 1000) * 1000000};
    nanosleep(&ts, NULL);
}

/* tables: t4[k] / n4[k] / t6[k] / n6[k] for k = 0, 1 (vc_net arrays in list order) */
int pin_loop_run(int device, const vc_net *t4a, int n4a, const vc_net *t6a, int n6a,
                 const vc_net *t4b, int n4b, const vc_net *t6b, int n6b, const uint32_t *keys,
                 int64_t nkeys, int32_t *exp_a, int32_t *exp_b, const pin_loop_cfg *cfg,
                 pin_loop_stats *st) {
    const vc_net *t4[2] = {t4a, t4b}, *t6[2] = {t6a, t6b};
    const int n4[2] = {n4a, n4b}, n6[2] = {n6a, n6b};
    struct _jobject b4[2], b6[2];
    int k, i;
    Loop *loops;
    pthread_t *th;
    double csum = 0, cmax = 0;
    int64_t tot = 0, nq = 0, nd = 0, na = 0, *lq, *ld;
    int serial_seen[4096] = {0};

    table.FindClass = fake_find_class;
    table.ThrowNew = fake_throw_new;
    table.GetDirectBufferAddress = fake_addr;
    table.GetDirectBufferCapacity = fake_cap;
    memset(st, 0, sizeof *st);
    g_cfg = *cfg;
    g_keys = keys;
    g_nkeys = nkeys;
    g_exp[0] = exp_a;
    g_exp[1] = exp_b;
    atomic_store(&stop_flag, 0);
    atomic_store(&g_err, 0);
    atomic_store(&g_mis, 0);
    atomic_store(&g_gmis, 0);
    atomic_store(&g_retry, 0);
    n_views = 0;
    if (cfg->batch <= 0 || nkeys < cfg->batch || cfg->threads <= 0 || cfg->recompiles > 4000)
        return -1;
    for (k = 0; k < 2; ++k) {
        b4[k].p = (void *) t4[k];
        b4[k].cap = (jlong) n4[k] * (jlong) sizeof(vc_net);
        b6[k].p = (void *) t6[k];
        b6[k].cap = (jlong) n6[k] * (jlong) sizeof(vc_net);
    }
    {   /* ReentrantReadWriteLock (non-fair) parks new readers behind a queued writer */
        pthread_rwlockattr_t a;
        pthread_rwlockattr_init(&a);
        pthread_rwlockattr_setkind_np(&a, PTHREAD_RWLOCK_PREFER_WRITER_NONRECURSIVE_NP);
        pthread_rwlock_destroy(&rw);
        pthread_rwlock_init(&rw, &a);
        pthread_rwlockattr_destroy(&a);
    }
    g_ctx = J(create)(env, NULL, device);
    if (threw()) return -2;
    /* the expected outputs of both tables, through the C ABI directly */
    for (k = 0; k < 2; ++k) {
        if (vc_compile_routes((vc_ctx *) (intptr_t) g_ctx, t4[k], n4[k], t6[k], n6[k]) ||
            vc_route_lookup_v4((vc_ctx *) (intptr_t) g_ctx, keys, nkeys, k ? exp_b : exp_a)) {
            fprintf(stderr, "setup: %s\n", vc_last_error());
            J(destroy)(env, NULL, g_ctx);
            return -3;
        }
    }
    for (i = 0; i < nkeys; ++i) st->differ += exp_a[i] != exp_b[i];
    /* publish table 0 (GpuContext.publish) */
    J(compileRoutes)(env, NULL, g_ctx, &b4[0], n4[0], &b6[0], n6[0]);
    {
        View *v = new_view();
        v->pin = J(pinAcquire)(env, NULL, g_ctx, SNAP_ALL);
        v->table = 0;
        v->gen = (uint64_t) J(pinGeneration)(env, NULL, v->pin, SNAP_ROUTE);
        v->serial = 0;
        atomic_init(&v->refs, 1);
        atomic_store(&current, v);
        r_table = 0;
    }
    if (threw()) return -4;

    loops = calloc((size_t) cfg->threads, sizeof *loops);
    th = calloc((size_t) cfg->threads, sizeof *th);
    for (k = 0; k < cfg->threads; ++k) {
        loops[k].id = k;
        loops[k].cap = 1 << 20;
        loops[k].lat_ns = malloc(sizeof(int64_t) * (size_t) loops[k].cap);
        loops[k].start_ns = malloc(sizeof(int64_t) * (size_t) loops[k].cap);
        loops[k].table = malloc(sizeof(int) * (size_t) loops[k].cap);
        loops[k].serial = malloc(sizeof(int) * (size_t) loops[k].cap);
        pthread_create(&th[k], NULL, event_loop, &loops[k]);
    }
    /* the control thread */
    sleep_ms(cfg->quiet_ms);
    atomic_store(&phase_start_ns, now_ns());
    for (i = 1; i <= cfg->recompiles; ++i) {
        const int tab = i & 1;
        const int64_t c0 = now_ns();
        if (cfg->mode == 0) {
            View *nv, *old;
            J(compileRoutes)(env, NULL, g_ctx, &b4[tab], n4[tab], &b6[tab], n6[tab]);
            if (threw()) break;
            nv = new_view();
            nv->pin = J(pinAcquire)(env, NULL, g_ctx, SNAP_ALL);
            nv->table = tab;
            nv->gen = (uint64_t) J(pinGeneration)(env, NULL, nv->pin, SNAP_ROUTE);
            nv->serial = i;
            atomic_init(&nv->refs, 1);
            old = atomic_exchange(&current, nv);
            release(old);
        } else {
            pthread_rwlock_wrlock(&rw);
            J(compileRoutes)(env, NULL, g_ctx, &b4[tab], n4[tab], &b6[tab], n6[tab]);
            r_table = tab;
            pthread_rwlock_unlock(&rw);
            if (threw()) break;
        }
        {
            const double ms = (now_ns() - c0) / 1e6;
            csum += ms;
            if (ms > cmax) cmax = ms;
        }
    }
    atomic_store(&phase_end_ns, now_ns());
    sleep_ms(cfg->tail_ms);
    atomic_store(&stop_flag, 1);
    for (k = 0; k < cfg->threads; ++k) pthread_join(th[k], NULL);

    for (k = 0; k < cfg->threads; ++k) tot += loops[k].n;
    lq = malloc(sizeof(int64_t) * (size_t) (tot + 1));
    ld = malloc(sizeof(int64_t) * (size_t) (tot + 1));
    for (k = 0; k < cfg->threads; ++k)
        for (i = 0; i < loops[k].n; ++i) {
            const int64_t s0 = loops[k].start_ns[i], s1 = s0 + loops[k].lat_ns[i];
            const int slow = loops[k].lat_ns[i] > 10000000;
            if (s1 <= atomic_load(&phase_start_ns)) {
                lq[nq++] = loops[k].lat_ns[i];
                st->slow_quiet += slow;
            } else if (s0 < atomic_load(&phase_end_ns)) {
                ld[nd++] = loops[k].lat_ns[i];
                st->slow_during += slow;
            } else {
                ++na;
            }
            st->table_batches[loops[k].table[i]]++;
            if (loops[k].serial[i] >= 0 && loops[k].serial[i] < 4096) serial_seen[loops[k].serial[i]] = 1;
        }
    st->batches_quiet = nq;
    st->batches_during = nd;
    st->batches_after = na;
    pct(lq, nq, &st->p50_quiet, &st->p99_quiet, &st->max_quiet);
    pct(ld, nd, &st->p50_during, &st->p99_during, &st->max_during);
    st->compile_ms_mean = cfg->recompiles ? csum / cfg->recompiles : 0;
    st->compile_ms_max = cmax;
    st->mismatches = atomic_load(&g_mis);
    st->gen_mismatches = atomic_load(&g_gmis);
    st->errors = atomic_load(&g_err);
    st->retries = atomic_load(&g_retry);
    for (i = 0; i < 4096; ++i) st->views_used += serial_seen[i];
    free(lq);
    free(ld);
    for (k = 0; k < cfg->threads; ++k) {
        free(loops[k].lat_ns);
        free(loops[k].start_ns);
        free(loops[k].table);
        free(loops[k].serial);
    }
    free(loops);
    free(th);
    if (cfg->mode == 0) release(atomic_load(&current));
    for (i = 0; i < n_views; ++i) free(all_views[i]);
    n_views = 0;
    J(destroy)(env, NULL, g_ctx);
    return 0;
}

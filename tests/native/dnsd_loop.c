/*
 * dnsd_loop.c -- test-only C replay of jni/DnsDrainBatcher.java: DNSServer's
 * drain loop (core/src/main/java/vproxy/dns/DNSServer.java:457-500) run in
 * batches through vc_dns_datagrams, with the batcher's per-status actions
 * and its event boundaries, so the GPU tier can check that the status
 * contract reproduces the reference loop's action sequence at any batch
 * size (tests/test_gpu_dnsd_loop.py) and the CPU tier the fallback
 * (tests/test_dnsd_loop_cpu.py).  Built as a shared library, called through
 * ctypes with a context the ctypes layer compiled.
 *
 * The "socket" is the whole input queue.  One readable event takes pending
 * datagrams first, then receives up to `batch`; one vc_dns_datagrams call
 * classifies them; then, in arrival order:
 *   REJECTED  -> "S i"  securityGroup.allow false: continue        (:469-472)
 *   EMPTY     -> "E i"  read == 0: return                          (:473-476)
 *   MALFORMED -> "E i"  parsePackets threw: return                 (:481-486)
 *   RESPONSE  -> "P i"  p.isResponse: logged, continue              (:489-492)
 *   RECURSIVE -> "R i"  runRecursive (opcode, qtype, unknown name)  (:493-496, :116-166)
 *   ANSWER    -> "A i nq k:v ..." handleRequest from the kinds     (:497, :116-166)
 *   HOST      -> "J i"  the Java loop body for that datagram
 * A "return" ends the event ("|"); the rest stay pending and the next event
 * (the batcher's nextTick, as the level-triggered selector would fire again
 * on a socket still holding them) starts with them.  When the call fails,
 * every datagram of the batch takes the Java path ("J i"); VC_EDEVICE /
 * VC_ENOMEM (IOException in the shim) marks the context dead for good ("D"),
 * VC_ESTATE (IllegalStateException) affects that batch only ("F").
 */
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "vclassify.h"

typedef struct {
    char *out;
    int64_t cap, len;
} trace_t;

static void put(trace_t *t, const char *s) {
    int64_t k = (int64_t) strlen(s);
    if (t->len + k + 1 < t->cap) {
        memcpy(t->out + t->len, s, (size_t) k);
        t->len += k;
        t->out[t->len] = 0;
    }
}

/* inject[b] != 0: batch b's call "returns" that status instead of running */
int dnsd_loop_trace(vc_ctx *ctx, const uint8_t *blob, const uint32_t *off, int64_t n,
                    const uint8_t *fam, const uint32_t *r4, const uint8_t *r6,
                    const uint16_t *port, int batch, const int *inject, int n_inject,
                    char *out, int64_t cap) {
    trace_t t = {out, cap, 0};
    /* [head, n) is not dispatched yet: the datagrams a batch received but an
     * EMPTY / MALFORMED left pending, then the socket; a batch is
     * [head, head + batch), pending first */
    int64_t head = 0;
    int dead = 0, calls = 0;
    char buf[256];
    uint8_t *bb, *bfam, *bst, *bnq, *bkind, *br6;
    uint32_t *boff, *br4;
    uint16_t *bport, *bqt;
    int32_t *bacl, *bval;
    int rc = 0;
    if (batch < 1 || cap < 1 || n < 0) return VC_EINVAL;
    out[0] = 0;
    bb = malloc((size_t) off[n] + 16);
    boff = malloc(sizeof(uint32_t) * (size_t) (batch + 1));
    bfam = malloc((size_t) batch);
    br4 = malloc(sizeof(uint32_t) * (size_t) batch);
    br6 = aligned_alloc(16, 16 * (size_t) batch);
    bport = malloc(sizeof(uint16_t) * (size_t) batch);
    bst = malloc((size_t) batch);
    bnq = malloc((size_t) batch);
    bkind = malloc((size_t) batch * VC_DNSD_MAXQ);
    bqt = malloc(sizeof(uint16_t) * (size_t) batch * VC_DNSD_MAXQ);
    bacl = malloc(sizeof(int32_t) * (size_t) batch);
    bval = malloc(sizeof(int32_t) * (size_t) batch * VC_DNSD_MAXQ);
    while (head < n) {                                /* readable events */
        int event_over = 0;
        while (!event_over && head < n) {             /* batches of one event */
            const int64_t lo = head, hi = head + batch < n ? head + batch : n;
            const int m = (int) (hi - lo);
            int i, status;
            int64_t k;
            boff[0] = 0;
            for (k = lo; k < hi; ++k) {
                const int j = (int) (k - lo);
                const uint32_t len = off[k + 1] - off[k];
                memcpy(bb + boff[j], blob + off[k], len);
                boff[j + 1] = boff[j] + len;
                bfam[j] = fam[k];
                br4[j] = r4[k];
                memcpy(br6 + 16 * j, r6 + 16 * k, 16);
                bport[j] = port[k];
            }
            status = dead ? VC_EDEVICE : calls < n_inject && inject[calls] ? inject[calls] : VC_OK;
            ++calls;
            if (status == VC_OK) {
                vc_dnsd_out o;
                o.status = bst; o.acl = bacl; o.nq = bnq; o.qtype = bqt; o.kind = bkind;
                o.value = bval;
                status = vc_dns_datagrams(ctx, bb, boff, m, bfam, br4, br6, bport, &o);
                if (status != VC_OK && status != VC_ESTATE && status != VC_EDEVICE &&
                    status != VC_ENOMEM) {
                    rc = status;                      /* a caller bug: rethrown */
                    goto done;
                }
            }
            if (status != VC_OK) {                    /* GpuContext.call returned false */
                if (!dead) put(&t, status == VC_ESTATE ? "F " : "D ");
                if (status != VC_ESTATE) dead = 1;
                for (i = 0; i < m; ++i) {
                    snprintf(buf, sizeof buf, "J %lld ", (long long) (lo + i));
                    put(&t, buf);
                }
                head = hi;
                continue;
            }
            head = hi;
            for (i = 0; i < m; ++i) {
                const long long g = (long long) (lo + i);
                switch (bst[i]) {
                case VC_DNSD_REJECTED: snprintf(buf, sizeof buf, "S %lld ", g); break;
                case VC_DNSD_RESPONSE: snprintf(buf, sizeof buf, "P %lld ", g); break;
                case VC_DNSD_RECURSIVE: snprintf(buf, sizeof buf, "R %lld ", g); break;
                case VC_DNSD_HOST: snprintf(buf, sizeof buf, "J %lld ", g); break;
                case VC_DNSD_EMPTY:
                case VC_DNSD_MALFORMED:
                    /* return: the rest of the batch stays pending for the next event */
                    snprintf(buf, sizeof buf, "E %lld | ", g);
                    event_over = 1;
                    head = lo + i + 1;
                    break;
                case VC_DNSD_ANSWER: {
                    int q, p = snprintf(buf, sizeof buf, "A %lld %d", g, bnq[i]);
                    for (q = 0; q < bnq[i] && p < (int) sizeof buf - 32; ++q)
                        p += snprintf(buf + p, sizeof buf - (size_t) p, " %d:%d",
                                      bkind[i * VC_DNSD_MAXQ + q], bval[i * VC_DNSD_MAXQ + q]);
                    snprintf(buf + p, sizeof buf - (size_t) p, " ");
                    break;
                }
                default:
                    snprintf(buf, sizeof buf, "? %lld ", g);
                }
                put(&t, buf);
                if (event_over) break;
            }
        }
    }
done:
    free(bb); free(boff); free(bfam); free(br4); free(br6); free(bport); free(bst); free(bnq);
    free(bkind); free(bqt); free(bacl); free(bval);
    return rc;
}

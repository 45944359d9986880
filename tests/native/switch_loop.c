/*
 * switch_loop.c -- test-only C replay of jni/SwitchDrainBatcher.java: the
 * vswitch's UDP drain loop (core/src/main/java/vswitch/Switch.java:744-776
 * with handleNetworkAndGetVXLanPacket :643-731) run in batches through
 * vc_switch_classify, with the batcher's receive rule, its per-datagram
 * decision table and its fallback, so the GPU tier can check that the
 * classify contract reproduces the reference loop's action sequence at any
 * batch size (tests/test_gpu_switch_loop.py) and the CPU tier the fallback
 * (tests/test_switch_loop_cpu.py).  Built as a shared library, called
 * through ctypes with a context the ctypes layer compiled.
 *
 * The "socket" is the input queue; `decrypt[i]` stands for
 * VProxyEncryptedPacket.from(data) succeeding on datagram i (user-iface
 * traffic, decided in Java before the batch is built).  One readable event
 * receives datagrams until a read returns 0 bytes (an empty datagram, or the
 * end of the queue), dispatching a batch whenever `batch` datagrams or the
 * blob's bytes are reached, exactly as SwitchDrainBatcher.readable; one
 * vc_switch_classify call classifies a batch's bare datagrams; then, in
 * arrival order:
 *   decrypted                     -> "E i"        Host.handleEncrypted     (:650-676)
 *   call failed                   -> "J i"        Host.handleJava (reference body)
 *   bareVXLanAccess denies        -> "S i"        dropped                  (:711-714)
 *   parse throws / never returns  -> "J i"        the reference body      (VC_PKT_EXCEPTION / LOOP)
 *   parse error                   -> "X i"        dropped                  (:684-687)
 *   parsed                        -> "B i route"  Host.handleBare          (:688-731, L3 route)
 * An event ends with "|".  VC_EDEVICE / VC_ENOMEM (IOException in the shim)
 * marks the context dead for good ("D"), VC_ESTATE (IllegalStateException)
 * affects that batch only ("F").
 */
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "vclassify.h"

#define MAX_DATAGRAM 65536
#define BLOB_PER_SLOT 256          /* SwitchDrainBatcher: cap * 256 + MAX_DATAGRAM bytes */

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

/* inject[b] != 0: call b "returns" that status instead of running */
int switch_loop_trace(vc_ctx *ctx, const uint8_t *blob, const uint32_t *off, int64_t n,
                      const uint8_t *decrypt, const uint8_t *fam, const uint32_t *r4,
                      const uint8_t *r6, int bind_port, int batch, const int *inject,
                      int n_inject, char *out, int64_t cap) {
    trace_t t = {out, cap, 0};
    int64_t head = 0;                  /* next datagram the socket hands out */
    int dead = 0, calls = 0, rc = 0;
    char buf[96];
    const size_t blob_cap = (size_t) batch * BLOB_PER_SLOT + MAX_DATAGRAM;
    uint8_t *bb, *bfam, *bst, *ballow, *br6;
    uint32_t *boff, *br4;
    int32_t *bacl, *broute;
    int64_t *idx;                      /* datagrams of the batch, arrival order */
    int *bare;                         /* their bare index, -1 when decrypted */
    if (batch < 1 || cap < 1 || n < 0) return VC_EINVAL;
    out[0] = 0;
    bb = malloc(blob_cap);
    boff = malloc(sizeof(uint32_t) * (size_t) (batch + 1));
    bfam = malloc((size_t) batch);
    br4 = malloc(sizeof(uint32_t) * (size_t) batch);
    br6 = aligned_alloc(16, 16 * (size_t) batch);
    bst = malloc((size_t) batch);
    ballow = malloc((size_t) batch);
    bacl = malloc(sizeof(int32_t) * (size_t) batch);
    broute = malloc(sizeof(int32_t) * (size_t) batch);
    idx = malloc(sizeof(int64_t) * (size_t) batch);
    bare = malloc(sizeof(int) * (size_t) batch);
    while (head < n) {                                 /* readable events */
        int drained = 0;
        while (!drained) {                             /* SwitchDrainBatcher.readable */
            int m = 0, nb = 0, i, status = VC_OK;
            size_t bytes = 0;
            boff[0] = 0;
            for (;;) {                                 /* receive a batch */
                uint32_t len;
                if (m == batch || bytes + MAX_DATAGRAM > blob_cap) break;
                if (head >= n) {                       /* nothing read: quit (:757-759) */
                    drained = 1;
                    break;
                }
                len = off[head + 1] - off[head];
                if (len == 0) {                        /* an empty datagram reads as nothing too */
                    ++head;
                    drained = 1;
                    break;
                }
                idx[m] = head;
                if (decrypt[head]) {
                    bare[m] = -1;
                } else {
                    bare[m] = nb;
                    memcpy(bb + bytes, blob + off[head], len);
                    boff[nb + 1] = boff[nb] + len;
                    bfam[nb] = fam[head];
                    br4[nb] = r4[head];
                    memcpy(br6 + 16 * nb, r6 + 16 * head, 16);
                    bytes += len;
                    ++nb;
                }
                ++m;
                ++head;
            }
            if (nb > 0) {                              /* GpuContext.batch around the call */
                status = dead ? VC_EDEVICE
                              : calls < n_inject && inject[calls] ? inject[calls] : VC_OK;
                ++calls;
                if (status == VC_OK) {
                    vc_pkt_out o;
                    memset(&o, 0, sizeof o);
                    o.status = bst;
                    status = vc_switch_classify(ctx, bb, boff, nb, VC_LAYER_VXLAN, bfam, br4, br6,
                                                bind_port, &o, bacl, ballow, broute);
                    if (status != VC_OK && status != VC_ESTATE && status != VC_EDEVICE &&
                        status != VC_ENOMEM) {
                        rc = status;                   /* a caller bug: rethrown */
                        goto done;
                    }
                }
                if (status != VC_OK) {
                    if (!dead) put(&t, status == VC_ESTATE ? "F " : "D ");
                    if (status != VC_ESTATE) dead = 1;
                }
            }
            for (i = 0; i < m; ++i) {                  /* dispatch, arrival order */
                const long long g = (long long) idx[i];
                const int k = bare[i];
                if (k < 0) snprintf(buf, sizeof buf, "E %lld ", g);
                else if (status != VC_OK) snprintf(buf, sizeof buf, "J %lld ", g);
                else if (!ballow[k]) snprintf(buf, sizeof buf, "S %lld ", g);
                else if (bst[k] == VC_PKT_EXCEPTION || bst[k] == VC_PKT_LOOP)
                    snprintf(buf, sizeof buf, "J %lld ", g);
                else if (bst[k] != VC_PKT_OK) snprintf(buf, sizeof buf, "X %lld ", g);
                else snprintf(buf, sizeof buf, "B %lld %d ", g, broute[k]);
                put(&t, buf);
            }
        }
        put(&t, "| ");
    }
done:
    free(bb); free(boff); free(bfam); free(br4); free(br6); free(bst); free(ballow);
    free(bacl); free(broute); free(idx); free(bare);
    return rc;
}

/*
 * vc_oracle.c -- CPU restatement of vproxy's classification hot path.
 *
 * TEST INFRASTRUCTURE ONLY (see vc_oracle.h).  Plain C, linear scans exactly
 * as the Java reference does them; no tries, no hashing.  Each function
 * cites the reference file:line it restates (paths under /root/reference).
 */
#define _GNU_SOURCE
#include "vc_oracle.h"

#include <pthread.h>
#include <stdlib.h>
#include <string.h>

/* ------------------------------------------------------------------------ */
/* Java String helpers over ASCII bytes                                     */
/* ------------------------------------------------------------------------ */

static int j_index_of(const char *s, int n, const char *e, int en, int from)
{
    if (from < 0) from = 0;
    for (int i = from; i + en <= n; ++i)
        if (memcmp(s + i, e, (size_t)en) == 0) return i;
    return -1;
}

static int j_index_of_ch(const char *s, int n, char c)
{
    for (int i = 0; i < n; ++i)
        if (s[i] == c) return i;
    return -1;
}

static int j_last_index_of_ch(const char *s, int n, char c, int from)
{
    if (from >= n) from = n - 1;
    for (int i = from; i >= 0; --i)
        if (s[i] == c) return i;
    return -1;
}

static int j_starts_with(const char *s, int n, const char *p, int pn)
{
    return n >= pn && memcmp(s, p, (size_t)pn) == 0;
}

static int j_ends_with(const char *s, int n, const char *p, int pn)
{
    return n >= pn && memcmp(s + n - pn, p, (size_t)pn) == 0;
}

static int j_equals(const char *a, int an, const char *b, int bn)
{
    return an == bn && memcmp(a, b, (size_t)an) == 0;
}

/* Utils.split (base/src/main/java/vproxybase/util/Utils.java:162-177):
 * splits on the literal e, keeping every empty piece.  Writes piece offsets
 * and lengths; returns the piece count (<= n + 1). */
static int j_split(const char *s, int n, const char *e, int en, int *off, int *len)
{
    int cnt = 0;
    int idx = -en;
    int last = 0;
    for (;;) {
        idx = j_index_of(s, n, e, en, idx + en);
        if (idx == -1) {
            off[cnt] = last;
            len[cnt] = n - last;
            ++cnt;
            break;
        }
        off[cnt] = last;
        len[cnt] = idx - last;
        ++cnt;
        last = idx + en;
    }
    return cnt;
}

static int hexval(char c)
{
    if (c >= '0' && c <= '9') return c - '0';
    if (c >= 'a' && c <= 'f') return c - 'a' + 10;
    return c - 'A' + 10;
}

/* ------------------------------------------------------------------------ */
/* IP.java parsers                                                          */
/* ------------------------------------------------------------------------ */

/* IP.parseIpv4String(String, byte[], int) -- IP.java:129-155 */
static int parse_ipv4_into(const char *s, int n, uint8_t *bytes, int cap, int from_idx)
{
    int off[64], len[64];
    /* more than 63 dots can never be 4 pieces; bail before overflow */
    int dots = 0;
    for (int i = 0; i < n; ++i) dots += (s[i] == '.');
    if (dots != 3) return -1;
    int cnt = j_split(s, n, ".", 1, off, len);
    if (cnt != 4) return -1;
    for (int i = 0; i < cnt; ++i) {
        int idx = from_idx + i;
        if (idx >= cap) return -1;
        const char *p = s + off[i];
        int l = len[i];
        if (l > 3 || l == 0) return -1;
        for (int k = 0; k < l; ++k)
            if (p[k] < '0' || p[k] > '9') return -1;
        if (p[0] == '0' && l > 1) return -1;
        int num = 0;
        for (int k = 0; k < l; ++k) num = num * 10 + (p[k] - '0');
        if (num > 255) return -1;
        bytes[idx] = (uint8_t)num;
    }
    return cnt;
}

int vo_parse_ipv4(const char *s, int len, uint8_t out[4])
{
    uint8_t b[4] = {0, 0, 0, 0};
    if (parse_ipv4_into(s, len, b, 4, 0) == -1) return -1;
    memcpy(out, b, 4);
    return 4;
}

/* IP.parseIpv6ColonPart -- IP.java:200-248 (s == NULL is Java null) */
static int parse_ipv6_colon_part(const char *s, int n, uint8_t *bytes, int from_idx)
{
    if (s == NULL || n == 0) return 0;
    if (from_idx < 0) return -1;
    int *off = (int *)malloc(sizeof(int) * (size_t)(n + 1));
    int *len = (int *)malloc(sizeof(int) * (size_t)(n + 1));
    int cnt = j_split(s, n, ":", 1, off, len);
    int ret = cnt * 2;
    for (int i = 0; i < cnt; ++i) {
        int base = from_idx + 2 * i;
        if (base >= 16) { ret = -1; break; }
        const char *f = s + off[i];
        int l = len[i];
        if (l > 4 || l == 0) { ret = -1; break; }
        int bad = 0;
        for (int k = 0; k < l; ++k) {
            char c = f[k];
            if ((c < 'A' || c > 'F') && (c < 'a' || c > 'f') && (c < '0' || c > '9')) bad = 1;
        }
        if (bad) { ret = -1; break; }
        switch (l) {
        case 1: bytes[base + 1] = (uint8_t)hexval(f[0]); break;
        case 2: bytes[base + 1] = (uint8_t)(hexval(f[0]) * 16 + hexval(f[1])); break;
        case 3:
            bytes[base] = (uint8_t)hexval(f[0]);
            bytes[base + 1] = (uint8_t)(hexval(f[1]) * 16 + hexval(f[2]));
            break;
        case 4:
            bytes[base] = (uint8_t)(hexval(f[0]) * 16 + hexval(f[1]));
            bytes[base + 1] = (uint8_t)(hexval(f[2]) * 16 + hexval(f[3]));
            break;
        }
    }
    free(off);
    free(len);
    return ret;
}

static int count_pieces(const char *s, int n, char c)
{
    int k = 1;
    for (int i = 0; i < n; ++i) k += (s[i] == c);
    return k;
}

/* IP.parseIpv6LastBits -- IP.java:251-269.  NB the `4 + colonPart` sum at
 * :264 turns a failed colon part (-1) into 3, which the caller accepts when a
 * "::" is present; restated verbatim. */
static int parse_ipv6_last_bits(const char *s, int n, uint8_t *bytes)
{
    int dot = j_index_of_ch(s, n, '.');
    if (dot != -1) {
        int idx = j_last_index_of_ch(s, n, ':', dot);
        if (idx == -1) {
            return parse_ipv4_into(s, n, bytes, 16, 12);
        } else {
            const char *colon = s;
            int colon_n = idx;
            const char *dotp = s + idx + 1;
            int dot_n = n - idx - 1;
            int r = parse_ipv4_into(dotp, dot_n, bytes, 16, 12);
            if (r == -1) return -1;
            return 4 + parse_ipv6_colon_part(colon, colon_n, bytes,
                                             16 - 4 - count_pieces(colon, colon_n, ':') * 2);
        }
    } else {
        return parse_ipv6_colon_part(s, n, bytes, 16 - count_pieces(s, n, ':') * 2);
    }
}

/* IP.parseIpv6String -- IP.java:158-197 */
int vo_parse_ipv6(const char *s, int n, uint8_t out[16])
{
    if (j_starts_with(s, n, "[", 1) && j_ends_with(s, n, "]", 1) && n >= 1) {
        /* Java substring(1, len-1) on "[" alone would throw; "[" does not end
         * with "]" unless n >= 2, except the one-char string "]"... which does
         * not start with "[".  So n >= 2 here. */
        s = s + 1;
        n = n - 2;
    }
    {
        /* count of "::" pieces - 1 */
        int pieces = 1;
        int idx = -2;
        for (;;) {
            idx = j_index_of(s, n, "::", 2, idx + 2);
            if (idx == -1) break;
            ++pieces;
        }
        if (pieces - 1 > 1) return -1;
    }
    int has_dbl;
    const char *colon_only;
    int colon_only_n;
    const char *colon_and_dot;
    int colon_and_dot_n;
    int idx = j_index_of(s, n, "::", 2, 0);
    if (idx == -1) {
        has_dbl = 0;
        colon_only = NULL;
        colon_only_n = 0;
        colon_and_dot = s;
        colon_and_dot_n = n;
    } else {
        has_dbl = 1;
        colon_only = s;
        colon_only_n = idx;
        colon_and_dot = s + idx + 2;
        colon_and_dot_n = n - idx - 2;
    }
    uint8_t b[16];
    memset(b, 0, sizeof b);
    int consumed = parse_ipv6_colon_part(colon_only, colon_only_n, b, 0);
    if (consumed == -1) return -1;
    int consumed2 = parse_ipv6_last_bits(colon_and_dot, colon_and_dot_n, b);
    if (consumed2 == -1) return -1;
    if (has_dbl) {
        if (consumed + consumed2 >= 16) return -1;
    } else {
        if (consumed + consumed2 != 16) return -1;
    }
    memcpy(out, b, 16);
    return 16;
}

/* IP.parseIpString -- IP.java:112-117 */
int vo_parse_ip(const char *s, int n, uint8_t out[16])
{
    if (j_index_of_ch(s, n, ':') != -1) return vo_parse_ipv6(s, n, out);
    return vo_parse_ipv4(s, n, out);
}

int vo_is_ipv6(const char *s, int n)
{
    uint8_t b[16];
    return vo_parse_ipv6(s, n, b) != -1;
}

/* IP.isIpLiteral = isIpv4 || isIpv6 (IP.java:271-300).  isIpv4 goes through
 * parseIpv4StringConsiderV6Compatible: a parseable v6 string answers there
 * (null or not), but then isIpv6 is true anyway, so the disjunction reduces
 * to v6-parses || v4-parses. */
int vo_is_ip_literal(const char *s, int n)
{
    uint8_t b[16];
    if (vo_parse_ipv6(s, n, b) != -1) return 1;
    return vo_parse_ipv4(s, n, b) != -1;
}

/* ------------------------------------------------------------------------ */
/* Network.java                                                             */
/* ------------------------------------------------------------------------ */

/* Utils.getByte -- Utils.java:137-160 */
static uint8_t get_byte(int ones)
{
    switch (ones) {
    case 8: return 0xFF;
    case 7: return 0xFE;
    case 6: return 0xFC;
    case 5: return 0xF8;
    case 4: return 0xF0;
    case 3: return 0xE0;
    case 2: return 0xC0;
    case 1: return 0x80;
    default: return 0;
    }
}

/* Utils.zeros -- Utils.java:94-104 (trailing zero bits of a byte, 8 for 0) */
static int zeros(uint8_t b)
{
    for (int k = 0; k < 8; ++k)
        if (b & (1u << k)) return k;
    return 8;
}

/* Network.parseMask + getMask -- Network.java:101-133 */
int vo_parse_mask(int m, uint8_t out[16])
{
    if (m > 128) return -1;
    int len = m > 32 ? 16 : 4;
    for (int i = 0; i < len; ++i) {
        out[i] = get_byte(m > 8 ? 8 : m);
        m -= 8;
    }
    return len;
}

/* Network.maskInt -- Network.java:135-145 */
int vo_mask_int(const uint8_t *mask, int mlen)
{
    int m = 0;
    for (int i = mlen - 1; i >= 0; --i) {
        int cnt = zeros(mask[i]);
        if (cnt == 0) break;
        m += cnt;
    }
    return mlen * 8 - m;
}

/* Network.validNetwork -- Network.java:163-181 */
int vo_valid_network(const uint8_t *a, int alen, const uint8_t *m, int mlen)
{
    if (alen < mlen) return 0;
    for (int i = 0; i < mlen; ++i) {
        int ab = (int8_t)a[i], mb = (int8_t)m[i];
        if ((ab & mb) != ab) return 0;
    }
    for (int i = mlen; i < alen; ++i)
        if (a[i] != 0) return 0;
    return 1;
}

/* Utils.lowBitsV6V4 -- Utils.java:122-133 */
static int low_bits_v6v4(const uint8_t *ip, int last, int second)
{
    for (int i = 0; i < second; ++i)
        if (ip[i] != 0) return 0;
    if (ip[last] == 0) return ip[second] == 0;
    if (ip[last] == 0xFF) return ip[second] == 0xFF;
    return 0;
}

static int byte_ne(uint8_t in, uint8_t mask, uint8_t rule)
{
    /* Java: (inputB & maskB) != ruleB over sign-extended ints */
    return (((int)(int8_t)in) & ((int)(int8_t)mask)) != (int)(int8_t)rule;
}

/* Network.maskMatch -- Network.java:183-278 (five length cases) */
int vo_mask_match(const uint8_t *in, int inlen, const uint8_t *rule, int rlen,
                  const uint8_t *mask, int mlen)
{
    if (inlen == rlen && rlen > mlen) {                      /* case 1 */
        for (int i = 0; i < mlen; ++i)
            if (byte_ne(in[i], mask[i], rule[i])) return 0;
        return 1;
    } else if (inlen < rlen && rlen > mlen) {                /* case 2 */
        return 0;
    } else if (inlen < rlen && rlen == mlen) {               /* case 3 */
        int last = rlen - inlen - 1;
        int second = last - 1;
        for (int i = 0; i < inlen; ++i)
            if (byte_ne(in[i], mask[i + rlen - inlen], rule[i + rlen - inlen])) return 0;
        return low_bits_v6v4(rule, last, second);
    }
    int min_len = inlen;                                     /* cases 4, 5 */
    if (rlen < min_len) min_len = rlen;
    if (mlen < min_len) min_len = mlen;
    for (int i = 0; i < min_len; ++i)
        if (byte_ne(in[inlen - i - 1], mask[mlen - i - 1], rule[rlen - i - 1])) return 0;
    if (inlen > rlen) {
        int last = inlen - rlen - 1;
        int second = last - 1;
        return low_bits_v6v4(in, last, second);
    }
    return 1;
}

/* Network(String) -- Network.java:16-25 via validNetworkStr :73-99 */
int vo_net_from_str(const char *s, int n, vo_net *out)
{
    int slash = j_index_of_ch(s, n, '/');
    if (slash == -1) return -1;
    /* net.split("/") must give exactly 2 pieces: one '/', non-empty tail */
    int slashes = 0;
    for (int i = 0; i < n; ++i) slashes += s[i] == '/';
    if (slashes != 1 || slash == n - 1 || slash == 0) return -1;
    const char *ms = s + slash + 1;
    int mn = n - slash - 1;
    /* Integer.parseInt: optional sign then digits */
    int k = 0, neg = 0;
    if (ms[0] == '-' || ms[0] == '+') { neg = ms[0] == '-'; k = 1; }
    if (k >= mn) return -1;
    long v = 0;
    for (; k < mn; ++k) {
        if (ms[k] < '0' || ms[k] > '9') return -1;
        v = v * 10 + (ms[k] - '0');
        if (v > 2147483648L) return -1;
    }
    if (neg) v = -v;
    if (v > 2147483647L) return -1;
    memset(out, 0, sizeof *out);
    int iplen = vo_parse_ip(s, slash, out->ip);
    if (iplen == -1) return -1;
    int mlen = vo_parse_mask((int)v, out->mask);
    if (mlen == -1) return -1;
    if (!vo_valid_network(out->ip, iplen, out->mask, mlen)) return -1;
    out->ip_len = iplen;
    out->mask_len = mlen;
    return 0;
}

int vo_net_contains_ip(const vo_net *n, const uint8_t *ip, int iplen)
{
    return vo_mask_match(ip, iplen, n->ip, n->ip_len, n->mask, n->mask_len);
}

/* Network.contains(Network) -- Network.java:31-36 */
int vo_net_contains_net(const vo_net *a, const vo_net *b)
{
    if (!vo_net_contains_ip(a, b->ip, b->ip_len)) return 0;
    return vo_mask_int(a->mask, a->mask_len) < vo_mask_int(b->mask, b->mask_len);
}

int vo_net_equals(const vo_net *a, const vo_net *b)
{
    return a->ip_len == b->ip_len && a->mask_len == b->mask_len &&
           memcmp(a->ip, b->ip, (size_t)a->ip_len) == 0 &&
           memcmp(a->mask, b->mask, (size_t)a->mask_len) == 0;
}

/* ------------------------------------------------------------------------ */
/* SecurityGroup.allow -- SecurityGroup.java:30-45, SecurityGroupRule:27-29  */
/* ------------------------------------------------------------------------ */

int vo_sg_allow(const vo_sg_rule *tcp, int ntcp, const vo_sg_rule *udp, int nudp,
                int default_allow, int proto, const uint8_t *ip, int iplen, int port,
                int *verdict)
{
    const vo_sg_rule *rules = proto == 6 ? tcp : udp;
    int n = proto == 6 ? ntcp : nudp;
    if (n == 0) {
        if (verdict) *verdict = default_allow;
        return -1;
    }
    for (int i = 0; i < n; ++i) {
        const vo_sg_rule *r = &rules[i];
        if (vo_net_contains_ip(&r->net, ip, iplen) && r->min_port <= port && port <= r->max_port) {
            if (verdict) *verdict = r->allow;
            return i;
        }
    }
    if (verdict) *verdict = default_allow;
    return -1;
}

/* ---- pthread partition helper ---- */
typedef void (*range_fn)(void *ctx, int64_t lo, int64_t hi);
typedef struct { range_fn fn; void *ctx; int64_t lo, hi; } range_job;

static void *range_thread(void *p)
{
    range_job *j = (range_job *)p;
    j->fn(j->ctx, j->lo, j->hi);
    return NULL;
}

static void parallel_for(int64_t n, int nthreads, range_fn fn, void *ctx)
{
    if (nthreads <= 1 || n < 2) {
        fn(ctx, 0, n);
        return;
    }
    if (nthreads > 1024) nthreads = 1024;
    if (nthreads > n) nthreads = (int)n;
    pthread_t th[1024];
    range_job jobs[1024];
    int started[1024];
    for (int t = 0; t < nthreads; ++t) {
        jobs[t].fn = fn;
        jobs[t].ctx = ctx;
        jobs[t].lo = n * t / nthreads;
        jobs[t].hi = n * (t + 1) / nthreads;
        /* a thread the system refuses runs its range here instead */
        started[t] = pthread_create(&th[t], NULL, range_thread, &jobs[t]) == 0;
        if (!started[t]) fn(ctx, jobs[t].lo, jobs[t].hi);
    }
    for (int t = 0; t < nthreads; ++t)
        if (started[t]) pthread_join(th[t], NULL);
}

typedef struct {
    const vo_sg_rule *tcp; int ntcp; const vo_sg_rule *udp; int nudp; int dflt;
    const uint8_t *proto; const uint32_t *src4; const uint8_t *src6; const uint16_t *port;
    int32_t *out; uint8_t *verdict;
} sg_batch_ctx;

static void sg_v4_range(void *p, int64_t lo, int64_t hi)
{
    sg_batch_ctx *c = (sg_batch_ctx *)p;
    for (int64_t i = lo; i < hi; ++i) {
        uint32_t a = c->src4[i];
        uint8_t ip[4] = {(uint8_t)(a >> 24), (uint8_t)(a >> 16), (uint8_t)(a >> 8), (uint8_t)a};
        int v;
        c->out[i] = vo_sg_allow(c->tcp, c->ntcp, c->udp, c->nudp, c->dflt, c->proto[i], ip, 4,
                                c->port[i], &v);
        if (c->verdict) c->verdict[i] = (uint8_t)v;
    }
}

static void sg_v6_range(void *p, int64_t lo, int64_t hi)
{
    sg_batch_ctx *c = (sg_batch_ctx *)p;
    for (int64_t i = lo; i < hi; ++i) {
        int v;
        c->out[i] = vo_sg_allow(c->tcp, c->ntcp, c->udp, c->nudp, c->dflt, c->proto[i],
                                c->src6 + 16 * i, 16, c->port[i], &v);
        if (c->verdict) c->verdict[i] = (uint8_t)v;
    }
}

void vo_sg_allow_batch_v4(const vo_sg_rule *tcp, int ntcp, const vo_sg_rule *udp, int nudp,
                          int default_allow, const uint8_t *proto, const uint32_t *src4,
                          const uint16_t *port, int64_t n, int32_t *out_idx, uint8_t *out_verdict,
                          int nthreads)
{
    sg_batch_ctx c = {tcp, ntcp, udp, nudp, default_allow, proto, src4, NULL, port, out_idx, out_verdict};
    parallel_for(n, nthreads, sg_v4_range, &c);
}

void vo_sg_allow_batch_v6(const vo_sg_rule *tcp, int ntcp, const vo_sg_rule *udp, int nudp,
                          int default_allow, const uint8_t *proto, const uint8_t *src6,
                          const uint16_t *port, int64_t n, int32_t *out_idx, uint8_t *out_verdict,
                          int nthreads)
{
    sg_batch_ctx c = {tcp, ntcp, udp, nudp, default_allow, proto, NULL, src6, port, out_idx, out_verdict};
    parallel_for(n, nthreads, sg_v6_range, &c);
}

/* ------------------------------------------------------------------------ */
/* RouteTable -- core/src/main/java/vswitch/RouteTable.java                 */
/* ------------------------------------------------------------------------ */

void vo_rt_init(vo_route_table *t) { memset(t, 0, sizeof *t); }

void vo_rt_free(vo_route_table *t)
{
    free(t->v4);
    free(t->v6);
    memset(t, 0, sizeof *t);
}

/* RouteTable.addRule(RouteRule, List) -- RouteTable.java:110-154 */
static void rt_insert(vo_net **list, int *n, int *cap, const vo_net *r)
{
    int similar = -1;
    for (int i = 0; i < *n; ++i) {
        const vo_net *ri = &(*list)[i];
        if (vo_net_contains_net(ri, r) || vo_net_contains_net(r, ri)) {
            similar = i;
            break;
        }
    }
    int insert_index;
    if (similar == -1) {
        insert_index = *n;
    } else {
        insert_index = 0;
        for (int i = similar; i < *n; ++i) {
            const vo_net *curr = &(*list)[i];
            const vo_net *next = (i + 1) < *n ? &(*list)[i + 1] : NULL;
            if (vo_net_contains_net(curr, r)) {
                insert_index = i;
                break;
            }
            if (vo_net_contains_net(r, curr)) {
                if (next == NULL) {
                    insert_index = i + 1;
                    break;
                }
                if (vo_net_contains_net(r, next)) continue;
                if (vo_net_contains_net(next, r)) {
                    insert_index = i + 1;
                    break;
                }
            }
            insert_index = i + 1;
            break;
        }
    }
    if (*n == *cap) {
        *cap = *cap ? *cap * 2 : 16;
        *list = (vo_net *)realloc(*list, sizeof(vo_net) * (size_t)*cap);
    }
    memmove(&(*list)[insert_index + 1], &(*list)[insert_index],
            sizeof(vo_net) * (size_t)(*n - insert_index));
    (*list)[insert_index] = *r;
    ++*n;
}

/* RouteTable.addRule(RouteRule) -- RouteTable.java:68-108 (network part) */
int vo_rt_add(vo_route_table *t, const vo_net *r)
{
    for (int i = 0; i < t->n4; ++i)
        if (vo_net_equals(&t->v4[i], r)) return -1;
    for (int i = 0; i < t->n6; ++i)
        if (vo_net_equals(&t->v6[i], r)) return -1;
    if (r->ip_len == 4) rt_insert(&t->v4, &t->n4, &t->cap4, r);
    else rt_insert(&t->v6, &t->n6, &t->cap6, r);
    return 0;
}

int vo_rt_lookup_list(const vo_net *list, int n, const uint8_t *ip, int iplen)
{
    for (int i = 0; i < n; ++i)
        if (vo_net_contains_ip(&list[i], ip, iplen)) return i;
    return -1;
}

/* RouteTable.lookup -- RouteTable.java:44-59 */
int vo_rt_lookup(const vo_route_table *t, const uint8_t *ip, int iplen)
{
    if (iplen == 4) return vo_rt_lookup_list(t->v4, t->n4, ip, iplen);
    return vo_rt_lookup_list(t->v6, t->n6, ip, iplen);
}

typedef struct {
    const vo_net *list; int nl; const uint32_t *d4; const uint8_t *d6; int32_t *out;
} rt_batch_ctx;

static void rt_v4_range(void *p, int64_t lo, int64_t hi)
{
    rt_batch_ctx *c = (rt_batch_ctx *)p;
    for (int64_t i = lo; i < hi; ++i) {
        uint32_t a = c->d4[i];
        uint8_t ip[4] = {(uint8_t)(a >> 24), (uint8_t)(a >> 16), (uint8_t)(a >> 8), (uint8_t)a};
        c->out[i] = vo_rt_lookup_list(c->list, c->nl, ip, 4);
    }
}

static void rt_v6_range(void *p, int64_t lo, int64_t hi)
{
    rt_batch_ctx *c = (rt_batch_ctx *)p;
    for (int64_t i = lo; i < hi; ++i)
        c->out[i] = vo_rt_lookup_list(c->list, c->nl, c->d6 + 16 * i, 16);
}

void vo_rt_lookup_batch_v4(const vo_net *v4, int n4, const uint32_t *dst4, int64_t n,
                           int32_t *out, int nthreads)
{
    rt_batch_ctx c = {v4, n4, dst4, NULL, out};
    parallel_for(n, nthreads, rt_v4_range, &c);
}

void vo_rt_lookup_batch_v6(const vo_net *v6, int n6, const uint8_t *dst6, int64_t n,
                           int32_t *out, int nthreads)
{
    rt_batch_ctx c = {v6, n6, NULL, dst6, out};
    parallel_for(n, nthreads, rt_v6_range, &c);
}

/* ------------------------------------------------------------------------ */
/* Hint -- base/src/main/java/vproxybase/processor/Hint.java                */
/* ------------------------------------------------------------------------ */

/* Hint.formatHost -- Hint.java:57-73 */
int vo_format_host(const char *s, int len, int *off, int *olen)
{
    if (s == NULL) return 0;
    int colon = j_index_of_ch(s, len, ':');
    if (vo_is_ipv6(s, len) || colon == -1) {
        *off = 0;
        *olen = len;
        return 1;
    }
    int o = 0, l = colon;
    if (j_starts_with(s, l, "www.", 4)) {
        o = 4;
        l -= 4;
    }
    if (l == 0) return 0;
    *off = o;
    *olen = l;
    return 1;
}

/* Hint.formatUri -- Hint.java:75-90 */
int vo_format_uri(const char *s, int len, int *off, int *olen)
{
    if (s == NULL) return 0;
    int q = j_index_of_ch(s, len, '?');
    if (q != -1) len = q;
    *off = 0;
    if (len == 1 && s[0] == '/') {
        *olen = 1;
        return 1;
    }
    if (len > 0 && s[len - 1] == '/') len -= 1;
    *olen = len;
    return 1;
}

/* Hint.ofHostPortUri and friends -- Hint.java:17-55 */
vo_hint vo_hint_of(const char *host, int host_len, int port, const char *uri, int uri_len)
{
    vo_hint h;
    int off, l;
    if (vo_format_host(host, host_len, &off, &l)) {
        h.host = host + off;
        h.host_len = l;
    } else {
        h.host = NULL;
        h.host_len = 0;
    }
    h.port = port;
    if (vo_format_uri(uri, uri_len, &off, &l)) {
        h.uri = uri + off;
        h.uri_len = l;
    } else {
        h.uri = NULL;
        h.uri_len = 0;
    }
    return h;
}

/* String.length() of the Java string whose UTF-8 bytes (WTF-8 for unpaired
 * surrogates: the boundary's string encoding, include/vclassify.h) are s:
 * one UTF-16 unit per code point, two for a supplementary code point. */
static int j_length(const char *s, int n)
{
    int u = 0;
    for (int i = 0; i < n; ++i) {
        unsigned char c = (unsigned char)s[i];
        if ((c & 0xC0) != 0x80) ++u;
        if (c >= 0xF0) ++u;
    }
    return u;
}

/* Hint.matchLevel -- Hint.java:100-160 */
int vo_match_level(const vo_hint *h, const vo_annos *a, int na)
{
    const char *ah = NULL; int ahn = 0;
    int ap = 0;
    const char *au = NULL; int aun = 0;
    for (int i = 0; i < na; ++i) {
        if (ah == NULL) { ah = a[i].host; ahn = a[i].host_len; }
        if (ap == 0) ap = a[i].port;
        if (au == NULL) { au = a[i].uri; aun = a[i].uri_len; }
    }
    if (ah == NULL && ap == 0 && au == NULL) return 0;
    if (h->port != 0 && ap != 0 && h->port != ap) return 0;
    int level = 0;
    int host_level = 0;
    if (ah != NULL && h->host != NULL) {
        if (j_equals(h->host, h->host_len, ah, ahn)) {
            host_level = 3;
        } else if (h->host_len >= ahn + 1 && h->host[h->host_len - ahn - 1] == '.' &&
                   memcmp(h->host + h->host_len - ahn, ah, (size_t)ahn) == 0) {
            host_level = 2;  /* host.endsWith("." + annoHost) */
        } else if (j_equals(ah, ahn, "*", 1)) {
            host_level = 1;
        }
    }
    level += host_level << 10;
    int uri_level = 0;
    if (au != NULL && h->uri != NULL) {
        if (j_equals(h->uri, h->uri_len, au, aun)) {
            uri_level = j_length(h->uri, h->uri_len) + 1;    /* this.uri.length() + 1 */
        } else if (j_starts_with(h->uri, h->uri_len, au, aun)) {
            uri_level = j_length(au, aun) + 1;               /* annoUri.length() + 1 */
        } else if (j_equals(au, aun, "*", 1)) {
            uri_level = 1;
        }
    }
    if (uri_level > 1023) uri_level = 1023;
    level += uri_level;
    return level;
}

/* Upstream.searchForGroup -- Upstream.java:187-198 */
int vo_search_for_group(const vo_group *g, int ng, const vo_hint *h)
{
    int level = 0;
    int last_max = -1;
    for (int i = 0; i < ng; ++i) {
        vo_annos a[2] = {g[i].handle, g[i].group};
        int l = vo_match_level(h, a, 2);
        if (l > level) {
            level = l;
            last_max = i;
        }
    }
    return last_max;
}

typedef struct {
    const vo_group *g; int ng; const uint8_t *blob; const uint32_t *off; const uint16_t *port;
    int32_t *out;
} hint_batch_ctx;

static void hint_range(void *p, int64_t lo, int64_t hi)
{
    hint_batch_ctx *c = (hint_batch_ctx *)p;
    for (int64_t i = lo; i < hi; ++i) {
        const char *s = (const char *)c->blob + c->off[i];
        int len = (int)(c->off[i + 1] - c->off[i]);
        vo_hint h = vo_hint_of(s, len, c->port ? c->port[i] : 0, NULL, 0);
        c->out[i] = vo_search_for_group(c->g, c->ng, &h);
    }
}

void vo_hint_batch(const vo_group *g, int ng, const uint8_t *blob, const uint32_t *off,
                   const uint16_t *port, int64_t n, int32_t *out, int nthreads)
{
    hint_batch_ctx c = {g, ng, blob, off, port, out};
    parallel_for(n, nthreads, hint_range, &c);
}

/* searchForGroup(Hint.ofHostPortUri(host, port, uri)) per item: the hint
 * HttpContext.connectionHint builds for an HTTP request (HttpContext.java:
 * 55-71, Hint.ofHostUri with port 0); uri_null[i] != 0 = a null uri. */
typedef struct {
    const vo_group *g; int ng; const uint8_t *hblob; const uint32_t *hoff;
    const uint8_t *ublob; const uint32_t *uoff; const uint8_t *unull; const uint16_t *port;
    int32_t *out;
} hint_uri_ctx;

static void hint_uri_range(void *p, int64_t lo, int64_t hi)
{
    hint_uri_ctx *c = (hint_uri_ctx *)p;
    for (int64_t i = lo; i < hi; ++i) {
        const char *s = (const char *)c->hblob + c->hoff[i];
        const int len = (int)(c->hoff[i + 1] - c->hoff[i]);
        const int has_uri = !(c->unull && c->unull[i]);
        const char *u = has_uri ? (const char *)c->ublob + c->uoff[i] : NULL;
        const int ulen = has_uri ? (int)(c->uoff[i + 1] - c->uoff[i]) : 0;
        vo_hint h = vo_hint_of(s, len, c->port ? c->port[i] : 0, u, ulen);
        c->out[i] = vo_search_for_group(c->g, c->ng, &h);
    }
}

void vo_hint_uri_batch(const vo_group *g, int ng, const uint8_t *hblob, const uint32_t *hoff,
                       const uint8_t *ublob, const uint32_t *uoff, const uint8_t *unull,
                       const uint16_t *port, int64_t n, int32_t *out, int nthreads)
{
    hint_uri_ctx c = {g, ng, hblob, hoff, ublob, uoff, unull, port, out};
    parallel_for(n, nthreads, hint_uri_range, &c);
}

/* ------------------------------------------------------------------------ */
/* DNSServer.handleRequest classification -- DNSServer.java:116-166         */
/* ------------------------------------------------------------------------ */

static int hosts_get(const vo_hosts *hs, const char *k, int kn)
{
    if (hs == NULL) return -1;
    for (int i = 0; i < hs->n; ++i)
        if (j_equals(hs->keys[i], hs->key_lens[i], k, kn)) return hs->values[i];
    return -1;
}

int vo_dns_classify(const vo_hosts *hosts, const vo_group *g, int ng,
                    const char *qwire, int qwlen, int32_t *value)
{
    /* Formatter.parseDomainName (Formatter.java:225-257) builds the qname
     * with sb.append((char) b) per wire byte b, a Java byte: the cast
     * sign-extends (JLS 5.1.4), so a byte c >= 0x80 is the char U+FF00 | c.
     * Strings here are the UTF-8 bytes of the Java strings: such a char is
     * three bytes, EF (BE | BF) (80 | c & 3F). */
    char qbuf[1536];
    const char *qname = qwire;
    int qlen = qwlen, ascii = 1;
    for (int i = 0; i < qwlen; ++i)
        if ((unsigned char)qwire[i] >= 0x80) ascii = 0;
    if (!ascii) {
        if (qwlen > 512) {            /* no wire name is this long (the library's limit) */
            *value = 0;
            return VO_DNS_RECURSIVE;
        }
        qlen = 0;
        for (int i = 0; i < qwlen; ++i) {
            unsigned char c = (unsigned char)qwire[i];
            if (c < 0x80) {
                qbuf[qlen++] = (char)c;
            } else {
                qbuf[qlen++] = (char)0xEF;
                qbuf[qlen++] = (char)(0xBC | (c >> 6));
                qbuf[qlen++] = (char)(0x80 | (c & 0x3F));
            }
        }
        qname = qbuf;
    }
    int hv = hosts_get(hosts, qname, qlen);                  /* :127 */
    if (hv >= 0) {
        *value = hv;
        return VO_DNS_HOSTS;
    }
    int dlen = qlen;
    if (dlen > 0 && qname[dlen - 1] == '.') dlen -= 1;        /* :133-135 */
    vo_hint h = vo_hint_of(qname, dlen, 0, NULL, 0);          /* :136 Hint.ofHost */
    int gi = vo_search_for_group(g, ng, &h);
    if (gi >= 0) {
        *value = gi;
        return VO_DNS_GROUP;
    }
    if (vo_is_ip_literal(qname, dlen)) {                      /* :140-149 */
        *value = j_index_of_ch(qname, dlen, ':') != -1 ? 6 : 4;
        return VO_DNS_IP_LITERAL;
    }
    if (j_ends_with(qname, dlen, ".vproxy.local", 13)) {      /* :150-157 */
        *value = 0;
        return VO_DNS_INTERNAL;
    }
    *value = 0;                                               /* :164 */
    return VO_DNS_RECURSIVE;
}

/* ------------------------------------------------------------------------ */
/* Resolver.getHosts -- base/src/main/java/vproxybase/dns/Resolver.java:62-153 */
/* ------------------------------------------------------------------------ */

static int java_ws(char c)  /* Character.isWhitespace over ASCII */
{
    return c == ' ' || c == '\t' || c == '\n' || c == 0x0B || c == '\f' || c == '\r' ||
           (c >= 0x1C && c <= 0x1F);
}

int vo_hosts_parse(const char *text, int len,
                   char *keybuf, int keybuf_cap, int32_t *key_off, int32_t *key_len,
                   int32_t *value, int cap,
                   uint8_t *line_ip, int32_t *line_iplen, int line_cap)
{
    int nkeys = 0, kb = 0, nlines = 0;
    int pos = 0;
    while (pos < len) {
        /* BufferedReader.readLine: \n, \r or \r\n terminate a line */
        int end = pos;
        while (end < len && text[end] != '\n' && text[end] != '\r') ++end;
        int next = end + 1;
        if (end < len && text[end] == '\r' && next < len && text[next] == '\n') ++next;
        const char *line = text + pos;
        int ln = end - pos;
        pos = next;

        int hash = j_index_of_ch(line, ln, '#');                  /* :100-102 */
        if (hash != -1) ln = hash;
        int blank = 1;                                            /* :103-105 */
        for (int i = 0; i < ln; ++i)
            if (!java_ws(line[i])) { blank = 0; break; }
        if (blank) continue;
        while (ln > 0 && (unsigned char)line[0] <= ' ') { ++line; --ln; }      /* trim */
        while (ln > 0 && (unsigned char)line[ln - 1] <= ' ') --ln;
        /* split("[ \t]") then trim + drop empties */
        int toff[512], tlen[512], nt = 0;
        int s = 0;
        for (int i = 0; i <= ln; ++i) {
            if (i == ln || line[i] == ' ' || line[i] == '\t') {
                int a = s, b = i;
                while (a < b && (unsigned char)line[a] <= ' ') ++a;
                while (b > a && (unsigned char)line[b - 1] <= ' ') --b;
                if (b > a && nt < 512) {
                    toff[nt] = a;
                    tlen[nt] = b - a;
                    ++nt;
                }
                s = i + 1;
            }
        }
        if (nt < 2) continue;                                     /* :108-113 */
        uint8_t ip[16];
        int iplen = vo_parse_ip(line + toff[0], tlen[0], ip);     /* :114-120 */
        if (iplen == -1) continue;
        if (nlines >= line_cap) return -1;
        int entry = nlines++;
        memcpy(line_ip + 16 * entry, ip, (size_t)iplen);
        line_iplen[entry] = iplen;
        for (int i = 1; i < nt; ++i) {                            /* :122-141 */
            const char *d1 = line + toff[i];
            int d1n = tlen[i];
            char d2[1024];
            int d2n;
            if (d1n >= 1023) continue;
            if (d1[d1n - 1] == '.') {
                memcpy(d2, d1, (size_t)(d1n - 1));
                d2n = d1n - 1;
            } else {
                memcpy(d2, d1, (size_t)d1n);
                d2[d1n] = '.';
                d2n = d1n + 1;
            }
            int present = 0;
            for (int k = 0; k < nkeys; ++k) {
                if (j_equals(keybuf + key_off[k], key_len[k], d1, d1n) ||
                    j_equals(keybuf + key_off[k], key_len[k], d2, d2n)) {
                    present = 1;
                    break;
                }
            }
            if (present) continue;
            if (nkeys + 2 > cap || kb + d1n + d2n > keybuf_cap) return -1;
            memcpy(keybuf + kb, d1, (size_t)d1n);
            key_off[nkeys] = kb; key_len[nkeys] = d1n; value[nkeys] = entry; ++nkeys; kb += d1n;
            memcpy(keybuf + kb, d2, (size_t)d2n);
            key_off[nkeys] = kb; key_len[nkeys] = d2n; value[nkeys] = entry; ++nkeys; kb += d2n;
        }
    }
    return nkeys;
}

/* ------------------------------------------------------------------------ */
/* ServerGroup source hashing                                               */
/* ------------------------------------------------------------------------ */

/* SOURCE.hash, ServerGroup.java:387-397: Java int arithmetic (wrapping),
 * `aByte` sign-extended. */
int32_t vo_source_hash(const uint8_t *bytes, int len) {
    uint32_t hash = 0;
    for (int i = 0; i < len; ++i) {
        const int32_t b = (int8_t)bytes[i];
        hash = (uint32_t)b + (hash << 6) + (hash << 16) - hash;
    }
    int32_t h = (int32_t)hash;
    if (h == INT32_MIN) return 0;             /* Math.abs(MIN_VALUE) < 0 -> 0 */
    return h < 0 ? -h : h;
}

/* the comparator of sourceReset, ServerGroup.java:629-642 */
static int vo_server_cmp(const vo_server *a, const vo_server *b) {
    if (a->ip_len > b->ip_len) return 1;
    if (b->ip_len > a->ip_len) return -1;
    for (int i = 0; i < a->ip_len; ++i) {
        const int diff = (int8_t)a->ip[i] - (int8_t)b->ip[i];
        if (diff != 0) return diff;
    }
    return a->port - b->port;
}

int vo_source_list(const vo_server *servers, int n, int view, int32_t *order) {
    int k = 0;
    for (int i = 0; i < n; ++i) {
        if (view == 4 && servers[i].ip_len != 4) continue;   /* :622 instanceof IPv4 */
        if (view == 6 && servers[i].ip_len != 16) continue;  /* :623 instanceof IPv6 */
        if (servers[i].weight <= 0) continue;                /* :628 weight > 0 */
        /* stable insertion sort (List.sort is stable) */
        int j = k++;
        while (j > 0 && vo_server_cmp(&servers[order[j - 1]], &servers[i]) > 0) {
            order[j] = order[j - 1];
            --j;
        }
        order[j] = i;
    }
    return k;
}

int vo_source_select(const vo_server *servers, int n, int view, const uint8_t *src, int src_len) {
    int32_t *order = (int32_t *)malloc(sizeof(int32_t) * (size_t)(n > 0 ? n : 1));
    const int size = vo_source_list(servers, n, view, order);
    int32_t hash = vo_source_hash(src, src_len);
    int result = -1;
    for (int recurse = 0; recurse < size; ++recurse) {      /* :480 recurse >= size -> null */
        const int idx = hash % size;                         /* :483 */
        if (servers[order[idx]].healthy) {
            result = order[idx];
            break;
        }
        hash = idx + 1;                                      /* :489 next server in the list */
    }
    free(order);
    return result;
}

/* ------------------------------------------------------------------------ */
/* Packet header extraction (base/src/main/java/vpacket)                    */
/* ------------------------------------------------------------------------ */
/* Result codes of one `from` call: NULL (ok) / an error string / a thrown
 * exception / no return at all. */
enum { VO_OK = 0, VO_ERR = 1, VO_THROW = 2, VO_HANG = 3 };

static int vo_u8(const uint8_t *p, int i) { return p[i]; }
static int vo_u16(const uint8_t *p, int i) { return (p[i] << 8) | p[i + 1]; }

/* TcpPacket.from, TcpPacket.java:164-227, with TcpOption.from/check
 * (:399-434): an option of length 0 or 1 makes TcpOption.from read past its
 * own sub-array, which throws. */
static int vo_tcp(const uint8_t *p, int len, vo_pkt *o) {
    if (len < 20) return VO_ERR;
    o->sport = vo_u16(p, 0);
    o->dport = vo_u16(p, 2);
    const int data_offset = ((vo_u16(p, 12) >> 12) & 0xf) * 4;
    if (data_offset > len) return VO_ERR;
    if (data_offset > 20) {
        int off = 20;
        while (off < data_offset) {
            const int kind = (int8_t)p[off];
            if (kind == 0 || kind == 1) {              /* CASE_1_OPTION_KINDS: END, NOP */
                off += 1;
                if (kind == 0) break;
            } else {
                if (off + 1 >= data_offset) return VO_ERR;
                const int olen = vo_u8(p, off + 1);
                if (off + olen > data_offset) return VO_ERR;
                if (olen < 2) return VO_THROW;         /* get(0) / uint8(1) out of the sub-array */
                if (kind == 3 && olen != 3) return VO_ERR;   /* window scale */
                if (kind == 2 && olen != 4) return VO_ERR;   /* mss */
                off += olen;
            }
        }
    }
    return VO_OK;
}

/* IcmpPacket.from, IcmpPacket.java:22-33 */
static int vo_icmp(int len) { return len < 8 ? VO_ERR : VO_OK; }

/* the transport of an IP packet: ICMP / TCP / PacketBytes */
static int vo_l4(const uint8_t *p, int len, int proto, int v6, vo_pkt *o) {
    if (proto == 1 || (v6 && proto == 58)) {
        o->l4 = proto == 58 ? 58 : 1;
        return vo_icmp(len);
    }
    if (proto == 6) {
        o->l4 = 6;
        return vo_tcp(p, len, o);
    }
    o->l4 = 0;
    return VO_OK;                                       /* PacketBytes.from never fails */
}

/* Ipv4Packet.from, Ipv4Packet.java:28-101 */
static int vo_ipv4(const uint8_t *p, int len, vo_pkt *o) {
    if (len < 20) return VO_ERR;
    const int version = (vo_u8(p, 0) >> 4) & 0xff;
    if (version != 4) return VO_ERR;
    const int ihl = vo_u8(p, 0) & 0x0f;
    if (len < ihl * 4) return VO_ERR;
    if (ihl < 5) return VO_ERR;
    const int total = vo_u16(p, 2);
    if (total < ihl * 4) return VO_ERR;
    if (total != len) return VO_ERR;
    o->proto = vo_u8(p, 9);
    memcpy(o->src, p + 12, 4);
    memcpy(o->dst, p + 16, 4);
    return vo_l4(p + ihl * 4, total - ihl * 4, o->proto, 0, o);
}

static int vo_v6_ext(int nh) {                          /* Consts.IPv6_needs_next_header */
    return nh == 0 || nh == 60 || nh == 43 || nh == 44 || nh == 51 || nh == 50 || nh == 135 ||
           nh == 139 || nh == 140 || nh == 253 || nh == 254;
}

/* Ipv6Packet.from, Ipv6Packet.java:24-106.  The extension-header loop
 * re-parses the first header (xhBuf = xhBuf.sub(0, len), :77): when that
 * header's next header is itself an extension header the loop never ends. */
static int vo_ipv6(const uint8_t *p, int len, vo_pkt *o) {
    if (len < 40) return VO_ERR;
    const int version = (((int8_t)p[0]) >> 4) & 0x0f;
    if (version != 6) return VO_ERR;
    const int payload = vo_u16(p, 4);
    const int next = vo_u8(p, 6);
    if (payload == 0) return VO_ERR;
    if (40 + payload != len) return VO_ERR;
    memcpy(o->src, p + 8, 16);
    memcpy(o->dst, p + 24, 16);
    int skip = 0, proto = next;
    if (vo_v6_ext(next)) {
        const uint8_t *x = p + 40;
        const int xlen = len - 40;
        if (xlen < 8) return VO_ERR;                    /* ExtHeader.from */
        const int hdr_ext_len = vo_u8(x, 1);
        if (xlen < 8 + hdr_ext_len) return VO_ERR;
        const int xnext = vo_u8(x, 0);
        if (vo_v6_ext(xnext)) return VO_HANG;
        skip = 8 + hdr_ext_len;
        proto = xnext;
    }
    o->proto = proto;
    const int rest = len - 40 - skip;
    if (proto == 59 && rest != 0) return VO_ERR;        /* NO_NEXT_HEADER with bytes */
    return vo_l4(p + 40 + skip, rest, proto, 1, o);
}

/* ArpPacket.from, ArpPacket.java:22-64 */
static int vo_arp(const uint8_t *p, int len) {
    if (len < 8) return VO_ERR;
    const int hs = vo_u8(p, 4), ps = vo_u8(p, 5);
    if (len != 8 + 2 * hs + 2 * ps) return VO_ERR;      /* every shorter length errs first */
    return VO_OK;
}

/* EthernetPacket.from, EthernetPacket.java:14-50: an IP parse error is
 * logged and the payload kept as PacketBytes (mayIgnoreError) */
static int vo_ether(const uint8_t *p, int len, vo_pkt *o) {
    if (len < 14) return VO_ERR;
    o->ether_type = vo_u16(p, 12);
    const uint8_t *d = p + 14;
    const int dl = len - 14;
    if (o->ether_type == 0x0806) {
        o->l3 = 1;
        return vo_arp(d, dl);
    }
    if (o->ether_type == 0x0800 || o->ether_type == 0x86dd) {
        vo_pkt ip;
        memset(&ip, 0, sizeof(ip));
        const int v6 = o->ether_type == 0x86dd;
        const int r = v6 ? vo_ipv6(d, dl, &ip) : vo_ipv4(d, dl, &ip);
        if (r == VO_THROW || r == VO_HANG) return r;
        if (r == VO_ERR) {
            o->l3 = 5;
            return VO_OK;
        }
        o->l3 = v6 ? 6 : 4;
        o->l4 = ip.l4;
        o->proto = ip.proto;
        memcpy(o->src, ip.src, 16);
        memcpy(o->dst, ip.dst, 16);
        o->sport = ip.sport;
        o->dport = ip.dport;
        return VO_OK;
    }
    o->l3 = 0;
    return VO_OK;
}

void vo_parse_packet(const uint8_t *p, int len, int layer, vo_pkt *out) {
    memset(out, 0, sizeof(*out));
    int r;
    if (layer == 0) {                                   /* VXLanPacket.from, :16-33 */
        if (len < 8) {
            out->status = 1;
            return;
        }
        out->vni = (uint32_t)((p[4] << 16) | (p[5] << 8) | p[6]);
        r = vo_ether(p + 8, len - 8, out);
        out->status = r == VO_OK ? 0 : r == VO_ERR ? 2 : r == VO_THROW ? 4 : 5;
    } else if (layer == 1) {
        r = vo_ether(p, len, out);
        out->status = r == VO_OK ? 0 : r == VO_ERR ? 2 : r == VO_THROW ? 4 : 5;
    } else {
        vo_pkt ip;
        memset(&ip, 0, sizeof(ip));
        r = layer == 6 ? vo_ipv6(p, len, &ip) : vo_ipv4(p, len, &ip);
        *out = ip;
        out->l3 = layer == 6 ? 6 : 4;
        out->status = r == VO_OK ? 0 : r == VO_ERR ? 3 : r == VO_THROW ? 4 : 5;
    }
    if (out->status != 0) {                             /* no packet object: fields unset */
        const uint32_t vni = out->vni;
        const int et = out->ether_type;
        memset(out->src, 0, 16);
        memset(out->dst, 0, 16);
        out->l3 = out->l4 = out->proto = out->sport = out->dport = 0;
        out->vni = vni;
        out->ether_type = et;
        if (out->status == 1) out->vni = 0;
    }
}

/* ------------------------------------------------------------------------
 * SSLContextHolder.choose / chooseNoDefault / checkSNI / compare
 * (SSLContextHolder.java:51-186), restated as the literal scan: holders in
 * add() order, each holder's names in order, first holder with a match.
 * The quickAccess cache (:68-72, :111, :163) only memoises that scan's
 * result for an SNI; holders are only ever appended, so a memoised answer
 * equals a fresh scan and the cache is omitted.
 * ------------------------------------------------------------------------ */
static int cert_compare(const char *dns, int dl, const uint8_t *sni, int sl) {
    if (dl >= 2 && dns[0] == '*' && dns[1] == '.') {     /* wildcard record, :172-181 */
        const char *suffix = dns + 1;                     /* dnsName.substring(1) */
        int xl = dl - 1;
        if (sl > xl && memcmp(sni + sl - xl, suffix, (size_t)xl) == 0) {
            for (int i = 0; i < sl - xl; ++i)             /* !prefix.contains(".") */
                if (sni[i] == '.') return 0;
            return 1;
        }
        return 0;
    }
    return sl == dl && (dl == 0 || memcmp(sni, dns, (size_t)dl) == 0);  /* equals, :184 */
}

int vo_cert_choose(const char *const *names, const int32_t *name_lens, const int32_t *holder,
                   int n_names, int n_holders, const uint8_t *sni, int sni_len, int sni_null) {
    if (n_holders == 1) return 0;                         /* :53-55 */
    if (n_holders == 0) return -1;                        /* :56-58 */
    if (!sni_null) {                                      /* chooseNoDefault, :67-79 */
        /* the first holder (add() order) with any matching name = the
         * smallest holder index over the matching names */
        int best = n_holders;
        for (int i = 0; i < n_names; ++i)
            if (holder[i] < best && cert_compare(names[i], name_lens[i], sni, sni_len))
                best = holder[i];
        if (best < n_holders) return best;
    }
    return 0;                                             /* the default (first) one, :62 */
}

/* ------------------------------------------------------------------------
 * Traffic-mirror filters: FilterConfig.matchEthernet / matchIp /
 * matchTransport / matchApplication (FilterConfig.java:27-94), the level
 * choice of Mirror.mirror (Mirror.java:104-117) and Mirror.switchPacket
 * (:73-87), each filter tested in list order and the mirrors collected as
 * a set (checkHelper, :133-139).
 * ------------------------------------------------------------------------ */
static int mo_mac_eq(const uint8_t *a, const uint8_t *b) { return memcmp(a, b, 6) == 0; }

static int mo_ether(const vo_mirror_filter *f, const uint8_t *src, const uint8_t *dst) {
    if (f->has_mac_x && f->has_mac_y)
        return (mo_mac_eq(f->mac_x, src) && mo_mac_eq(f->mac_y, dst)) ||
               (mo_mac_eq(f->mac_y, src) && mo_mac_eq(f->mac_x, dst));
    if (f->has_mac_x) return mo_mac_eq(f->mac_x, src) || mo_mac_eq(f->mac_x, dst);
    return 1;
}

static int mo_contains(const vo_net *n, const uint8_t *ip, int len) {   /* Network.contains(IP) */
    return vo_mask_match(ip, len, n->ip, n->ip_len, n->mask, n->mask_len);
}

static int mo_ip(const vo_mirror_filter *f, const uint8_t *ms, const uint8_t *md,
                 const uint8_t *is, int isl, const uint8_t *id, int idl) {
    if (!mo_ether(f, ms, md)) return 0;
    if (f->has_net_x && f->has_net_y)
        return (mo_contains(&f->net_x, is, isl) && mo_contains(&f->net_y, id, idl)) ||
               (mo_contains(&f->net_y, is, isl) && mo_contains(&f->net_x, id, idl));
    if (f->has_net_x) return mo_contains(&f->net_x, is, isl) || mo_contains(&f->net_x, id, idl);
    return 1;
}

static int mo_in(const int32_t r[2], int p) { return r[0] <= p && p <= r[1]; }

static int mo_transport(const vo_mirror_filter *f, const uint8_t *ms, const uint8_t *md,
                        const uint8_t *is, int isl, const uint8_t *id, int idl, int transport,
                        int ps, int pd) {
    if (!mo_ip(f, ms, md, is, isl, id, idl)) return 0;
    if (f->transport != -1 && f->transport != transport) return 0;
    if (f->has_port_x && f->has_port_y)
        return (mo_in(f->port_x, ps) && mo_in(f->port_y, pd)) ||
               (mo_in(f->port_y, ps) && mo_in(f->port_x, pd));
    if (f->has_port_x) return mo_in(f->port_x, ps) || mo_in(f->port_x, pd);
    return 1;
}

uint64_t vo_mirror_match(const vo_mirror_filter *f, int n, int origin,
                         const uint8_t *mac_src, const uint8_t *mac_dst,
                         const uint8_t *ip_src, int src_len, const uint8_t *ip_dst, int dst_len,
                         int transport, int port_src, int port_dst, int app) {
    uint64_t m = 0;
    for (int i = 0; i < n; ++i) {
        const vo_mirror_filter *x = &f[i];
        if (x->origin != origin) continue;
        int hit;
        if (src_len == 0 || dst_len == 0)
            hit = mo_ether(x, mac_src, mac_dst);
        else if (transport == -1)
            hit = mo_ip(x, mac_src, mac_dst, ip_src, src_len, ip_dst, dst_len);
        else if (app == -1)
            hit = mo_transport(x, mac_src, mac_dst, ip_src, src_len, ip_dst, dst_len, transport,
                               port_src, port_dst);
        else
            hit = mo_transport(x, mac_src, mac_dst, ip_src, src_len, ip_dst, dst_len, transport,
                               port_src, port_dst) && (x->app == -1 || x->app == app);
        if (hit) m |= (uint64_t)1 << x->mirror;
    }
    return m;
}

uint64_t vo_mirror_switch(const vo_mirror_filter *f, int n, int origin, const uint8_t *frame,
                          int len, int layer) {
    vo_pkt p;
    vo_parse_packet(frame, len, layer, &p);
    if (p.status != 0) return 0;
    const uint8_t *eth = layer == 0 ? frame + 8 : frame;    /* dst 0-5, src 6-11 */
    uint64_t m = 0;
    int is_ip = p.l3 == 4 || p.l3 == 6;
    int al = p.l3 == 6 ? 16 : 4;
    for (int i = 0; i < n; ++i) {
        const vo_mirror_filter *x = &f[i];
        if (x->origin != origin) continue;
        int hit = is_ip ? mo_ip(x, eth + 6, eth, p.src, al, p.dst, al) : mo_ether(x, eth + 6, eth);
        if (hit) m |= (uint64_t)1 << x->mirror;
    }
    return m;
}

/* ------------------------------------------------------------------------ */
/* Batched forms (pthread partitions) -- checkers and bench cpu_baseline     */
/* ------------------------------------------------------------------------ */
typedef struct {
    const vo_hosts *hosts; const vo_group *g; int ng;
    const uint8_t *blob; const uint32_t *off; uint8_t *kind; int32_t *value;
} dns_batch_ctx;

static void dns_range(void *p, int64_t lo, int64_t hi)
{
    dns_batch_ctx *c = (dns_batch_ctx *)p;
    for (int64_t i = lo; i < hi; ++i) {
        int32_t v = 0;
        const int k = vo_dns_classify(c->hosts, c->g, c->ng, (const char *)c->blob + c->off[i],
                                      (int)(c->off[i + 1] - c->off[i]), &v);
        c->kind[i] = (uint8_t)k;
        c->value[i] = v;
    }
}

void vo_dns_batch(const vo_hosts *hosts, const vo_group *g, int ng, const uint8_t *blob,
                  const uint32_t *off, int64_t n, uint8_t *kind, int32_t *value, int nthreads)
{
    dns_batch_ctx c = {hosts, g, ng, blob, off, kind, value};
    parallel_for(n, nthreads, dns_range, &c);
}

typedef struct { const uint8_t *blob; const uint32_t *off; int layer; vo_pkt *out; } parse_batch_ctx;

static void parse_range(void *p, int64_t lo, int64_t hi)
{
    parse_batch_ctx *c = (parse_batch_ctx *)p;
    for (int64_t i = lo; i < hi; ++i)
        vo_parse_packet(c->blob + c->off[i], (int)(c->off[i + 1] - c->off[i]), c->layer, &c->out[i]);
}

void vo_parse_batch(const uint8_t *blob, const uint32_t *off, int64_t n, int layer, vo_pkt *out,
                    int nthreads)
{
    parse_batch_ctx c = {blob, off, layer, out};
    parallel_for(n, nthreads, parse_range, &c);
}

typedef struct {
    const vo_sg_rule *tcp; int ntcp; const vo_sg_rule *udp; int nudp; int dflt;
    const uint8_t *blob; const uint32_t *off; const uint32_t *remote4; int bind_port;
    const vo_net *v4; int n4; const vo_net *v6; int n6;
    int32_t *acl; uint8_t *allow; int32_t *route;
} switch_batch_ctx;

static void switch_range(void *p, int64_t lo, int64_t hi)
{
    switch_batch_ctx *c = (switch_batch_ctx *)p;
    for (int64_t i = lo; i < hi; ++i) {
        const uint32_t r = c->remote4[i];
        const uint8_t rb[4] = {(uint8_t)(r >> 24), (uint8_t)(r >> 16), (uint8_t)(r >> 8), (uint8_t)r};
        int verdict = 0;
        const int a = vo_sg_allow(c->tcp, c->ntcp, c->udp, c->nudp, c->dflt, 17, rb, 4,
                                  c->bind_port, &verdict);
        if (c->acl) c->acl[i] = a;
        if (c->allow) c->allow[i] = (uint8_t)verdict;
        vo_pkt pk;
        vo_parse_packet(c->blob + c->off[i], (int)(c->off[i + 1] - c->off[i]), 0, &pk);
        int32_t rt = -1;
        if (verdict && pk.status == 0 && (pk.l3 == 4 || pk.l3 == 6))
            rt = pk.l3 == 4 ? vo_rt_lookup_list(c->v4, c->n4, pk.dst, 4)
                            : vo_rt_lookup_list(c->v6, c->n6, pk.dst, 16);
        c->route[i] = rt;
    }
}

void vo_switch_batch(const vo_sg_rule *tcp, int ntcp, const vo_sg_rule *udp, int nudp,
                     int default_allow, const uint8_t *blob, const uint32_t *off, int64_t n,
                     const uint32_t *remote4, int bind_port, const vo_net *v4, int n4,
                     const vo_net *v6, int n6, int32_t *acl, uint8_t *allow, int32_t *route,
                     int nthreads)
{
    switch_batch_ctx c = {tcp, ntcp, udp, nudp, default_allow, blob, off, remote4, bind_port,
                          v4, n4, v6, n6, acl, allow, route};
    parallel_for(n, nthreads, switch_range, &c);
}

typedef struct {
    const char *const *names; const int32_t *lens; const int32_t *holder; int n_names, n_holders;
    const uint8_t *blob; const uint32_t *off; const uint8_t *sni_null; int32_t *out;
} cert_batch_ctx;

static void cert_range(void *p, int64_t lo, int64_t hi)
{
    cert_batch_ctx *c = (cert_batch_ctx *)p;
    for (int64_t i = lo; i < hi; ++i)
        c->out[i] = vo_cert_choose(c->names, c->lens, c->holder, c->n_names, c->n_holders,
                                   c->blob + c->off[i], (int)(c->off[i + 1] - c->off[i]),
                                   c->sni_null ? c->sni_null[i] : 0);
}

void vo_cert_batch(const char *const *names, const int32_t *name_lens, const int32_t *holder,
                   int n_names, int n_holders, const uint8_t *blob, const uint32_t *off,
                   const uint8_t *sni_null, int64_t n, int32_t *out, int nthreads)
{
    cert_batch_ctx c = {names, name_lens, holder, n_names, n_holders, blob, off, sni_null, out};
    parallel_for(n, nthreads, cert_range, &c);
}

typedef struct {
    const vo_mirror_filter *f; int nf, origin, layer;
    const uint8_t *blob; const uint32_t *off; uint64_t *out;
} mirror_batch_ctx;

static void mirror_range(void *p, int64_t lo, int64_t hi)
{
    mirror_batch_ctx *c = (mirror_batch_ctx *)p;
    for (int64_t i = lo; i < hi; ++i)
        c->out[i] = vo_mirror_switch(c->f, c->nf, c->origin, c->blob + c->off[i],
                                     (int)(c->off[i + 1] - c->off[i]), c->layer);
}

void vo_mirror_switch_batch(const vo_mirror_filter *f, int nf, int origin, const uint8_t *blob,
                            const uint32_t *off, int64_t n, int layer, uint64_t *out, int nthreads)
{
    mirror_batch_ctx c = {f, nf, origin, layer, blob, off, out};
    parallel_for(n, nthreads, mirror_range, &c);
}

typedef struct {
    const vo_mirror_filter *f; int nf, origin;
    const uint8_t *mac_src, *mac_dst, *src_len, *dst_len, *ip_src, *ip_dst;
    const int32_t *transport, *port_src, *port_dst, *app;
    uint64_t *out;
} mirror_items_ctx;

static void mirror_items_range(void *p, int64_t lo, int64_t hi)
{
    mirror_items_ctx *c = (mirror_items_ctx *)p;
    for (int64_t i = lo; i < hi; ++i) {
        const int ls = c->src_len[i], ld = c->dst_len[i];
        c->out[i] = vo_mirror_match(c->f, c->nf, c->origin, c->mac_src + 6 * i, c->mac_dst + 6 * i,
                                    c->ip_src + 16 * i, ls == 4 || ls == 16 ? ls : 0,
                                    c->ip_dst + 16 * i, ld == 4 || ld == 16 ? ld : 0,
                                    c->transport[i], c->port_src[i], c->port_dst[i], c->app[i]);
    }
}

/* vo_mirror_match over SoA columns laid out as vc_mirror_items (MACs 6 B,
 * IP rows 16 B, lengths 0 / 4 / 16), every column present */
void vo_mirror_match_batch(const vo_mirror_filter *f, int nf, int origin, const uint8_t *mac_src,
                           const uint8_t *mac_dst, const uint8_t *src_len, const uint8_t *dst_len,
                           const uint8_t *ip_src, const uint8_t *ip_dst, const int32_t *transport,
                           const int32_t *port_src, const int32_t *port_dst, const int32_t *app,
                           int64_t n, uint64_t *out, int nthreads)
{
    mirror_items_ctx c = {f, nf, origin, mac_src, mac_dst, src_len, dst_len, ip_src, ip_dst,
                          transport, port_src, port_dst, app, out};
    parallel_for(n, nthreads, mirror_items_range, &c);
}

typedef struct {
    const vo_server *servers; const int32_t *goff; const int32_t *order; const int32_t *size;
    const int32_t *grp; const uint32_t *src4; int32_t *out;
} source_batch_ctx;

static void source_range(void *p, int64_t lo, int64_t hi)
{
    source_batch_ctx *c = (source_batch_ctx *)p;
    for (int64_t i = lo; i < hi; ++i) {
        const int g = c->grp[i];
        const int32_t *ord = c->order + c->goff[g];
        const int size = c->size[g];
        const uint32_t s = c->src4[i];
        const uint8_t sb[4] = {(uint8_t)(s >> 24), (uint8_t)(s >> 16), (uint8_t)(s >> 8), (uint8_t)s};
        int32_t hash = vo_source_hash(sb, 4);
        int result = -1;
        for (int recurse = 0; recurse < size; ++recurse) {      /* ServerGroup.java:480-489 */
            const int idx = hash % size;
            if (c->servers[c->goff[g] + ord[idx]].healthy) {
                result = ord[idx];
                break;
            }
            hash = idx + 1;
        }
        c->out[i] = result;
    }
}

void vo_source_batch(const vo_server *servers, const int32_t *goff, int n_groups, int view,
                     const int32_t *grp, const uint32_t *src4, int64_t n, int32_t *out,
                     int nthreads)
{
    const int total = n_groups > 0 ? goff[n_groups] : 0;
    int32_t *order = (int32_t *)malloc(sizeof(int32_t) * (size_t)(total > 0 ? total : 1));
    int32_t *size = (int32_t *)malloc(sizeof(int32_t) * (size_t)(n_groups > 0 ? n_groups : 1));
    for (int g = 0; g < n_groups; ++g)
        size[g] = vo_source_list(servers + goff[g], goff[g + 1] - goff[g], view, order + goff[g]);
    source_batch_ctx c = {servers, goff, order, size, grp, src4, out};
    parallel_for(n, nthreads, source_range, &c);
    free(order);
    free(size);
}

/* ------------------------------------------------------------------------ */
/* DNSServer's drain loop per datagram -- core/src/main/java/vproxy/dns/     */
/* DNSServer.java:457-500: securityGroup.allow(UDP, remote, remote port),    */
/* `read == 0`, Formatter.parsePackets (base/.../dns/Formatter.java:162-372) */
/* with the rdata parsers (dns/rdata/A.java:51-56, AAAA.java:45-50,          */
/* CNAME.java:51-58, PTR.java:22-29, TXT.java:54-73, SRV.java:27-36), then   */
/* isResponse / opcode / handleRequest (DNSServer.java:116-166).  Restated   */
/* the Java way: a recursive parseDomainName over ByteArray views whose      */
/* get(i) throws past the view's end.  The library's contract (VO_DNSD_HOST) */
/* is applied on top: more than one packet, more than VO_DNSD_MAXQ          */
/* questions, a qname of more than VO_DNSD_NAMECAP chars, a pointer chain   */
/* deeper than VO_DNSD_MAXPTR (Java would recurse on; a loop overflows).    */
/* ------------------------------------------------------------------------ */
#define DN_BAD (-1)    /* IndexOutOfBoundsException / InvalidDNSPacketException */
#define DN_DEEP (-2)   /* deeper than VO_DNSD_MAXPTR pointers */

typedef struct {
    const uint8_t *raw; int rawlen;      /* rawPacket: the whole datagram */
    char *sb; int sbn, sbcap;            /* the StringBuilder (chars = wire bytes) */
} dn_ctx;

/* ByteArray view [vs, vs + vlen) of the datagram: get(i) */
static int dn_get(const dn_ctx *c, int vs, int vlen, int i, int *b)
{
    if (i >= vlen) return DN_BAD;         /* AbstractByteArray.checkBoundForOffset */
    *b = c->raw[vs + i];
    return 0;
}

static void dn_append(dn_ctx *c, int ch)
{
    if (c->sb && c->sbn < c->sbcap) c->sb[c->sbn] = (char)ch;
    c->sbn++;
}

/* Formatter.parseDomainName(data, rawPacket, offsetHolder), data = view */
static int dn_name(dn_ctx *c, int vs, int vlen, int *holder, int depth)
{
    int len = 0, i = 0, b;
    for (;; ++i) {
        if (dn_get(c, vs, vlen, i, &b)) return DN_BAD;
        if (len == 0) {
            if (b == 0) {
                break;
            } else if ((b & 0xC0) == 0xC0) {             /* is pointer */
                int off = (b & 0x3F) << 8, b2;
                if (dn_get(c, vs, vlen, ++i, &b2)) return DN_BAD;
                off |= b2;
                if (depth + 1 > VO_DNSD_MAXPTR) return DN_DEEP;
                /* rawPacket.sub(offset, rawPacket.length() - offset) */
                int rc = dn_name(c, off, c->rawlen - off, holder, depth + 1);
                if (rc) return rc;
                break;                                   /* pointer ends the name */
            } else {
                len = b;
            }
        } else {
            dn_append(c, b);
            --len;
            if (len == 0) dn_append(c, '.');
        }
    }
    *holder = i + 1;
    return 0;
}

static int dn_u16(const dn_ctx *c, int vs, int vlen, int i, int *v)
{
    int a, b;
    if (dn_get(c, vs, vlen, i, &a) || dn_get(c, vs, vlen, i + 1, &b)) return DN_BAD;
    *v = (a << 8) | b;
    return 0;
}

/* DNSClass lookup (Formatter.parseClass) */
static int dn_class(int clazz, int question)
{
    if (clazz == 1 || clazz == 3 || clazz == 4) return 0;
    if (clazz == 254 || clazz == 255) return question ? 0 : DN_BAD;
    return DN_BAD;                                       /* unknown class */
}

/* Formatter.parseQuestion over the view [vs, vs + vlen) */
static int dn_question(dn_ctx *c, int vs, int vlen, int *used, int *qtype)
{
    int holder = 0, qclass, rc = dn_name(c, vs, vlen, &holder, 0);
    if (rc) return rc;
    if (dn_u16(c, vs, vlen, holder, qtype) || dn_u16(c, vs, vlen, holder + 2, &qclass))
        return DN_BAD;
    /* parseType(qtype, true) never throws (unknown -> OTHER) */
    if (dn_class(qclass, 1)) return DN_BAD;
    *used = holder + 4;
    return 0;
}

/* Formatter.parseResource over the view [vs, vs + vlen) */
static int dn_resource(dn_ctx *c, int vs, int vlen, int *used)
{
    int holder = 0, type, clazz, rdlen, x, rc = dn_name(c, vs, vlen, &holder, 0);
    if (rc) return rc;
    int off = holder;
    if (dn_u16(c, vs, vlen, off, &type) || dn_u16(c, vs, vlen, off + 2, &clazz) ||
        dn_u16(c, vs, vlen, off + 4, &x) || dn_u16(c, vs, vlen, off + 6, &x) ||
        dn_u16(c, vs, vlen, off + 8, &rdlen))
        return DN_BAD;
    if (type >= 252 && type <= 255) return DN_BAD;       /* question-only DNSType */
    if (type != 41 && dn_class(clazz, 0)) return DN_BAD; /* OPT: NOT_CLASS */
    off += 10;
    if (vlen - off < rdlen) return DN_BAD;               /* data.sub(offset, rdlen) */
    const int rs = vs + off;                             /* rdataBytes view [rs, rs + rdlen) */
    if (type == 1) {                                     /* A */
        if (rdlen != 4) return DN_BAD;
    } else if (type == 28) {                             /* AAAA */
        if (rdlen != 16) return DN_BAD;
    } else if (type == 5 || type == 12) {                /* CNAME, PTR */
        int h = 0;
        rc = dn_name(c, rs, rdlen, &h, 0);
        if (rc) return rc;
        if (h != rdlen) return DN_BAD;
    } else if (type == 16) {                             /* TXT */
        int o = 0;
        while (o < rdlen) {
            int l = c->raw[rs + o];
            ++o;
            if (rdlen - o < l) return DN_BAD;
            o += l;
        }
    } else if (type == 33) {                             /* SRV */
        /* priority/weight/port read from rawPacket (offsets 0..5), then the
         * target from data.sub(6, len - 6); its offsetHolder is compared with
         * data.length(), which it can never equal */
        int h = 0;
        rc = dn_name(c, rs + 6, rdlen - 6, &h, 0);
        if (rc) return rc;
        if (h != rdlen) return DN_BAD;
    }
    *used = off + rdlen;
    return 0;
}

void vo_dns_datagram(const vo_sg_rule *tcp, int ntcp, const vo_sg_rule *udp, int nudp,
                     int default_allow, const vo_hosts *hosts, const vo_group *g, int ng,
                     const uint8_t *p, int n, const uint8_t *ip, int iplen, int port,
                     vo_dnsd_out *out)
{
    memset(out, 0, sizeof *out);
    int verdict = 0;
    out->acl = vo_sg_allow(tcp, ntcp, udp, nudp, default_allow, 17, ip, iplen, port, &verdict);
    if (!verdict) {                                      /* DNSServer.java:469-472 */
        out->status = VO_DNSD_REJECTED;
        return;
    }
    if (n == 0) {                                        /* :473-476 */
        out->status = VO_DNSD_EMPTY;
        return;
    }
    dn_ctx c = {p, n, NULL, 0, 0};
    /* Formatter.parsePackets, first packet (totalOffset 0: data == input) */
    int qtype[VO_DNSD_MAXQ + 1], qat[VO_DNSD_MAXQ + 1];
    int st = 0, b2 = 0, b3 = 0, opcode = 0, qd = 0, nres = 0, at = 12, x;
    if (dn_get(&c, 0, n, 0, &x) || dn_get(&c, 0, n, 1, &x) || dn_get(&c, 0, n, 2, &b2)) {
        st = DN_BAD;
    } else {
        opcode = (b2 >> 3) & 0x0F;                       /* parseOpcode */
        if (!(opcode == 0 || opcode == 1 || opcode == 2 || opcode == 4 || opcode == 5 ||
              opcode == 6))
            st = DN_BAD;
        else if (dn_get(&c, 0, n, 3, &b3) || (b3 & 0x0F) > 11)     /* parseRCode */
            st = DN_BAD;
        else {
            int an, ns, ar;
            if (dn_u16(&c, 0, n, 4, &qd) || dn_u16(&c, 0, n, 6, &an) ||
                dn_u16(&c, 0, n, 8, &ns) || dn_u16(&c, 0, n, 10, &ar))
                st = DN_BAD;
            nres = an + ns + ar;
        }
    }
    for (int q = 0; q < qd && !st; ++q) {
        int used = 0, t = 0;
        st = dn_question(&c, at, n - at, &used, &t);
        if (!st && q <= VO_DNSD_MAXQ) {
            qtype[q] = t;
            qat[q] = at;
        }
        at += used;
    }
    for (int k = 0; k < nres && !st; ++k) {
        int used = 0;
        st = dn_resource(&c, at, n - at, &used);
        at += used;
    }
    if (st) {
        out->status = st == DN_BAD ? VO_DNSD_MALFORMED : VO_DNSD_HOST;
        return;
    }
    if (at < n) {                                        /* another packet follows */
        out->status = VO_DNSD_HOST;
        return;
    }
    if (b2 & 0x80) {                                     /* p.isResponse: :490-493 */
        out->status = VO_DNSD_RESPONSE;
        return;
    }
    if (opcode != 0) {                                   /* runRecursive: :494-497 */
        out->status = VO_DNSD_RECURSIVE;
        return;
    }
    if (qd > VO_DNSD_MAXQ) {
        out->status = VO_DNSD_HOST;
        return;
    }
    out->status = VO_DNSD_ANSWER;
    for (int q = 0; q < qd; ++q) {                       /* handleRequest */
        char name[VO_DNSD_NAMECAP];
        dn_ctx d = {p, n, name, 0, VO_DNSD_NAMECAP};
        int holder = 0;
        dn_name(&d, qat[q], n - qat[q], &holder, 0);
        out->nq = q + 1;
        out->qtype[q] = qtype[q];
        if (qtype[q] != 1 && qtype[q] != 28 && qtype[q] != 33) {   /* not A / AAAA / SRV */
            out->kind[q] = VO_DNS_RECURSIVE;
            out->status = VO_DNSD_RECURSIVE;
            return;
        }
        if (d.sbn > VO_DNSD_NAMECAP) {                   /* the Java path decides */
            out->status = VO_DNSD_HOST;
            out->nq = 0;
            return;
        }
        int32_t v = 0;
        out->kind[q] = vo_dns_classify(hosts, g, ng, name, d.sbn, &v);
        out->value[q] = v;
        if (out->kind[q] == VO_DNS_RECURSIVE) {
            out->status = VO_DNSD_RECURSIVE;
            return;
        }
    }
}

typedef struct {
    const vo_sg_rule *tcp; int ntcp; const vo_sg_rule *udp; int nudp; int dflt;
    const vo_hosts *hosts; const vo_group *g; int ng;
    const uint8_t *blob; const uint32_t *off; const uint8_t *fam; const uint32_t *r4;
    const uint8_t *r6; const uint16_t *rport; vo_dnsd_out *out;
} dnsd_batch_ctx;

static void dnsd_range(void *p, int64_t lo, int64_t hi)
{
    dnsd_batch_ctx *c = (dnsd_batch_ctx *)p;
    for (int64_t i = lo; i < hi; ++i) {
        uint8_t ip[16];
        int iplen = 4;
        if (c->fam && c->fam[i] == 6) {
            memcpy(ip, c->r6 + 16 * i, 16);
            iplen = 16;
        } else {
            const uint32_t r = c->r4[i];
            ip[0] = (uint8_t)(r >> 24); ip[1] = (uint8_t)(r >> 16);
            ip[2] = (uint8_t)(r >> 8); ip[3] = (uint8_t)r;
        }
        vo_dns_datagram(c->tcp, c->ntcp, c->udp, c->nudp, c->dflt, c->hosts, c->g, c->ng,
                        c->blob + c->off[i], (int)(c->off[i + 1] - c->off[i]), ip, iplen,
                        c->rport[i], &c->out[i]);
    }
}

void vo_dnsd_batch(const vo_sg_rule *tcp, int ntcp, const vo_sg_rule *udp, int nudp,
                   int default_allow, const vo_hosts *hosts, const vo_group *g, int ng,
                   const uint8_t *blob, const uint32_t *off, int64_t n, const uint8_t *family,
                   const uint32_t *remote4, const uint8_t *remote6, const uint16_t *remote_port,
                   vo_dnsd_out *out, int nthreads)
{
    dnsd_batch_ctx c = {tcp, ntcp, udp, nudp, default_allow, hosts, g, ng, blob, off, family,
                        remote4, remote6, remote_port, out};
    parallel_for(n, nthreads, dnsd_range, &c);
}

/* ------------------------------------------------------------------------ */
/* HTTP/1 request head -> connection hint -> group                          */
/* HttpSubContext.java:394-534, HttpContext.java:55-71                      */
/* ------------------------------------------------------------------------ */

/* The parser builds its strings with sb.append((char) b) of Java bytes: a
 * byte c >= 0x80 is the char U+FF00 | c (as in Formatter.parseDomainName);
 * here as its UTF-8 bytes EF (BC | c >> 6) (80 | c & 3F). */
static int jchars_utf8(const unsigned char *s, int n, char *out)
{
    int k = 0;
    for (int i = 0; i < n; ++i) {
        unsigned char c = s[i];
        if (c < 0x80) {
            out[k++] = (char)c;
        } else {
            out[k++] = (char)0xEF;
            out[k++] = (char)(0xBC | (c >> 6));
            out[k++] = (char)(0x80 | (c & 0x3F));
        }
    }
    return k;
}

/* String.trim(): chars <= ' ' off both ends (every char of a byte >= 0x80 is
 * above ' ') */
static void j_trim(const unsigned char *s, int n, int *from, int *to)
{
    int a = 0, e = n;
    while (a < e && s[a] <= ' ') ++a;
    while (e > a && s[e - 1] <= ' ') --e;
    *from = a;
    *to = e;
}

int vo_http_extract(const uint8_t *p, int n, uint8_t *uri, int *uri_len, uint8_t *host,
                    int *host_len)
{
    unsigned char *key = malloc((size_t)n + 1), *val = malloc((size_t)n + 1);
    int ul = 0, kl = 0, vl = 0, hl = 0;
    int uri_set = 0, host_set = 0;     /* theUri / theHostHeader != null */
    int header = 0;                    /* the HeaderBuilder exists */
    int state = 0;
    for (int i = 0; i < n && state != 9; ++i) {
        const unsigned char b = p[i];
    again:
        switch (state) {
        case 0:                                        /* :394-404 (frontend) */
            state = 1;
            goto again;
        case 1:                                        /* method :406-412 */
            if (b == ' ') state = 2;
            break;
        case 2:                                        /* uri :414-426 */
            if (b == ' ') {
                uri_set = 1;
                state = 3;
            } else if (b == '\r') {
            } else if (b == '\n') {
                uri_set = 1;
                state = 4;
            } else {
                uri[ul++] = b;
            }
            break;
        case 3:                                        /* version :428-439 */
            if (b == '\n') state = 4;
            break;
        case 4:                                        /* end-first-line :441-451 */
            if (b == '\r') {
            } else if (b == '\n') {
                state = 9;
            } else {
                state = 5;
                goto again;
            }
            break;
        case 5:                                        /* header-key :453-464 */
            if (!header) {
                header = 1;
                kl = vl = 0;
            }
            if (b == ':') state = 7;                   /* state6(':') -> 7, :466-472 */
            else key[kl++] = b;
            break;
        case 7:                                        /* header-value :474-484 */
            if (b == '\r') {
            } else if (b == '\n') {
                state = 8;
            } else if (b != ' ' || vl != 0) {
                val[vl++] = b;
            }
            break;
        case 8:                                        /* end-one-header :486-534 */
            if (header) {
                int a, e;
                j_trim(key, kl, &a, &e);               /* key.trim().toLowerCase() */
                if (e - a == 4 && (key[a] | 0x20) == 'h' && (key[a + 1] | 0x20) == 'o' &&
                    (key[a + 2] | 0x20) == 's' && (key[a + 3] | 0x20) == 't') {
                    int va, ve;
                    j_trim(val, vl, &va, &ve);         /* theHostHeader = value.trim() */
                    hl = ve - va;
                    memcpy(host, val + va, (size_t)hl);
                    host_set = 1;
                }
                header = 0;
            }
            if (b == '\r') {
            } else if (b == '\n') {
                state = 9;
            } else {
                state = 5;
                goto again;
            }
            break;
        }
    }
    free(key);
    free(val);
    *uri_len = ul;
    *host_len = hl;
    return (host_set ? VO_HTTP_HOST : 0) | (uri_set ? VO_HTTP_URI : 0);
}

int vo_http_hint(const vo_group *g, int ng, const uint8_t *p, int n, int *kind)
{
    unsigned char *uri = malloc((size_t)n + 1), *host = malloc((size_t)n + 1);
    int ul = 0, hl = 0;
    /* HttpContext.connectionHint, :55-71 */
    const int k = vo_http_extract(p, n, uri, &ul, host, &hl);
    const int host_set = (k & VO_HTTP_HOST) != 0, uri_set = (k & VO_HTTP_URI) != 0;
    int out = -1;
    if (k) {
        char *hu = malloc((size_t)hl * 3 + 1), *uu = malloc((size_t)ul * 3 + 1);
        const int hn = host_set ? jchars_utf8(host, hl, hu) : 0;
        const int un = uri_set ? jchars_utf8(uri, ul, uu) : 0;
        vo_hint h = vo_hint_of(host_set ? hu : NULL, hn, 0, uri_set ? uu : NULL, un);
        out = vo_search_for_group(g, ng, &h);
        free(hu);
        free(uu);
    }
    free(uri);
    free(host);
    *kind = k;
    return out;
}

typedef struct {
    const vo_group *g; int ng; const uint8_t *blob; const uint32_t *off;
    uint8_t *kind; int32_t *group;
} http_batch_ctx;

static void http_range(void *p, int64_t lo, int64_t hi)
{
    http_batch_ctx *c = (http_batch_ctx *)p;
    for (int64_t i = lo; i < hi; ++i) {
        int k = 0;
        c->group[i] = vo_http_hint(c->g, c->ng, c->blob + c->off[i],
                                   (int)(c->off[i + 1] - c->off[i]), &k);
        if (c->kind) c->kind[i] = (uint8_t)k;
    }
}

void vo_http_batch(const vo_group *g, int ng, const uint8_t *blob, const uint32_t *off, int64_t n,
                   uint8_t *kind, int32_t *group, int nthreads)
{
    http_batch_ctx c = {g, ng, blob, off, kind, group};
    parallel_for(n, nthreads, http_range, &c);
}

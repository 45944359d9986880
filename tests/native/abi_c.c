/*
 * abi_c.c -- a plain C99 consumer of include/vclassify.h (test only).
 *
 * Runs the call sequence the JNI shim (jni/vproxy_component_secure_GpuClassifier.c)
 * makes for a vswitch / security-group caller, against libvclassify.so:
 *   create -> SecurityGroup and RouteTable control-plane mirrors -> compile
 *   -> register the "direct buffers" once -> vc_acl_classify_v4 ->
 *   vc_route_lookup_v4 -> vc_pipeline over IPv4 + IPv6 packets ->
 *   vc_counters_prometheus with its size-query protocol -> destroy.
 * Built with gcc -std=c99 -Wall -Wextra -Werror -pedantic, so header or ABI
 * drift that ctypes would not notice breaks the build.
 *
 * Usage: abi_c OUT.bin   Writes the rules, inputs and outputs for
 * tests/test_gpu_abi_c.py to compare with the ctypes path and the oracle.
 * Exit status: 0 ok, 1 a call failed or two paths disagreed, 3 no usable
 * GPU (vc_create returned VC_EDEVICE: the CPU test tier expects this).
 */
#define _POSIX_C_SOURCE 200112L
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "vclassify.h"

#define N_ITEMS 65539

static uint64_t g_rng = 0x5EEDu;

static uint32_t rnd(void) {
    g_rng ^= g_rng << 13;
    g_rng ^= g_rng >> 7;
    g_rng ^= g_rng << 17;
    return (uint32_t) (g_rng >> 11);
}

static int check(int rc, const char *what) {
    if (rc < 0) {
        fprintf(stderr, "%s failed: %d %s\n", what, rc, vc_last_error());
        exit(1);
    }
    return rc;
}

static void *buf(size_t bytes) {           /* 16-byte aligned, like a direct ByteBuffer */
    void *p = NULL;
    if (posix_memalign(&p, 64, bytes ? bytes : 16) != 0) {
        fprintf(stderr, "out of memory\n");
        exit(1);
    }
    memset(p, 0, bytes ? bytes : 16);
    return p;
}

static void put(FILE *f, const void *p, size_t bytes) {
    if (bytes && fwrite(p, 1, bytes, f) != bytes) {
        fprintf(stderr, "write failed\n");
        exit(1);
    }
}

static void net_or_die(const char *s, vc_net *out) {
    check(vc_net_parse(s, out), s);
}

int main(int argc, char **argv) {
    const char *tcp_specs[] = {"10.0.0.0/8", "192.168.0.0/16", "::ffff:0:0/96", "0.0.0.0/0",
                               "2001:db8::/32"};
    const int tcp_ports[][3] = {{80, 80, 0}, {0, 65535, 1}, {0, 1000, 1}, {1024, 2048, 1},
                                {0, 65535, 0}};
    const char *udp_specs[] = {"0.0.0.0/0", "8.8.0.0/16", "::/0"};
    const int udp_ports[][3] = {{53, 53, 1}, {0, 65535, 0}, {0, 0, 0}};
    vc_ctx *ctx = NULL;
    vc_secgroup *sg = NULL;
    vc_routetable *rt = NULL;
    vc_net v4net, v6net, net;
    char alias[64];
    int i, rc, n_tcp, n_udp, n4, n6;
    const int64_t n = N_ITEMS;
    FILE *f;

    if (argc != 2) {
        fprintf(stderr, "usage: abi_c OUT.bin\n");
        return 2;
    }
    printf("%s\n", vc_version());
    rc = vc_create(0, &ctx);
    if (rc == VC_EDEVICE) {
        printf("VC_EDEVICE: %s\n", vc_last_error());
        return 3;
    }
    check(rc, "vc_create");

    /* SecurityGroup: new SecurityGroup("secg", false) + addRule in list order */
    check(vc_secgroup_new("secg", 0, &sg), "vc_secgroup_new");
    for (i = 0; i < 5; ++i) {
        net_or_die(tcp_specs[i], &net);
        sprintf(alias, "tcp%d", i);
        check(vc_secgroup_add_rule(sg, alias, &net, VC_PROTO_TCP, tcp_ports[i][0], tcp_ports[i][1],
                                   tcp_ports[i][2]), "add tcp rule");
    }
    for (i = 0; i < 200; ++i) {
        uint8_t ip[16];
        uint32_t a = rnd();
        int m = 16 + (int) (rnd() % 13);
        a &= m ? 0xFFFFFFFFu << (32 - m) : 0;
        ip[0] = (uint8_t) (a >> 24); ip[1] = (uint8_t) (a >> 16);
        ip[2] = (uint8_t) (a >> 8); ip[3] = (uint8_t) a;
        check(vc_net_from_prefix(ip, 4, m, &net), "vc_net_from_prefix");
        sprintf(alias, "r%d", i);
        {
            const int lo = (int) (rnd() % 65536), w = (int) (rnd() % 4096);
            const int hi = lo + w > 65535 ? 65535 : lo + w;
            check(vc_secgroup_add_rule(sg, alias, &net, (rnd() & 1) ? VC_PROTO_TCP : VC_PROTO_UDP,
                                       lo, hi, (int) (rnd() & 1)), "add rule");
        }
    }
    for (i = 0; i < 3; ++i) {
        net_or_die(udp_specs[i], &net);
        sprintf(alias, "udp%d", i);
        check(vc_secgroup_add_rule(sg, alias, &net, VC_PROTO_UDP, udp_ports[i][0], udp_ports[i][1],
                                   udp_ports[i][2]), "add udp rule");
    }
    /* the reference's error behaviour through the ABI */
    net_or_die("10.0.0.0/8", &net);
    if (vc_secgroup_add_rule(sg, "tcp0", &net, VC_PROTO_TCP, 1, 2, 1) != VC_EEXIST ||
        vc_secgroup_remove_rule(sg, "nope") != VC_ENOTFOUND ||
        vc_net_parse("10.0.0.1/8", &net) != VC_EINVAL) {
        fprintf(stderr, "error codes differ from the reference's exceptions\n");
        return 1;
    }
    check(vc_secgroup_compile(ctx, sg), "vc_secgroup_compile");

    /* RouteTable(Table 10.0.0.0/8 + fd00::/8, vni 7) + addRule in random order */
    net_or_die("10.0.0.0/8", &v4net);
    net_or_die("fd00::/8", &v6net);
    check(vc_routetable_new(&v4net, &v6net, 7, &rt), "vc_routetable_new");
    for (i = 0; i < 300; ++i) {
        uint8_t ip[16];
        uint32_t a = rnd();
        int m = 8 + (int) (rnd() % 23);
        a &= 0xFFFFFFFFu << (32 - m);
        ip[0] = (uint8_t) (a >> 24); ip[1] = (uint8_t) (a >> 16);
        ip[2] = (uint8_t) (a >> 8); ip[3] = (uint8_t) a;
        check(vc_net_from_prefix(ip, 4, m, &net), "vc_net_from_prefix");
        sprintf(alias, "v4r%d", i);
        rc = vc_routetable_add_rule(rt, alias, &net, i, NULL, 0);
        if (rc != VC_OK && rc != VC_EXEXC && rc != VC_EEXIST) check(rc, "add route");
    }
    for (i = 0; i < 100; ++i) {
        uint8_t ip[16];
        int k, m = 16 + (int) (rnd() % 49);
        memset(ip, 0, sizeof ip);
        ip[0] = 0xfd;
        for (k = 1; k < 8; ++k) ip[k] = (uint8_t) rnd();
        for (k = m; k < 128; ++k) ip[k >> 3] &= (uint8_t) ~(0x80u >> (k & 7));
        if (vc_net_from_prefix(ip, 16, m, &net) != VC_OK) continue;
        sprintf(alias, "v6r%d", i);
        rc = vc_routetable_add_rule(rt, alias, &net, 0, ip, 16);
        if (rc != VC_OK && rc != VC_EXEXC && rc != VC_EEXIST) check(rc, "add v6 route");
    }
    check(vc_routetable_compile(ctx, rt), "vc_routetable_compile");
    check(vc_counters_enable(ctx, 1), "vc_counters_enable");

    {
        uint8_t *proto = buf((size_t) n), *family = buf((size_t) n), *allow = buf((size_t) n);
        uint32_t *src4 = buf((size_t) n * 4), *dst4 = buf((size_t) n * 4);
        uint16_t *port = buf((size_t) n * 2);
        uint8_t *src6 = buf((size_t) n * 16), *dst6 = buf((size_t) n * 16);
        int32_t *idx = buf((size_t) n * 4), *route = buf((size_t) n * 4);
        int32_t *idx2 = buf((size_t) n * 4), *route2 = buf((size_t) n * 4);
        int32_t *p_acl = buf((size_t) n * 4), *p_route = buf((size_t) n * 4);
        int32_t *p_group = buf((size_t) n * 4);
        uint8_t *p_allow = buf((size_t) n);
        void *reg[] = {proto, src4, port, dst4, idx, allow, route};
        const int64_t reg_len[] = {n, n * 4, n * 2, n * 4, n * 4, n, n * 4};
        vc_acl_rule *tcp, *udp;
        vc_net *v4l, *v6l;
        uint64_t *acl_cnt;
        int64_t n_cnt = 0, len = 0;
        char *text;
        int64_t k;

        for (k = 0; k < n; ++k) {
            const uint32_t r = rnd();
            proto[k] = (r & 1) ? VC_PROTO_TCP : VC_PROTO_UDP;
            src4[k] = (r & 2) ? (0xC0A80000u | (rnd() & 0xFFFF)) : rnd();
            dst4[k] = (r & 4) ? (0x0A000000u | (rnd() & 0xFFFFFF)) : rnd();
            port[k] = (uint16_t) ((r & 8) ? 53 + (rnd() % 2048) : rnd());
            family[k] = (r & 16) ? 6 : 4;
            src6[16 * k] = 0x20; src6[16 * k + 1] = 0x01; src6[16 * k + 2] = 0x0d;
            src6[16 * k + 3] = 0xb8;
            if (r & 32) {                       /* ::ffff:a.b.c.d */
                memset(src6 + 16 * k, 0, 10);
                src6[16 * k + 10] = 0xff; src6[16 * k + 11] = 0xff;
                memcpy(src6 + 16 * k + 12, &src4[k], 4);
            }
            dst6[16 * k] = 0xfd;
            dst6[16 * k + 1] = (uint8_t) rnd();
            dst6[16 * k + 2] = (uint8_t) rnd();
            dst6[16 * k + 15] = (uint8_t) rnd();
        }
        /* direct buffers registered once (page-locked, mapped): zero-copy calls */
        for (i = 0; i < 7; ++i) check(vc_host_register(reg[i], reg_len[i]), "vc_host_register");
        check(vc_acl_classify_v4(ctx, proto, src4, port, n, idx, allow), "vc_acl_classify_v4");
        check(vc_route_lookup_v4(ctx, dst4, n, route), "vc_route_lookup_v4");
        /* the same calls from pageable memory (chunked staging) */
        check(vc_acl_classify_v4(ctx, proto, src4, port, n, idx2, NULL), "vc_acl_classify_v4 (p)");
        check(vc_route_lookup_v4(ctx, dst4, n, route2), "vc_route_lookup_v4 (pageable)");
        for (i = 0; i < 7; ++i) check(vc_host_unregister(reg[i]), "vc_host_unregister");
        if (memcmp(idx, idx2, (size_t) n * 4) || memcmp(route, route2, (size_t) n * 4)) {
            fprintf(stderr, "zero-copy and staged results differ\n");
            return 1;
        }
        {
            const vc_packets in = {family, proto, src4, dst4, src6, dst6, port, NULL};
            const vc_pipeline_out out = {p_acl, p_route, p_group, p_allow};
            check(vc_pipeline(ctx, &in, n, NULL, 0, &out), "vc_pipeline");
        }
        for (k = 0; k < n; ++k) {
            if (family[k] == 4 && (p_acl[k] != idx[k] || p_route[k] != route[k] ||
                                   p_allow[k] != allow[k])) {
                fprintf(stderr, "pipeline differs from the single calls at %lld\n", (long long) k);
                return 1;
            }
            if (p_group[k] != -1) {
                fprintf(stderr, "group without a hostname stage\n");
                return 1;
            }
        }
        /* hit counters: the device pointer, a read, and the Prometheus text
         * with the size-query protocol (cap 0 -> VC_ENOMEM + needed length) */
        check(vc_counters_device(ctx, VC_COUNTERS_ACL, NULL, &n_cnt), "vc_counters_device");
        acl_cnt = buf((size_t) n_cnt * 8);
        check(vc_counters_read(ctx, VC_COUNTERS_ACL, acl_cnt, n_cnt), "vc_counters_read");
        rc = vc_counters_prometheus(ctx, "host=gpu0", NULL, 0, &len);
        if (rc != VC_ENOMEM || len <= 0) {
            fprintf(stderr, "size query: rc %d len %lld\n", rc, (long long) len);
            return 1;
        }
        text = buf((size_t) len + 1);
        check(vc_counters_prometheus(ctx, "host=gpu0", text, len + 1, &len), "prometheus");

        n_tcp = check(vc_secgroup_rules(sg, VC_PROTO_TCP, NULL, 0), "rules");
        n_udp = check(vc_secgroup_rules(sg, VC_PROTO_UDP, NULL, 0), "rules");
        n4 = check(vc_routetable_rules(rt, 4, NULL, 0), "routes");
        n6 = check(vc_routetable_rules(rt, 6, NULL, 0), "routes");
        tcp = buf(sizeof(vc_acl_rule) * (size_t) n_tcp);
        udp = buf(sizeof(vc_acl_rule) * (size_t) n_udp);
        v4l = buf(sizeof(vc_net) * (size_t) n4);
        v6l = buf(sizeof(vc_net) * (size_t) n6);
        vc_secgroup_rules(sg, VC_PROTO_TCP, tcp, n_tcp);
        vc_secgroup_rules(sg, VC_PROTO_UDP, udp, n_udp);
        vc_routetable_rules(rt, 4, v4l, n4);
        vc_routetable_rules(rt, 6, v6l, n6);

        f = fopen(argv[1], "wb");
        if (!f) {
            perror(argv[1]);
            return 1;
        }
        {
            const int32_t sizes[6] = {(int32_t) sizeof(vc_acl_rule), (int32_t) sizeof(vc_net),
                                      n_tcp, n_udp, n4, n6};
            put(f, "VCABI1\0\0", 8);
            put(f, &n, 8);
            put(f, sizes, sizeof sizes);
        }
        put(f, tcp, sizeof(vc_acl_rule) * (size_t) n_tcp);
        put(f, udp, sizeof(vc_acl_rule) * (size_t) n_udp);
        put(f, v4l, sizeof(vc_net) * (size_t) n4);
        put(f, v6l, sizeof(vc_net) * (size_t) n6);
        put(f, proto, (size_t) n);
        put(f, src4, (size_t) n * 4);
        put(f, port, (size_t) n * 2);
        put(f, dst4, (size_t) n * 4);
        put(f, family, (size_t) n);
        put(f, src6, (size_t) n * 16);
        put(f, dst6, (size_t) n * 16);
        put(f, idx, (size_t) n * 4);
        put(f, allow, (size_t) n);
        put(f, route, (size_t) n * 4);
        put(f, p_acl, (size_t) n * 4);
        put(f, p_route, (size_t) n * 4);
        put(f, p_allow, (size_t) n);
        put(f, &n_cnt, 8);
        put(f, acl_cnt, (size_t) n_cnt * 8);
        put(f, &len, 8);
        put(f, text, (size_t) len);
        fclose(f);
        printf("ok: %lld items, %d+%d rules, %d+%d routes, %lld bytes of metrics\n",
               (long long) n, n_tcp, n_udp, n4, n6, (long long) len);
    }
    vc_routetable_free(rt);
    vc_secgroup_free(sg);
    vc_destroy(ctx);
    return 0;
}

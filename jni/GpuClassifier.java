package vproxy.component.secure;

import vproxybase.util.Utils;

import java.io.IOException;
import java.nio.ByteBuffer;

/**
 * JNI face of libvclassify (include/vclassify.h), selected with
 * -Dclassifier=gpu (ClassifierConfig) and loaded the way
 * vfd/posix/PosixFDs.java:12-21 loads vfdposix.  Every batch is a set of
 * direct ByteBuffers (native byte order, SoA, n items); results are indices
 * into the live Java lists, -1 = null / default, so callers map them back
 * exactly as SecurityGroup.allow, RouteTable.lookup and
 * Upstream.searchForGroup would have returned them.  Strings are UTF-8
 * (include/vclassify.h "String encoding").
 *
 * Failures: IllegalArgumentException (VC_EINVAL, a short or null buffer,
 * offsets that decrease), IllegalStateException (VC_ESTATE: nothing compiled
 * yet), IOException (VC_EDEVICE / VC_ENOMEM: the device failed; sticky in the
 * HIP runtime).  GpuContext turns the last two into the Java fallback.
 * Native side: jni/vproxy_component_secure_GpuClassifier.c.
 */
public final class GpuClassifier {
    private static boolean loaded;

    /** Loads the JNI library once; prints a hint and exits when it is missing (PosixFDs.java:12-21). */
    public static synchronized void load() {
        if (loaded) {
            return;
        }
        String lib = ClassifierConfig.libname;
        try {
            System.loadLibrary(lib);
        } catch (UnsatisfiedLinkError e) {
            System.out.println(lib + " not found, requires lib" + lib + ".so and libvclassify.so on java.library.path");
            e.printStackTrace(System.out);
            Utils.exit(1);
        }
        loaded = true;
    }

    private GpuClassifier() {
    }

    public static native long create(int device) throws IOException;
    public static native void destroy(long ctx);

    /** VC_SNAP_* bits of vc_pin_acquire: the snapshots GpuContext maps result indices through. */
    public static final int SNAP_ACL = 0, SNAP_ROUTE = 1, SNAP_UPSTREAM = 2, SNAP_HOSTS = 3,
        SNAP_SERVERS = 4, SNAP_CERTS = 5, SNAP_MIRROR = 6, SNAP_VNI = 7, SNAP_ALL = 0xFF;
    /** Pins the snapshots of {@code kinds} (bit set of SNAP_*) current now; a handle for bindPin / pinRelease. */
    public static native long pinAcquire(long ctx, int kinds) throws IOException;
    /** Calls on ctx from this thread use pin's snapshots (0 = the current ones again). */
    public static native void bindPin(long ctx, long pin) throws IOException;
    /** The generation of a pinned snapshot (every publish on a context takes the next one; 0 = none). */
    public static native long pinGeneration(long pin, int kind) throws IOException;
    public static native void pinRelease(long pin);
    /** Page-lock and map a long-lived direct buffer once: calls on it become zero-copy. */
    public static native void registerBuffer(ByteBuffer buf) throws IOException;
    public static native void unregisterBuffer(ByteBuffer buf) throws IOException;

    /** tcp / udp: packed vc_acl_rule[] (52 B each) in SecurityGroup list order. */
    public static native void compileAcl(long ctx, ByteBuffer tcp, int nTcp, ByteBuffer udp, int nUdp,
                                         boolean defaultAllow) throws IOException;
    public static native void classifyAclV4(long ctx, ByteBuffer proto, ByteBuffer src4, ByteBuffer port,
                                            int n, ByteBuffer outIdx, ByteBuffer outAllow) throws IOException;
    public static native void classifyAclV6(long ctx, ByteBuffer proto, ByteBuffer src6, ByteBuffer port,
                                            int n, ByteBuffer outIdx, ByteBuffer outAllow) throws IOException;

    /** v4 / v6: packed vc_net[] (40 B each) of rulesV4 / rulesV6 in list order. */
    public static native void compileRoutes(long ctx, ByteBuffer v4, int n4, ByteBuffer v6, int n6)
        throws IOException;
    /**
     * Switch.tables (Switch.java:560-566): vni[n] ints; v4 / v6 packed vc_net[] of every table in turn,
     * split by the n + 1 int offsets v4Off / v6Off.  switchClassify then routes each packet in the
     * table of its VNI (VC_SWITCH_NO_TABLE = -2: tables.get(vni) is null).
     */
    public static native void compileVniRoutes(long ctx, ByteBuffer vni, ByteBuffer v4, ByteBuffer v4Off,
                                               ByteBuffer v6, ByteBuffer v6Off, int n) throws IOException;
    public static native void lookupRouteV4(long ctx, ByteBuffer dst4, int n, ByteBuffer out) throws IOException;
    public static native void lookupRouteV6(long ctx, ByteBuffer dst6, int n, ByteBuffer out) throws IOException;

    /**
     * groups: packed vc_group_annos[] whose string slots hold offsets into `strings` (-1 = null);
     * the buffer is not modified (the shim rebases a copy).
     */
    public static native void compileUpstream(long ctx, ByteBuffer groups, int n, ByteBuffer strings)
        throws IOException;
    public static native void searchHints(long ctx, ByteBuffer hostBlob, ByteBuffer hostOff, ByteBuffer hostNull,
                                          ByteBuffer port, ByteBuffer uriBlob, ByteBuffer uriOff,
                                          ByteBuffer uriNull, int n, ByteBuffer outGroup) throws IOException;
    public static native void compileHostsText(long ctx, ByteBuffer text, int len) throws IOException;
    /** qnames as Formatter.parseDomainName's wire bytes (blob + n + 1 int offsets). */
    public static native void classifyDns(long ctx, ByteBuffer qBlob, ByteBuffer qOff, int n,
                                          ByteBuffer outKind, ByteBuffer outValue) throws IOException;

    /** The first read of each new HTTP/1 connection (blob + n + 1 int offsets): group = handle
     *  index of HttpContext.connectionHint's Upstream.searchForGroup or -1, kind = VC_HTTP_*
     *  (0: the hint is null). */
    public static native void httpHint(long ctx, ByteBuffer heads, ByteBuffer off, int n,
                                       ByteBuffer outGroup, ByteBuffer outKind) throws IOException;

    /** A Switch drain-loop batch: family (4/6), proto, src4, dst4, src6, dst6, dport, host ids. */
    public static native void pipeline(long ctx, ByteBuffer family, ByteBuffer proto, ByteBuffer src4,
                                       ByteBuffer dst4, ByteBuffer src6, ByteBuffer dst6, ByteBuffer dport,
                                       ByteBuffer hostId, ByteBuffer poolGroup, int nPool, int n,
                                       ByteBuffer outAcl, ByteBuffer outRoute, ByteBuffer outGroup,
                                       ByteBuffer outAllow) throws IOException;

    /**
     * pipeline with compact IPv6 rows: src6 / dst6 hold n6 rows of 16 bytes, row k the addresses
     * of the batch's k-th family-6 packet (packet order); family is required.  Runs zero-copy over
     * registered buffers; n6 must equal the number of family-6 packets.
     */
    public static native void pipelineCompact6(long ctx, ByteBuffer family, ByteBuffer proto,
                                               ByteBuffer src4, ByteBuffer dst4, ByteBuffer src6,
                                               ByteBuffer dst6, int n6, ByteBuffer dport,
                                               ByteBuffer hostId, ByteBuffer poolGroup, int nPool,
                                               int n, ByteBuffer outAcl, ByteBuffer outRoute,
                                               ByteBuffer outGroup, ByteBuffer outAllow)
        throws IOException;

    /**
     * Switch.PacketHandler.readable per datagram: bareVXLanAccess.allow on the sender, the VXLAN
     * parse (out: 12 buffers in vc_pkt_out order, null = skip) and the inner packet's route in the
     * table of its VNI.  Only datagrams VProxyEncryptedPacket.from rejected belong in the batch
     * (Switch.java:648-679): user-iface traffic takes the Java path first.
     */
    public static native void switchClassify(long ctx, ByteBuffer blob, ByteBuffer off, int n, int layer,
                                             ByteBuffer remoteFamily, ByteBuffer remote4, ByteBuffer remote6,
                                             int bindPort, ByteBuffer[] out, ByteBuffer outAcl,
                                             ByteBuffer outAllow, ByteBuffer outRoute) throws IOException;

    /**
     * DNSServer's drain loop per datagram (DNSServer.java:457-500): securityGroup.allow(UDP,
     * remote, remote port), Formatter.parsePackets, isResponse / opcode / handleRequest's
     * question classification.  out: status, acl, nq, qtype, kind, value (vc_dnsd_out order;
     * the per-question arrays hold VC_DNSD_MAXQ entries per datagram).
     */
    public static native void dnsDatagrams(long ctx, ByteBuffer blob, ByteBuffer off, int n,
                                           ByteBuffer remoteFamily, ByteBuffer remote4, ByteBuffer remote6,
                                           ByteBuffer remotePort, ByteBuffer[] out) throws IOException;

    /** servers: packed vc_server[] (32 B each) per group; groupOff: n + 1 ints. */
    public static native void compileServers(long ctx, ByteBuffer servers, ByteBuffer groupOff, int nGroups)
        throws IOException;
    public static native void setServerHealth(long ctx, ByteBuffer healthy, int nServers) throws IOException;
    /** view 0 = next(source), 4 = nextIPv4, 6 = nextIPv6; out: index in the group's server list or -1. */
    public static native void selectSourceV4(long ctx, ByteBuffer group, ByteBuffer src4, int n, int view,
                                             ByteBuffer outServer) throws IOException;

    /** frames: blob + n + 1 int offsets; out: 12 direct buffers in vc_pkt_out order (null = skip). */
    public static native void parsePackets(long ctx, ByteBuffer blob, ByteBuffer off, int n, int layer,
                                           ByteBuffer[] out) throws IOException;

    public static native void compileCerts(long ctx, ByteBuffer names, ByteBuffer off, ByteBuffer holder,
                                           int nNames, int nHolders) throws IOException;
    public static native void chooseCerts(long ctx, ByteBuffer sni, ByteBuffer off, ByteBuffer isNull, int n,
                                          ByteBuffer outHolder) throws IOException;

    public static native void compileMirror(long ctx, ByteBuffer filters, int n) throws IOException;
    public static native void mirrorSwitch(long ctx, int origin, ByteBuffer blob, ByteBuffer off, int n,
                                           int layer, ByteBuffer outMirrors) throws IOException;

    public static native void enableCounters(long ctx, boolean on) throws IOException;
    /** GlobalInspection-style text of the per-rule hit counters. */
    public static native String countersPrometheus(long ctx, String extraLabels) throws IOException;
}

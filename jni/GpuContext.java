package vproxy.component.secure;

import vfd.IP;
import vfd.IPv4;
import vproxy.component.svrgroup.Upstream;
import vproxybase.connection.Protocol;
import vproxybase.util.Annotations;
import vproxybase.util.LogType;
import vproxybase.util.Logger;
import vproxybase.util.Network;
import vswitch.RouteTable;

import java.io.IOException;
import java.nio.ByteBuffer;
import java.nio.ByteOrder;
import java.nio.charset.StandardCharsets;
import java.util.ArrayList;
import java.util.List;
import java.util.concurrent.locks.ReentrantReadWriteLock;
import java.util.function.Function;

/**
 * One libvclassify context (one GPU) with the fallback INTEGRATION.md
 * promises: every batched native call goes through {@link #call}, which
 * returns false when the caller must answer that batch with the reference's
 * Java classifiers instead (SecurityGroup.allow, RouteTable.lookup,
 * Upstream.searchForGroup, the DNS parse):
 *
 * <ul>
 *   <li>IOException (VC_EDEVICE / VC_ENOMEM): the device failed.  HIP errors
 *   are sticky, so the context is marked dead, the failure is logged once,
 *   and this batch and every later one take the Java path until restart.</li>
 *   <li>IllegalStateException (VC_ESTATE): nothing compiled yet for that
 *   classifier (a table arrives after the first packets).  Java path for
 *   this batch only; the context stays alive.</li>
 *   <li>IllegalArgumentException (VC_EINVAL, a short buffer): a bug in the
 *   caller, rethrown.</li>
 * </ul>
 *
 * The Java lists stay live and authoritative: the library only holds
 * compiled snapshots of them, so the fallback needs no state transfer.  The
 * compile helpers pack the lists in the vclassify.h layouts and keep the
 * list each index refers to.  A result maps back to the rule object of the
 * snapshot that produced it because publishing is one critical section:
 * compile* hold the write side of {@code snap} across the native compile
 * and the list swap, and {@link #batch} holds the read side across a
 * batch's native call and its index mapping (aclRule / route / group), so
 * no recompile can land between the two.  Batches on different event-loop
 * threads share the read side and never wait for each other.
 */
public final class GpuContext {
    // include/vclassify.h struct sizes (tests/test_jni_shim.py checks them
    // against the C layouts)
    public static final int NET_BYTES = 40;          // vc_net
    public static final int ACL_RULE_BYTES = 52;     // vc_acl_rule
    public static final int ANNOS_BYTES = 32;        // vc_annos
    public static final int GROUP_ANNOS_BYTES = 64;  // vc_group_annos

    public interface Call {
        void run(long ctx) throws IOException;
    }

    private final long ctx;
    private final String name;
    private volatile boolean dead;

    // the lists the compiled snapshots index into
    private volatile List<SecurityGroupRule> tcpRules = List.of();
    private volatile List<SecurityGroupRule> udpRules = List.of();
    private volatile List<RouteTable.RouteRule> routesV4 = List.of();
    private volatile List<RouteTable.RouteRule> routesV6 = List.of();
    private volatile List<Upstream.ServerGroupHandle> handles = List.of();

    // write: a compile + list swap; read: a batch's call + index mapping
    private final ReentrantReadWriteLock snap = new ReentrantReadWriteLock();

    private GpuContext(long ctx, String name) {
        this.ctx = ctx;
        this.name = name;
    }

    /**
     * A context on -Dclassifier_device when -Dclassifier=gpu, else null (the
     * callers then never build batches).  vc_create failing at start-up is
     * fatal, as PosixFDs treats a missing vfdposix: there is no silent CPU
     * path behind -Dclassifier=gpu.
     */
    public static GpuContext createIfEnabled(String name) {
        if (!ClassifierConfig.useGpu) {
            return null;
        }
        GpuClassifier.load();
        try {
            return new GpuContext(GpuClassifier.create(ClassifierConfig.device), name);
        } catch (IOException e) {
            Logger.shouldNotHappen("creating gpu classifier " + name + " on device " + ClassifierConfig.device + " failed", e);
            vproxybase.util.Utils.exit(1);
            return null;
        }
    }

    public boolean alive() {
        return !dead;
    }

    /** Runs one native call; false = answer this batch with the Java classifiers. */
    public boolean call(Call c) {
        if (dead) {
            return false;
        }
        try {
            c.run(ctx);
            return true;
        } catch (IllegalStateException e) {
            assert Logger.lowLevelDebug("gpu classifier " + name + ": " + e.getMessage() + ", java path for this batch");
            return false;
        } catch (IOException e) {
            if (!dead) {
                dead = true;
                Logger.error(LogType.SYS_ERROR, "gpu classifier " + name + " failed, the java classifiers answer every batch from now on", e);
            }
            return false;
        }
    }

    /**
     * One batch: the native call, then {@code map} with its outcome (true =
     * the outputs are valid; false = answer the batch with the Java
     * classifiers), both under the read side of the snapshot lock, so every
     * aclRule / route / group lookup inside {@code map} sees the lists of
     * the snapshot the call classified against.
     */
    public <T> T batch(Call c, Function<Boolean, T> map) {
        snap.readLock().lock();
        try {
            return map.apply(call(c));
        } finally {
            snap.readLock().unlock();
        }
    }

    /** A control-plane call (compile, register): false when it failed and the context is not usable for it. */
    public boolean control(Call c) {
        return call(c);
    }

    /** A compile and the swap of the lists its indices refer to, as one publish (see the class comment). */
    private boolean publish(Call compile, Runnable swap) {
        snap.writeLock().lock();
        try {
            boolean ok = control(compile);
            if (ok) {
                swap.run();
            }
            return ok;
        } finally {
            snap.writeLock().unlock();
        }
    }

    // ------------------------------------------------------------------
    // packing (native byte order, the layouts of include/vclassify.h)
    // ------------------------------------------------------------------
    public static ByteBuffer direct(long bytes) {
        if (bytes > Integer.MAX_VALUE) {
            throw new IllegalArgumentException("batch of " + bytes + " bytes");
        }
        return ByteBuffer.allocateDirect((int) Math.max(bytes, 1)).order(ByteOrder.nativeOrder());
    }

    /** vc_net: 16 ip bytes, 16 mask bytes, ip_len, mask_len (Network.parseMask form). */
    private static void putNet(ByteBuffer b, Network n) {
        byte[] ip = n.getRawIpBytes();
        byte[] mask = Network.parseMask(n.getMask());
        int p = b.position();
        for (int i = 0; i < 16; ++i) b.put(p + i, i < ip.length ? ip[i] : 0);
        for (int i = 0; i < 16; ++i) b.put(p + 16 + i, i < mask.length ? mask[i] : 0);
        b.position(p + 32);
        b.putInt(ip.length);
        b.putInt(mask.length);
    }

    /** SecurityGroup lists -> compileAcl (after every addRule / removeRule, SecurityGroup.java:56-103). */
    public boolean compileSecurityGroup(SecurityGroup sg) {
        List<SecurityGroupRule> tcp = new ArrayList<>();
        List<SecurityGroupRule> udp = new ArrayList<>();
        for (SecurityGroupRule r : sg.getRules()) {
            (r.protocol == Protocol.TCP ? tcp : udp).add(r);
        }
        ByteBuffer t = packRules(tcp), u = packRules(udp);
        return publish(c -> GpuClassifier.compileAcl(c, t, tcp.size(), u, udp.size(), sg.defaultAllow), () -> {
            tcpRules = tcp;
            udpRules = udp;
        });
    }

    private static ByteBuffer packRules(List<SecurityGroupRule> rules) {
        ByteBuffer b = direct((long) rules.size() * ACL_RULE_BYTES);
        for (SecurityGroupRule r : rules) {
            putNet(b, r.network);
            b.putInt(r.minPort);
            b.putInt(r.maxPort);
            b.putInt(r.allow ? 1 : 0);
        }
        return b;
    }

    /** RouteTable lists -> compileRoutes (RouteTable.java:68-172 keeps their order). */
    public boolean compileRouteTable(RouteTable rt) {
        List<RouteTable.RouteRule> v4 = new ArrayList<>();
        List<RouteTable.RouteRule> v6 = new ArrayList<>();
        for (RouteTable.RouteRule r : rt.getRules()) {
            (r.rule.getIp() instanceof IPv4 ? v4 : v6).add(r);
        }
        ByteBuffer a = packNets(v4), b = packNets(v6);
        return publish(c -> GpuClassifier.compileRoutes(c, a, v4.size(), b, v6.size()), () -> {
            routesV4 = v4;
            routesV6 = v6;
        });
    }

    private static ByteBuffer packNets(List<RouteTable.RouteRule> rules) {
        ByteBuffer b = direct((long) rules.size() * NET_BYTES);
        for (RouteTable.RouteRule r : rules) {
            putNet(b, r.rule);
        }
        return b;
    }

    /** Upstream.serverGroupHandles -> compileUpstream (handle annotations, then the group's). */
    public boolean compileUpstream(Upstream ups) {
        List<Upstream.ServerGroupHandle> hs = ups.getServerGroupHandles();
        ByteArrayBuilder strings = new ByteArrayBuilder();
        ByteBuffer g = direct((long) hs.size() * GROUP_ANNOS_BYTES);
        for (Upstream.ServerGroupHandle h : hs) {
            putAnnos(g, h.getAnnotations(), strings);
            putAnnos(g, h.group.getAnnotations(), strings);
        }
        ByteBuffer s = strings.toDirect();
        return publish(c -> GpuClassifier.compileUpstream(c, g, hs.size(), s), () -> handles = hs);
    }

    /**
     * The hosts map -> compileHostsText (Resolver.getHosts' text); a hosts
     * value is the index of the file's valid line, so {@code swap} installs
     * the caller's line -> IP list of the same text under the same publish.
     */
    public boolean compileHostsText(ByteBuffer text, int len, Runnable swap) {
        return publish(c -> GpuClassifier.compileHostsText(c, text, len), swap);
    }

    /** vc_annos with string slots as offsets into `strings` (-1 = null). */
    private static void putAnnos(ByteBuffer b, Annotations a, ByteArrayBuilder strings) {
        putString(b, a.ServerGroup_HintHost, strings);
        b.putInt(a.ServerGroup_HintPort);
        putString(b, a.ServerGroup_HintUri, strings);
        b.putInt(0);  // padding to 32 bytes
    }

    private static void putString(ByteBuffer b, String s, ByteArrayBuilder strings) {
        if (s == null) {
            b.putLong(-1);
            b.putInt(0);
            return;
        }
        byte[] u = s.getBytes(StandardCharsets.UTF_8);
        b.putLong(strings.size());
        b.putInt(u.length);
        strings.append(u);
    }

    // ------------------------------------------------------------------
    // results -> the Java objects of the compiled snapshot (call these
    // inside batch(): the read side pins the lists to the call's snapshot)
    // ------------------------------------------------------------------
    public SecurityGroupRule aclRule(Protocol p, int idx) {
        return idx < 0 ? null : (p == Protocol.TCP ? tcpRules : udpRules).get(idx);
    }

    public RouteTable.RouteRule route(IP dst, int idx) {
        return idx < 0 ? null : (dst instanceof IPv4 ? routesV4 : routesV6).get(idx);
    }

    public Upstream.ServerGroupHandle group(int idx) {
        return idx < 0 ? null : handles.get(idx);
    }

    public void close() {
        GpuClassifier.destroy(ctx);
    }

    /** A growable byte array for the annotation strings. */
    static final class ByteArrayBuilder {
        private byte[] a = new byte[256];
        private int n;

        int size() {
            return n;
        }

        void append(byte[] b) {
            if (n + b.length > a.length) {
                a = java.util.Arrays.copyOf(a, Math.max(2 * a.length, n + b.length));
            }
            System.arraycopy(b, 0, a, n, b.length);
            n += b.length;
        }

        ByteBuffer toDirect() {
            ByteBuffer b = direct(n);
            b.put(a, 0, n).flip();
            return b;
        }
    }
}

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
import java.util.concurrent.atomic.AtomicInteger;
import java.util.function.BiFunction;

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
 * list each index refers to.
 *
 * <p>Readers never wait for a compile, as the reference's copy-on-write
 * swaps never make them wait (SecurityGroup.java:56-103,
 * Upstream.java:146-157).  A {@link View} is one published state: a native
 * pin of the snapshots (vc_pin_acquire) and the Java lists their indices
 * refer to.  A compile runs the native compile with no lock a batch takes,
 * pins what it published, and swaps {@link #view} in one volatile write.
 * {@link #batch} retains the current view (a compare-and-set, retried only
 * when a swap raced it), binds its pin to the thread for the native call
 * (vc_pin_bind), and hands the view to {@code map}, which maps indices
 * through the view's lists -- those of the snapshot the call classified
 * against -- with nothing held, so {@code map} may do I/O or even compile.
 * A replaced view's pin is released when its last batch ends.
 * tests/native/pin_loop.c replays this protocol on the GPU while the
 * control thread recompiles C3-size route tables.
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

    // the current view; every compile replaces it (publish)
    private volatile View view;
    // serialises compiles (control threads only): batches never take it
    private final Object compileLock = new Object();

    private GpuContext(long ctx, String name) throws IOException {
        this.ctx = ctx;
        this.name = name;
        // nothing compiled: every kind pinned empty, so a batch before the
        // first publish gets VC_ESTATE (the Java path), never a snapshot its
        // view has no lists for
        this.view = new View(GpuClassifier.pinAcquire(ctx, GpuClassifier.SNAP_ALL), List.of(), List.of(),
            List.of(), List.of(), List.of(), null);
    }

    /**
     * One published state: the pinned native snapshots and the Java lists
     * their result indices refer to.  Immutable.  {@code refs} counts the
     * holders: 1 for being {@link #view}, 1 per batch running on it.
     */
    public static final class View {
        final long pin;
        public final List<SecurityGroupRule> tcpRules, udpRules;
        public final List<RouteTable.RouteRule> routesV4, routesV6;
        public final List<Upstream.ServerGroupHandle> handles;
        /** What the caller installed with compileHostsText (its line -> IP list for hosts values). */
        public final Object hosts;
        private final AtomicInteger refs = new AtomicInteger(1);

        View(long pin, List<SecurityGroupRule> tcpRules, List<SecurityGroupRule> udpRules,
             List<RouteTable.RouteRule> routesV4, List<RouteTable.RouteRule> routesV6,
             List<Upstream.ServerGroupHandle> handles, Object hosts) {
            this.pin = pin;
            this.tcpRules = tcpRules;
            this.udpRules = udpRules;
            this.routesV4 = routesV4;
            this.routesV6 = routesV6;
            this.handles = handles;
            this.hosts = hosts;
        }

        View withPin(long p) {
            return new View(p, tcpRules, udpRules, routesV4, routesV6, handles, hosts);
        }

        /** false once the view was replaced and its last batch ended (its pin is gone). */
        boolean retain() {
            while (true) {
                int r = refs.get();
                if (r == 0) {
                    return false;
                }
                if (refs.compareAndSet(r, r + 1)) {
                    return true;
                }
            }
        }

        void release() {
            if (refs.decrementAndGet() == 0) {
                GpuClassifier.pinRelease(pin);
            }
        }

        // results -> the Java objects of this view's snapshot
        public SecurityGroupRule aclRule(Protocol p, int idx) {
            return idx < 0 ? null : (p == Protocol.TCP ? tcpRules : udpRules).get(idx);
        }

        public RouteTable.RouteRule route(IP dst, int idx) {
            return idx < 0 ? null : (dst instanceof IPv4 ? routesV4 : routesV6).get(idx);
        }

        public Upstream.ServerGroupHandle group(int idx) {
            return idx < 0 ? null : handles.get(idx);
        }
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
     * One batch: the native call on the current view's snapshots, then
     * {@code map} with its outcome (true = the outputs are valid; false =
     * answer the batch with the Java classifiers) and that view, whose
     * aclRule / route / group map the outputs to the objects of the
     * snapshot that produced them.  No lock is held at any point: a
     * concurrent compile publishes a new view, and this batch keeps its own.
     */
    public <T> T batch(Call c, BiFunction<Boolean, View, T> map) {
        View v;
        do {
            v = view;
        } while (!v.retain());      // lost a race with a swap and its last release: read again
        final long pin = v.pin;
        boolean ok;
        try {
            ok = call(h -> {
                GpuClassifier.bindPin(h, pin);
                try {
                    c.run(h);
                } finally {
                    GpuClassifier.bindPin(h, 0);
                }
            });
        } finally {
            v.release();            // the outputs are in the caller's buffers: the pin may go
        }
        return map.apply(ok, v);
    }

    /** The current view (control-plane reads; a batch gets its own from {@link #batch}). */
    public View view() {
        return view;
    }

    /** A control-plane call (compile, register): false when it failed and the context is not usable for it. */
    public boolean control(Call c) {
        return call(c);
    }

    /** Builds the next view from the previous one and the pin of what the compile published. */
    interface Next {
        View make(long pin, View old);
    }

    /**
     * A compile and the view that describes it: the native compile (no
     * batch waits for it), a pin of the snapshots it published, and the swap.
     * Compiles are serialised by {@code compileLock}, so the pin holds
     * exactly this compile's snapshot beside the ones the old view pinned.
     */
    private boolean publish(Call compile, Next next) {
        synchronized (compileLock) {
            if (!control(compile)) {
                return false;
            }
            long pin;
            try {
                pin = GpuClassifier.pinAcquire(ctx, GpuClassifier.SNAP_ALL);
            } catch (IOException e) {
                return control(c -> {
                    throw e;
                });
            }
            View old = view;
            view = next.make(pin, old);
            old.release();
            return true;
        }
    }

    /**
     * Every other call that publishes a snapshot -- compileServers,
     * setServerHealth, compileCerts, compileMirror, compileVniRoutes -- goes
     * through here, so the next batch's view pins it.
     */
    public boolean publish(Call compile) {
        return publish(compile, (pin, old) -> old.withPin(pin));
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
        return publish(c -> GpuClassifier.compileAcl(c, t, tcp.size(), u, udp.size(), sg.defaultAllow),
            (pin, old) -> new View(pin, tcp, udp, old.routesV4, old.routesV6, old.handles, old.hosts));
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
        return publish(c -> GpuClassifier.compileRoutes(c, a, v4.size(), b, v6.size()),
            (pin, old) -> new View(pin, old.tcpRules, old.udpRules, v4, v6, old.handles, old.hosts));
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
        return publish(c -> GpuClassifier.compileUpstream(c, g, hs.size(), s),
            (pin, old) -> new View(pin, old.tcpRules, old.udpRules, old.routesV4, old.routesV6, hs, old.hosts));
    }

    /**
     * The hosts map -> compileHostsText (Resolver.getHosts' text); a hosts
     * value is the index of the file's valid line, so {@code lines} (the
     * caller's line -> IP list of the same text) goes into the same view.
     */
    public boolean compileHostsText(ByteBuffer text, int len, Object lines) {
        return publish(c -> GpuClassifier.compileHostsText(c, text, len),
            (pin, old) -> new View(pin, old.tcpRules, old.udpRules, old.routesV4, old.routesV6, old.handles, lines));
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

    public void close() {
        view.release();
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

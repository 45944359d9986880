package vswitch;

import vfd.DatagramFD;
import vfd.IP;
import vfd.IPPort;
import vfd.IPv4;
import vproxy.component.secure.ClassifierConfig;
import vproxy.component.secure.GpuClassifier;
import vproxy.component.secure.GpuContext;
import vproxybase.selector.HandlerContext;
import vproxybase.selector.SelectorEventLoop;
import vproxybase.util.ByteArray;
import vproxybase.util.LogType;
import vproxybase.util.Logger;
import vpacket.VProxyEncryptedPacket;

import java.io.IOException;
import java.nio.ByteBuffer;

/**
 * Switch.PacketHandler.readable (core/src/main/java/vswitch/Switch.java:744-776)
 * in batches.  The handler drains the socket into a batch of up to
 * ClassifierConfig.batch datagrams.  Each datagram first goes through
 * VProxyEncryptedPacket.from in Java, as handleNetworkAndGetVXLanPacket does
 * (:643-676): user-iface traffic stays on the Java path.  The datagrams it
 * rejects -- the bare-VXLAN branch (:677-684) -- are classified in one
 * GpuClassifier.switchClassify call (vc_switch_classify:
 * bareVXLanAccess.allow(UDP, remote, bind port), VXLanPacket.from, the
 * VNI's table and its RouteTable.lookup of the inner destination).  Then
 * every datagram of the batch is handled in arrival order, so the network
 * stack sees the same sequence as from the reference loop:
 *
 * <pre>
 *   decrypted              Host.handleEncrypted (the err == null branch, :650-676)
 *   bare, denied           dropped ("not in allowed security-group", :711-714)
 *   bare, parse error      dropped ("invalid packet for vxlan", :684-687)
 *   bare, parse throws     Host.handleJava: whatever the reference body does
 *   bare, parsed           Host.handleBare with the route index (-1 = null,
 *                          VC_SWITCH_NO_TABLE = -2: tables.get(vni) is null)
 * </pre>
 *
 * When the GPU call fails (GpuContext.call: device dead or nothing compiled
 * yet) every bare datagram of the batch takes Host.handleJava, the
 * reference body.  The kernel's results are bit-exact with the Java calls
 * they replace (tests/test_gpu_switch.py).
 */
public final class SwitchDrainBatcher {
    public static final int PKT_OK = 0, PKT_EXCEPTION = 4, PKT_LOOP = 5;   // VC_PKT_*
    private static final int LAYER_VXLAN = 0;                              // VC_LAYER_VXLAN
    private static final int MAX_DATAGRAM = 65536;

    public interface Host {
        /** new VProxyEncryptedPacket(Switch.this::getKey), when its from(data) returns null (:644-648). */
        VProxyEncryptedPacket tryDecrypt(ByteArray data);

        void handleEncrypted(String uuid, SelectorEventLoop loop, IPPort remote, VProxyEncryptedPacket p);

        /**
         * The bare branch after VXLanPacket.from succeeded (:688-731), then inputVXLan with the route:
         * an index into the VNI table's lists of the snapshot the batch ran on, which {@code view} pins.
         */
        void handleBare(String uuid, SelectorEventLoop loop, IPPort remote, ByteArray data, int route,
                        GpuContext.View view);

        /** The reference body: handleNetworkAndGetVXLanPacket + inputVXLan (:760-774). */
        void handleJava(String uuid, SelectorEventLoop loop, IPPort remote, ByteArray data);

        String newHandlingUUID();

        int bindPort();
    }

    private final GpuContext gpu;
    private final Host host;
    private final int cap = ClassifierConfig.batch;
    private final ByteBuffer recv = ByteBuffer.allocate(MAX_DATAGRAM);

    // the bare datagrams of the batch (SoA, registered once: zero-copy calls);
    // room for cap datagrams of 256 bytes plus one largest datagram, so
    // every pass of the drain loop receives at least one whatever
    // -Dclassifier_batch says (tests/native/switch_loop.c replays this rule)
    private final ByteBuffer blob = GpuContext.direct((long) cap * 256 + MAX_DATAGRAM);
    private final ByteBuffer off = GpuContext.direct(4L * (cap + 1));
    private final ByteBuffer family = GpuContext.direct(cap);
    private final ByteBuffer remote4 = GpuContext.direct(4L * cap);
    private final ByteBuffer remote6 = GpuContext.direct(16L * cap);
    private final ByteBuffer status = GpuContext.direct(cap);
    private final ByteBuffer outAcl = GpuContext.direct(4L * cap);
    private final ByteBuffer outAllow = GpuContext.direct(cap);
    private final ByteBuffer outRoute = GpuContext.direct(4L * cap);
    private final ByteBuffer[] pktOut = new ByteBuffer[12];   // vc_pkt_out order: status only

    // every datagram of the batch in arrival order
    private final IPPort[] remotes = new IPPort[cap];
    private final ByteArray[] datas = new ByteArray[cap];
    private final VProxyEncryptedPacket[] decrypted = new VProxyEncryptedPacket[cap];
    private final int[] bareIndex = new int[cap];

    public SwitchDrainBatcher(GpuContext gpu, Host host) {
        this.gpu = gpu;
        this.host = host;
        pktOut[0] = status;
        for (ByteBuffer b : new ByteBuffer[]{blob, off, family, remote4, remote6, status, outAcl, outAllow, outRoute}) {
            gpu.control(c -> GpuClassifier.registerBuffer(b));
        }
    }

    /** PacketHandler.readable (Switch.java:744). */
    public void readable(HandlerContext<DatagramFD> ctx) {
        DatagramFD sock = ctx.getChannel();
        SelectorEventLoop loop = ctx.getEventLoop();
        boolean drained = false;
        while (!drained) {
            int n = 0, nb = 0, bytes = 0;
            while (true) {
                if (n == cap || bytes + MAX_DATAGRAM > blob.capacity()) {
                    break;  // batch full: classify it, then keep draining
                }
                recv.limit(recv.capacity()).position(0);
                IPPort remote;
                try {
                    remote = sock.receive(recv);
                } catch (IOException e) {
                    Logger.error(LogType.CONN_ERROR, "udp sock " + sock + " got error when reading", e);
                    drained = true;
                    break;
                }
                if (recv.position() == 0) {
                    drained = true;
                    break;  // nothing read, quit loop (:757-759)
                }
                byte[] b = new byte[recv.position()];
                recv.flip();
                recv.get(b);
                ByteArray data = ByteArray.from(b);
                remotes[n] = remote;
                datas[n] = data;
                decrypted[n] = host.tryDecrypt(data);
                if (decrypted[n] == null) {
                    bareIndex[n] = nb;
                    packBare(nb++, remote, data, bytes);
                    bytes += b.length;
                }
                ++n;
            }
            dispatch(loop, n, nb);
        }
    }

    private void packBare(int k, IPPort remote, ByteArray data, int pos) {
        off.putInt(4 * k, pos);
        for (int j = 0; j < data.length(); ++j) {
            blob.put(pos + j, data.get(j));
        }
        off.putInt(4 * (k + 1), pos + data.length());
        IP ip = remote.getAddress();
        byte[] a = ip.getAddress();
        if (ip instanceof IPv4) {
            family.put(k, (byte) 4);
            remote4.putInt(4 * k, ((a[0] & 0xff) << 24) | ((a[1] & 0xff) << 16) | ((a[2] & 0xff) << 8) | (a[3] & 0xff));
        } else {
            family.put(k, (byte) 6);
            for (int j = 0; j < 16; ++j) {
                remote6.put(16 * k + j, a[j]);
            }
        }
    }

    private void dispatch(SelectorEventLoop loop, int n, int nb) {
        final int m = nb;
        if (m == 0) {
            act(loop, n, true, null);
            return;
        }
        // route indices resolve against the snapshot that produced them: the
        // view the call ran on (GpuContext.batch), with no lock held
        gpu.batch(c -> GpuClassifier.switchClassify(c, blob, off, m, LAYER_VXLAN, family,
            remote4, remote6, host.bindPort(), pktOut, outAcl, outAllow, outRoute), (ok, view) -> {
            act(loop, n, ok, view);
            return null;
        });
    }

    private void act(SelectorEventLoop loop, int n, boolean ok, GpuContext.View view) {
        for (int i = 0; i < n; ++i) {
            String uuid = host.newHandlingUUID();
            if (decrypted[i] != null) {
                host.handleEncrypted(uuid, loop, remotes[i], decrypted[i]);
                decrypted[i] = null;
                continue;
            }
            if (!ok) {
                host.handleJava(uuid, loop, remotes[i], datas[i]);
                continue;
            }
            int k = bareIndex[i];
            if (outAllow.get(k) == 0) {
                assert Logger.lowLevelDebug(uuid + " not in allowed security-group or invalid packet, drop it");
                continue;
            }
            int st = status.get(k);
            if (st == PKT_EXCEPTION || st == PKT_LOOP) {
                host.handleJava(uuid, loop, remotes[i], datas[i]);
            } else if (st != PKT_OK) {
                assert Logger.lowLevelDebug(uuid + " invalid packet for vxlan, drop it");
            } else {
                host.handleBare(uuid, loop, remotes[i], datas[i], outRoute.getInt(4 * k), view);
            }
        }
    }
}

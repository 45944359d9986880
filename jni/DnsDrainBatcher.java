package vproxy.dns;

import vfd.DatagramFD;
import vfd.IP;
import vfd.IPPort;
import vfd.IPv4;
import vproxy.component.secure.ClassifierConfig;
import vproxy.component.secure.GpuClassifier;
import vproxy.component.secure.GpuContext;
import vproxybase.selector.HandlerContext;
import vproxybase.util.ByteArray;
import vproxybase.util.LogType;
import vproxybase.util.Logger;

import java.io.IOException;
import java.nio.ByteBuffer;

/**
 * DNSServer's drain loop (core/src/main/java/vproxy/dns/DNSServer.java:457-500)
 * in batches: the readable handler receives up to ClassifierConfig.batch
 * datagrams, classifies them in one GpuClassifier.dnsDatagrams call
 * (vc_dns_datagrams: securityGroup.allow(UDP, remote, remote port), read ==
 * 0, Formatter.parsePackets, isResponse / opcode and handleRequest's
 * per-question classification), then acts on each in arrival order exactly
 * as the loop would:
 *
 * <pre>
 *   REJECTED   skipped (continue, :469-472)
 *   EMPTY      read == 0: return (:473-476)
 *   MALFORMED  parsePackets threw: logged, return (:481-486)
 *   RESPONSE   logged, skipped (:489-492)
 *   RECURSIVE  runRecursive (opcode != QUERY :493-496, or a question
 *              handleRequest sends there :116-166)
 *   ANSWER     handleRequest with each question's hosts value / group
 *              index / IP literal / .vproxy.local decided (Host.answer)
 *   HOST       a shape outside the kernel's contract: the loop body in Java
 * </pre>
 *
 * A "return" ends this readable event at that datagram.  The datagrams the
 * batch received after it stay pending and go first into the next event,
 * which the batcher schedules with nextTick: the reference left them in the
 * socket, and the level-triggered selector fires again at once.
 *
 * When the GPU call fails (GpuContext.call returns false: device dead, or
 * nothing compiled yet) every datagram of the batch runs the reference loop
 * body (Host.javaPath), which stops where that body returns.  The C replay
 * of this class, tests/native/dnsd_loop.c, is what the GPU tier checks
 * against the reference loop (tests/test_gpu_dnsd_loop.py).
 *
 * Wiring (DNSServer.start, :457): when {@code gpu != null} the anonymous
 * Handler's readable becomes {@code batcher.readable(ctx)}; the UDP list of
 * {@code securityGroup}, the rrsets Upstream and the hosts map are compiled
 * into {@code gpu} after each change (GpuContext.compileSecurityGroup /
 * compileUpstream / compileHostsText).  Host.answer gets the batch's
 * GpuContext.View with the indices, so the group indices and hosts values
 * map through the lists of the snapshot the call classified against; no
 * lock is held while the batch is acted on (a recompile never waits for
 * it, and it never waits for a recompile).
 */
public final class DnsDrainBatcher {
    public static final int ANSWER = 0, RECURSIVE = 1, RESPONSE = 2, REJECTED = 3,
        EMPTY = 4, MALFORMED = 5, HOST = 6;                          // VC_DNSD_*
    public static final int MAXQ = 4;                                // VC_DNSD_MAXQ
    private static final int MAX_DATAGRAM = 65536;

    public interface Host {
        /** The reference loop body (:468-498) for one received datagram; false where it returns. */
        boolean javaPath(IPPort remote, ByteArray data);

        /** runRecursive(p, remote) for the datagram's packet (parsed again in Java to forward it). */
        void recursive(IPPort remote, ByteArray data);

        /**
         * handleRequest(p, remote) for the datagram's packet with question q already classified:
         * kind[q] = VC_DNS_HOSTS / GROUP / IP_LITERAL / INTERNAL, value[q] its hosts value, group
         * index (view.group), IP family or 0.  Server choice and the records stay in Java.
         */
        void answer(IPPort remote, ByteArray data, int nq, byte[] kind, int[] value, GpuContext.View view);
    }

    private final GpuContext gpu;
    private final Host host;
    private final int cap = ClassifierConfig.batch;

    // one batch, SoA, registered once so the calls run zero-copy; room for
    // cap datagrams of 512 bytes plus one largest datagram, so fill() always
    // makes progress whatever -Dclassifier_batch says
    private final ByteBuffer blob = GpuContext.direct((long) cap * 512 + MAX_DATAGRAM);
    private final ByteBuffer off = GpuContext.direct(4L * (cap + 1));
    private final ByteBuffer family = GpuContext.direct(cap);
    private final ByteBuffer remote4 = GpuContext.direct(4L * cap);
    private final ByteBuffer remote6 = GpuContext.direct(16L * cap);
    private final ByteBuffer remotePort = GpuContext.direct(2L * cap);
    private final ByteBuffer[] out = {
        GpuContext.direct(cap), GpuContext.direct(4L * cap), GpuContext.direct(cap),
        GpuContext.direct(2L * cap * MAXQ), GpuContext.direct((long) cap * MAXQ),
        GpuContext.direct(4L * cap * MAXQ)};
    private final ByteBuffer recv = ByteBuffer.allocate(MAX_DATAGRAM);

    // the datagrams of the batch, in arrival order; [head, n) not yet dispatched
    private final IPPort[] remotes = new IPPort[cap];
    private final ByteArray[] datas = new ByteArray[cap];
    private int n, head;
    private final byte[] kind = new byte[MAXQ];
    private final int[] value = new int[MAXQ];

    public DnsDrainBatcher(GpuContext gpu, Host host) {
        this.gpu = gpu;
        this.host = host;
        for (ByteBuffer b : new ByteBuffer[]{blob, off, family, remote4, remote6, remotePort}) {
            gpu.control(c -> GpuClassifier.registerBuffer(b));
        }
        for (ByteBuffer b : out) {
            gpu.control(c -> GpuClassifier.registerBuffer(b));
        }
    }

    /** The Handler's readable (DNSServer.java:457). */
    public void readable(HandlerContext<DatagramFD> ctx) {
        while (true) {
            boolean socketEmpty = fill(ctx.getChannel());
            if (n == head) {
                return;
            }
            if (!dispatch()) {   // a return at some datagram: the rest next event
                ctx.getEventLoop().nextTick(() -> readable(ctx));
                return;
            }
            if (socketEmpty) {
                return;
            }
        }
    }

    /**
     * Moves the pending datagrams to the front, then receives until the
     * batch is full or the socket is empty (remote == null, :463-465, or a
     * read error, logged as :460-462); true when the socket had no more.
     */
    private boolean fill(DatagramFD sock) {
        int k = 0;
        for (int i = head; i < n; ++i, ++k) {
            remotes[k] = remotes[i];
            datas[k] = datas[i];
        }
        n = k;
        head = 0;
        int bytes = 0;
        for (int i = 0; i < n; ++i) {
            bytes += datas[i].length();
        }
        while (n < cap && bytes + MAX_DATAGRAM <= blob.capacity()) {
            recv.limit(recv.capacity()).position(0);
            IPPort remote;
            try {
                remote = sock.receive(recv);
            } catch (IOException e) {
                Logger.error(LogType.CONN_ERROR, "reading data from dns sock " + sock + " failed", e);
                return true;
            }
            if (remote == null) {
                return true;
            }
            byte[] b = new byte[recv.position()];
            recv.flip();
            recv.get(b);
            remotes[n] = remote;
            datas[n] = ByteArray.from(b);
            bytes += b.length;
            ++n;
        }
        return false;
    }

    /** Acts on datagrams [head, n); false when the loop would have returned at one of them. */
    private boolean dispatch() {
        final int m = n;
        pack(m);
        // the native call and every group index of this batch resolve against
        // one snapshot: the view the call ran on (GpuContext.batch)
        return gpu.batch(c -> GpuClassifier.dnsDatagrams(c, blob, off, m, family, remote4, remote6,
            remotePort, out), (ok, view) -> act(m, ok, view));
    }

    private boolean act(int m, boolean ok, GpuContext.View view) {
        for (int i = 0; i < m; ++i) {
            head = i + 1;
            if (!ok) {
                if (!host.javaPath(remotes[i], datas[i])) {
                    return false;
                }
                continue;
            }
            int st = out[0].get(i);
            switch (st) {
                case REJECTED:
                    assert Logger.lowLevelDebug("remote " + remotes[i] + " rejected by security-group");
                    break;
                case EMPTY:
                    return false;
                case MALFORMED:
                    Logger.error(LogType.INVALID_EXTERNAL_DATA, "got malformed dns packet from " + remotes[i]);
                    return false;
                case RESPONSE:
                    Logger.error(LogType.INVALID_EXTERNAL_DATA, "received dns packet response from " + remotes[i]);
                    break;
                case RECURSIVE:
                    host.recursive(remotes[i], datas[i]);
                    break;
                case ANSWER: {
                    int nq = out[2].get(i);
                    for (int q = 0; q < nq; ++q) {
                        kind[q] = out[4].get(i * MAXQ + q);
                        value[q] = out[5].getInt(4 * (i * MAXQ + q));
                    }
                    host.answer(remotes[i], datas[i], nq, kind, value, view);
                    break;
                }
                default:  // HOST
                    if (!host.javaPath(remotes[i], datas[i])) {
                        return false;
                    }
            }
        }
        return true;
    }

    private void pack(int m) {
        int pos = 0;
        for (int i = 0; i < m; ++i) {
            off.putInt(4 * i, pos);
            ByteArray d = datas[i];
            for (int j = 0; j < d.length(); ++j) {
                blob.put(pos + j, d.get(j));
            }
            pos += d.length();
            IP ip = remotes[i].getAddress();
            byte[] a = ip.getAddress();
            if (ip instanceof IPv4) {
                family.put(i, (byte) 4);
                remote4.putInt(4 * i, ((a[0] & 0xff) << 24) | ((a[1] & 0xff) << 16) | ((a[2] & 0xff) << 8) | (a[3] & 0xff));
            } else {
                family.put(i, (byte) 6);
                for (int j = 0; j < 16; ++j) {
                    remote6.put(16 * i + j, a[j]);
                }
            }
            remotePort.putShort(2 * i, (short) remotes[i].getPort());
        }
        off.putInt(4 * m, pos);
    }
}

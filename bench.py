#!/usr/bin/env python3
"""Headline benchmark: M classifications/s (ACL + route + host) per BASELINE.json.

Default workload (`--workload c5`, SURVEY.md §8(d) C5, weak scaling): every
rank holds the replicated tables
    SecurityGroup   10k rules with port ranges (C2 generator)
    RouteTable      ~1M IPv4 + 200k IPv6 prefixes inserted shortest-first (C3)
    Upstream        100k hint-host groups (C4), hostname pool of 16M
and, per step, classifies its shard of one seeded global batch of
N = packets_per_gpu x world IPv4 packets (dist.shard: contiguous slices; the
packet generator is index-addressable, so rank r's slice is the same packets
whatever the world size), resident in HBM:
    1. the hostname pool once (Upstream.searchForGroup per hostname)
    2. the fused pipeline kernel per packet: SecurityGroup.allow(src, dport)
       -> RouteTable.lookup(dst) -> pool group of the packet's host id
    3. per-rule hit counters (ACL, route, group), one RCCL all-reduce per
       batch when N > 1 (or with --dist on one GPU).
A "classification" is one packet through all three.  Inputs are synthetic
and generated on the device; nothing is cached between steps.

Other workloads (c1, c2, c2host, c3, c4, mix, ...) time one classifier alone
for DESIGN.md / BASELINE.md, each with its own roofline and CPU baseline.

Launch: python bench.py [--gpus N --steps K --warmup W]; for N > 1 under
torch.distributed.run (one rank per GPU, RCCL).
"""
import argparse
import ctypes as C
import functools
import json
import os
import sys
import time
import types

import numpy as np
import torch

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

import vproxy_amd as V  # noqa: E402
from vproxy_amd import workloads as W  # noqa: E402
from vproxy_amd.dist import HitCounterBucket, check_replicated, shard  # noqa: E402

METRIC = "M classifications/sec (ACL+LPM+host) at 1/2/4/8 MI355X; % HBM roofline"
HBM_PEAK_GBS = 8000.0          # MI355X_MICROARCH.md chip table (spec)
HBM_ACHIEVABLE_GBS = 6290.0    # the same table: a float4 copy kernel, measured (79 % of spec)
PROFILES = os.path.join(ROOT, "profiles")
PACKET_SEED = 1234


def log(*a):
    if int(os.environ.get("RANK", "0")) == 0:
        print("[bench]", *a, file=sys.stderr, flush=True)


# ---------------------------------------------------------------------------
# index-addressable synthetic packets (torch, any device)
# ---------------------------------------------------------------------------
_M64 = (1 << 64) - 1


def _s64(c):
    c &= _M64
    return c - (1 << 64) if c >= 1 << 63 else c


_GOLD, _C1, _C2 = _s64(0x9E3779B97F4A7C15), _s64(0xBF58476D1CE4E5B9), _s64(0x94D049BB133111EB)


def _lsr(x, k):
    """logical right shift of an int64 tensor"""
    return (x >> k) & ((1 << (64 - k)) - 1)


def hash_u32(idx, seed, stream):
    """splitmix64 finaliser of (item index, seed, stream) -> uint32 in an
    int64 tensor.  Item i's fields depend on i only, so any slice of the
    global batch can be generated on its own (sharding)."""
    x = idx * _GOLD + _s64(seed * 0x100000001B3 + stream * 0xD6E8FEB86659FD93)
    x = (x ^ _lsr(x, 30)) * _C1
    x = (x ^ _lsr(x, 27)) * _C2
    return (x ^ _lsr(x, 31)) & 0xFFFFFFFF


def below(u, m):
    """uint32 u -> uniform integer in [0, m) (m a python int or int64 tensor < 2^31)"""
    return (u * m) >> 32


def dev_u32(x):
    """int64 tensor holding uint32 values -> int32 tensor with the same bits."""
    x = x & 0xFFFFFFFF
    return torch.where(x >= 2**31, x - 2**32, x).to(torch.int32)


def gen_packets(lo, n, t, pool_n, seed=PACKET_SEED, dev="cpu"):
    """Items [lo, lo + n) of the seeded global packet batch: proto (50/50
    TCP/UDP), src, dst, dport, host id.  Half the packets hit a random ACL
    rule of their protocol (network + port range); 90 % of destinations lie
    inside a random route prefix; host ids are uniform over the pool.
    Returns (proto u8, src i32, dst i32, dport i16, host_id i32) tensors
    (uint32 bits in the signed types)."""
    idx = torch.arange(lo, lo + n, device=dev, dtype=torch.int64)
    h = lambda s: hash_u32(idx, seed, s)
    proto = torch.where((h(1) & 1) == 0, 6, 17).to(torch.uint8)
    src = h(2)
    port = h(3) & 0xFFFF
    pick = (h(4) & 1) == 0
    for p, rules in ((6, t.tcp), (17, t.udp)):
        if len(rules) == 0:
            continue
        ip, mk = W.rule_v4_fields(rules)
        ipd = torch.from_numpy(ip.astype(np.int64)).to(dev)
        mkd = torch.from_numpy(mk.astype(np.int64)).to(dev)
        plo = torch.from_numpy(rules["min_port"].astype(np.int64)).to(dev)
        phi = torch.from_numpy(rules["max_port"].astype(np.int64)).to(dev)
        r = below(h(5 + p), len(rules))
        sel = pick & (proto == p)
        src = torch.where(sel, ipd[r] | (src & (~mkd[r] & 0xFFFFFFFF)), src)
        port = torch.where(sel, plo[r] + below(h(40 + p), phi[r] - plo[r] + 1), port)
        del r, sel
    netd = torch.from_numpy(t.net.astype(np.int64)).to(dev)
    mkd = torch.from_numpy(W._mask32(t.plen).astype(np.int64)).to(dev)
    r = below(h(30), len(t.net))
    dst = h(31)
    dst = torch.where(below(h(32), 10) < 9, netd[r] | (dst & (~mkd[r] & 0xFFFFFFFF)), dst)
    del r
    hid = below(h(33), pool_n)
    return (proto, dev_u32(src), dev_u32(dst), port.to(torch.int32).to(torch.int16),
            hid.to(torch.int32))


def gather_strings_dev(blob, off, idx, dev):
    """Build a device blob of names[idx[i]] (variable length) on the GPU."""
    blob_d = torch.from_numpy(blob.astype(np.uint8)).to(dev)
    off_d = torch.from_numpy(off.astype(np.int64)).to(dev)
    idx_d = torch.from_numpy(idx.astype(np.int64)).to(dev)
    start = off_d[idx_d]
    lens = off_d[idx_d + 1] - start
    out_off = torch.zeros(len(idx) + 1, dtype=torch.int64, device=dev)
    torch.cumsum(lens, 0, out=out_off[1:])
    total = int(out_off[-1])
    seg = torch.repeat_interleave(torch.arange(len(idx), device=dev), lens, output_size=total)
    pos = torch.arange(total, device=dev) - out_off[seg] + start[seg]
    out = blob_d[pos]
    del seg, pos
    return out, out_off.to(torch.int32), total


# ---------------------------------------------------------------------------
# C5 tables (replicated on every rank; also built by tests/test_gpu_c5.py)
# ---------------------------------------------------------------------------
def c5_rule_tables(acl_rules=10000, v4=1_000_000, v6=200_000, groups=100_000):
    """Host-side C5 rule lists (no device): the SecurityGroup lists, the
    route prefixes, the Upstream groups and the hostname source."""
    t = types.SimpleNamespace()
    t.tcp, t.udp = W.gen_sg_rules(acl_rules, W.SEED + 2, p_range=0.3)
    t.net, t.plen = W.gen_v4_prefixes(v4, W.SEED + 3)
    t.hi, t.lo, t.p6 = W.gen_v6_prefixes(v6, W.SEED + 4)
    t.groups, t.ghosts = W.gen_groups(groups, W.SEED + 5)
    names = W.gen_hostnames(t.ghosts, 1 << 20, W.SEED + 6)           # distinct pool source
    t.nblob, t.noff = W.pack(names)
    return t


def c5_tables(clf, dev, pool_n=16 << 20, **kw):
    """Compile the C5 tables into `clf` exactly as the benchmark does and
    build the device hostname pool (same on every rank)."""
    t = c5_rule_tables(**kw)
    a, na, ka = W.as_ctypes(t.tcp, V._lib.VcAclRule)
    b, nb, kb = W.as_ctypes(t.udp, V._lib.VcAclRule)
    V.check(V.lib().vc_compile_acl(clf.h, a, na, b, nb, 0))
    rt = V.RouteTable()
    allnets = np.concatenate([W.v4_nets(t.net, t.plen), W.v6_nets(t.hi, t.lo, t.p6)])
    arr, n_all, keep = W.as_ctypes(allnets, V._lib.VcNet)
    rt.add_rules("bgp", arr, n=n_all)
    clf.compile_route_table(rt)
    a4, t.n4 = rt.rules_raw(4)
    a6, t.n6 = rt.rules_raw(6)
    t.v4_list = np.frombuffer(bytes(a4)[:t.n4 * 40], W.NET_DT)
    t.v6_list = np.frombuffer(bytes(a6)[:t.n6 * 40], W.NET_DT)
    clf.compile_upstream(t.groups)
    t.pool_n = pool_n
    t.pidx = np.random.default_rng(W.SEED + 7).integers(0, len(t.noff) - 1, pool_n)
    t.pool_blob, t.pool_off, t.pool_bytes = gather_strings_dev(t.nblob, t.noff, t.pidx, dev)
    return t


class RawEvent:
    """hipEvent_t through ctypes (torch events cannot be handed to the C ABI)."""
    _hip = None

    def __init__(self):
        if RawEvent._hip is None:
            h = C.CDLL("libamdhip64.so")
            h.hipEventCreate.argtypes = [C.c_void_p]
            h.hipEventRecord.argtypes = [C.c_void_p, C.c_void_p]
            h.hipEventElapsedTime.argtypes = [C.c_void_p, C.c_void_p, C.c_void_p]
            h.hipStreamWaitEvent.argtypes = [C.c_void_p, C.c_void_p, C.c_uint]
            h.hipEventDestroy.argtypes = [C.c_void_p]
            RawEvent._hip = h
        self.h = C.c_void_p()
        assert RawEvent._hip.hipEventCreate(C.byref(self.h)) == 0

    def record(self, stream):
        assert RawEvent._hip.hipEventRecord(self.h, C.c_void_p(stream.cuda_stream)) == 0

    def wait(self, stream):
        """`stream` waits for this event (hipStreamWaitEvent)."""
        assert RawEvent._hip.hipStreamWaitEvent(C.c_void_p(stream.cuda_stream), self.h, 0) == 0

    def elapsed_time(self, other):
        ms = C.c_float()
        assert RawEvent._hip.hipEventElapsedTime(C.byref(ms), self.h, other.h) == 0
        return ms.value


def hip_stream(dev, cus=None):
    """A fresh non-blocking HIP stream wrapped for torch.  HIP spreads the
    streams a process creates round-robin over its hardware queues; three
    created back to back land on three queues, so the kernels on them can
    run concurrently (torch's pooled streams shared a queue here).  `cus`:
    the CU ids the stream may use (hipExtStreamCreateWithCUMask); the
    library sizes its grids to the mask."""
    hip = C.CDLL("libamdhip64.so")
    h = C.c_void_p()
    if cus is None:
        rc = hip.hipStreamCreateWithFlags(C.byref(h), C.c_uint(1))  # hipStreamNonBlocking
    else:
        words = (C.c_uint32 * 32)()
        for cu in cus:
            words[cu // 32] |= 1 << (cu % 32)
        rc = hip.hipExtStreamCreateWithCUMask(C.byref(h), C.c_uint32(32), words)
    assert rc == 0, rc
    return torch.cuda.ExternalStream(h.value, device=dev)


def cu_split(total, k):
    """k CU-mask bits for one stream and the rest for the other, both with
    the same number of CUs on every XCD.  Mask bit i selects a CU of XCD
    i mod 8 (interleaved), and workgroups are dealt to the XCDs round-robin,
    so a mask must give every XCD the same count -- a multiple of 4 -- or a
    share of the workgroups runs a second round (profiles/r03_cu_scaling.jsonl:
    an even spread of ids, every 256/k-th bit, leaves XCDs empty).  The top k
    bits give k/8 CUs per XCD."""
    pick = list(range(total - k, total)) if k > 0 else []
    rest = list(range(total - k))
    return pick, rest


class C5Steps:
    """The C5 step schedule on one rank.

    Step j = hint(j): classify the hostname pool; pipe(j): the fused
    pipeline kernel over this rank's packets (it counts ACL hits and
    route/group buckets; the library finishes the two large counter spaces
    on the counting stream); counters(j): when `bucket`, copy the library's
    three counter arrays into one int64 bucket (device-to-device on the
    counting stream) and all-reduce it (RCCL).  `inflight` batches in
    flight: outputs and pool results have that many buffers, so batch j+1's
    pool pass and pipeline kernel overlap batch j's counter finish.  Every
    step still does all of its work between the caller's synchronisations.
    """

    def __init__(self, clf, t, packets, dev, bucket=False, serial=False, counters="fused",
                 finish="stream", inflight=3, overlap="finish", gate=False, pool_cus=0,
                 pool_stream="pipe"):
        self.clf, self.t, self.dev = clf, t, dev
        self.proto, self.src, self.dst, self.dport, self.hid = packets
        self.B = len(self.src)
        self.serial = serial
        self.count = counters != "none"
        self.fused = counters == "fused"
        self.finish = finish
        self.overlap = overlap
        self.gate = gate
        self.nbuf = 1 if serial else max(1, inflight)
        pool_out = torch.empty(t.pool_n, dtype=torch.int32, device=dev)
        self.pools = [pool_out] + [torch.empty_like(pool_out) for _ in range(self.nbuf - 1)]
        self.outsb = [tuple(torch.empty(self.B, dtype=torch.int32, device=dev)
                            for _ in range(3)) + (None,) for _ in range(self.nbuf)]
        clf.counters_enable(False)
        self.csrc = [clf.counters_device(k)
                     for k in (V.COUNTERS_ACL, V.COUNTERS_ROUTE, V.COUNTERS_GROUP)]
        self.bucket = HitCounterBucket([n for _, n in self.csrc], dev) if bucket else None
        if serial:
            self.s_pipe = self.s_hint = self.s_cnt = torch.cuda.current_stream()
        elif pool_cus > 0:
            # the pool pass and the counter finish on pool_cus CUs, the
            # pipeline kernel on the others
            ncu = torch.cuda.get_device_properties(dev).multi_processor_count
            small, big = cu_split(ncu, pool_cus)
            self.s_pipe = hip_stream(dev, big)
            self.s_hint = hip_stream(dev, small)
            self.s_cnt = hip_stream(dev, small)
        else:
            self.s_pipe, self.s_hint, self.s_cnt = (hip_stream(dev) for _ in range(3))
            if pool_stream == "pipe" and overlap == "finish":
                # in order behind the previous pipeline kernel: no cross-stream
                # event wait between the two kernels of a step
                self.s_hint = self.s_pipe
        self.ev_hint, self.ev_pipe, self.ev_cnt, self.kdone = {}, {}, {}, {}
        self.timing = []
        self.host_ms = {"hint": 0.0, "pipe": 0.0, "counters": 0.0}   # host time issuing

    def _hint(self, j, rec):
        TE = lambda: torch.cuda.Event(enable_timing=True)
        with torch.cuda.stream(self.s_hint):
            if j - self.nbuf in self.ev_pipe:          # pool buffer no longer read
                self.s_hint.wait_event(self.ev_pipe[j - self.nbuf])
            if self.overlap == "finish" and j - 1 in self.kdone:
                self.kdone[j - 1].wait(self.s_hint)     # after the previous pipeline kernel
            e0, e1 = TE(), TE()
            e0.record()
            t = self.t
            V.check(V.lib().vc_hint_search_dev(
                self.clf.h, C.c_void_p(t.pool_blob.data_ptr()), C.c_void_p(t.pool_off.data_ptr()),
                None, None, None, None, None, t.pool_n,
                C.c_void_p(self.pools[j % self.nbuf].data_ptr()),
                C.c_void_p(self.s_hint.cuda_stream)))
            e1.record()
            self.ev_hint[j] = e1
            rec["hint"] = (e0, e1)

    def _pipe(self, j, rec):
        TE = lambda: torch.cuda.Event(enable_timing=True)
        with torch.cuda.stream(self.s_pipe):
            self.s_pipe.wait_event(self.ev_hint[j])
            if j - self.nbuf in self.ev_cnt:           # output buffers counted
                self.s_pipe.wait_event(self.ev_cnt[j - self.nbuf])
            if self.gate and j - 1 in self.ev_cnt:      # the previous batch's finish done
                self.s_pipe.wait_event(self.ev_cnt[j - 1])
            k0, k1 = RawEvent(), RawEvent()            # the classify kernel alone
            k0.record(self.s_pipe)
            if self.fused:                             # count packets only, not the pool pass
                self.clf.counters_enable(True)
            cs = self.s_cnt if (self.fused and self.finish == "stream" and not self.serial) \
                else None
            self.clf.pipeline_v4(self.proto, self.src, self.dst, self.dport, self.hid,
                                 self.pools[j % self.nbuf], outs=self.outsb[j % self.nbuf],
                                 kernel_done_event=k1.h.value, count_stream=cs)
            if self.fused:
                self.clf.counters_enable(False)
            e1 = TE()
            e1.record()
            self.ev_pipe[j] = e1
            self.kdone[j] = k1
            rec["pipe"] = (k0, k1)

    def _counters(self, j, rec):
        outs = self.outsb[j % self.nbuf]
        with torch.cuda.stream(self.s_cnt):
            self.s_cnt.wait_event(self.ev_pipe[j])     # also covers a finish on s_pipe
            k2 = RawEvent()
            k2.record(self.s_cnt)
            if self.count and not self.fused:
                self.clf.counters_add(V.COUNTERS_ACL, outs[0], aux=self.proto)
                self.clf.counters_add(V.COUNTERS_ROUTE, outs[1], family=4)
                self.clf.counters_add(V.COUNTERS_GROUP, outs[2])
            k3 = RawEvent()
            k3.record(self.s_cnt)
            if self.bucket is not None:                # one RCCL all-reduce per batch
                for i, cs in enumerate(self.csrc):
                    self.bucket.fill(i, cs)
                self.bucket.reduce()
            done = torch.cuda.Event()
            done.record()
            self.ev_cnt[j] = done
            rec["count"] = (self.kdone[j], k3)         # kernel end -> counters complete

    def run(self, first, k, timed):
        """Steps first .. first+k-1.  The hostname pool of the next step is
        issued before this step's counters, so it overlaps this step's
        pipeline."""
        if k <= 0:
            return
        recs = [dict() for _ in range(k)]
        T = time.perf_counter
        t = T()
        self._hint(first, recs[0])
        self.host_ms["hint"] += (T() - t) * 1e3
        for i in range(k):
            j = first + i
            t = T()
            self._pipe(j, recs[i])
            self.host_ms["pipe"] += (T() - t) * 1e3
            t = T()
            if i + 1 < k:
                self._hint(j + 1, recs[i + 1])
            self.host_ms["hint"] += (T() - t) * 1e3
            t = T()
            self._counters(j, recs[i])
            self.host_ms["counters"] += (T() - t) * 1e3
        if timed:
            self.timing.extend(recs)

    def reset_events(self):
        self.ev_hint.clear()
        self.ev_pipe.clear()
        self.ev_cnt.clear()
        self.kdone.clear()

    def span(self, key):
        return float(np.mean([r[key][0].elapsed_time(r[key][1]) for r in self.timing]))


# ---------------------------------------------------------------------------
# rank launcher: `python bench.py --gpus N` without torch.distributed.run
# ---------------------------------------------------------------------------
def _free_port():
    import socket
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def launch_ranks(n, argv, script=None, env=None, poll_s=0.2, grace_s=20.0):
    """Run `script argv` as n rank processes (RANK = LOCAL_RANK = 0..n-1,
    WORLD_SIZE = n, MASTER_ADDR 127.0.0.1 and one MASTER_PORT), the layout
    torch.distributed.run gives them.  Children, never exec: the caller must
    not have touched the GPU (this process only counts devices).  Rank 0's
    stdout is inherited, so its JSON line is the job's.  Returns 0 when every
    rank exits 0; otherwise the first failing rank's status (128 + signal for
    a signal), after terminating the ranks still running -- a rank waiting
    in a collective for a dead peer would otherwise hang the job."""
    import signal
    import subprocess
    base = dict(os.environ if env is None else env)
    base.setdefault("MASTER_ADDR", "127.0.0.1")
    if "MASTER_PORT" not in base:
        base["MASTER_PORT"] = str(_free_port())
    procs = []

    def stop_all(sig=signal.SIGTERM):
        for p in procs:
            if p.poll() is None:
                try:
                    p.send_signal(sig)
                except ProcessLookupError:
                    pass

    def on_signal(signum, frame):          # the driver's time limit: pass it on
        stop_all(signum)
        raise SystemExit(128 + signum)

    old = {s: signal.signal(s, on_signal) for s in (signal.SIGTERM, signal.SIGINT)}
    try:
        for r in range(n):
            e = dict(base, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(n),
                     LOCAL_WORLD_SIZE=str(n), GROUP_RANK="0")
            procs.append(subprocess.Popen([sys.executable, "-u", script or __file__] + list(argv),
                                          env=e))
        rc = 0
        while True:
            codes = [p.poll() for p in procs]
            bad = [c for c in codes if c not in (None, 0)]
            if bad:
                c = bad[0]
                rc = 128 - c if c < 0 else c
                stop_all()
                t0 = time.time()
                while any(p.poll() is None for p in procs) and time.time() - t0 < grace_s:
                    time.sleep(poll_s)
                stop_all(signal.SIGKILL)
                for p in procs:
                    p.wait()
                break
            if all(c == 0 for c in codes):
                break
            time.sleep(poll_s)
        return rc
    finally:
        for s, h in old.items():
            signal.signal(s, h)


def visible_gpus(environ=None, topology="/sys/class/kfd/kfd/topology/nodes", dri="/dev/dri"):
    """The GPUs this process's ranks could use, counted without any HIP or
    HSA call (the parent of the ranks must not initialise the GPU: it
    spawns them, and on ROCm torch.cuda.device_count() falls back to
    hipGetDeviceCount when its amdsmi count fails): KFD topology nodes with
    a non-zero gfx_target_version whose render node /dev/dri/renderD<minor>
    exists (a container sees the host's nodes but only its own devices; the
    GPU box hides the other nodes' properties), then the ROCR_VISIBLE_DEVICES,
    HIP_VISIBLE_DEVICES and CUDA_VISIBLE_DEVICES lists in that order, each
    cut at its first entry that names no device.  0 without KFD."""
    environ = os.environ if environ is None else environ
    n = 0
    try:
        nodes = sorted(os.listdir(topology))
    except OSError:
        nodes = []
    for d in nodes:
        try:
            with open(os.path.join(topology, d, "properties")) as f:
                props = dict(l.split()[:2] for l in f if len(l.split()) >= 2)
        except (OSError, ValueError):
            continue
        if int(props.get("gfx_target_version", "0")) == 0:
            continue                                    # a CPU node
        minor = props.get("drm_render_minor")
        if minor is not None and os.path.exists(os.path.join(dri, "renderD%s" % minor)):
            n += 1
    for var in ("ROCR_VISIBLE_DEVICES", "HIP_VISIBLE_DEVICES", "CUDA_VISIBLE_DEVICES"):
        v = environ.get(var)
        if v is None:
            continue
        k = 0
        for x in (t.strip() for t in v.split(",")):
            if not ((x.isdigit() and int(x) < n) or x.startswith("GPU-")):
                break
            k += 1
        n = min(n, k)
    return n


def resolve_world(gpus, environ=None, shared=False, device_count=None):
    """What `--gpus N` means for this process: ("run", world) when it is one
    rank of a launched job (WORLD_SIZE set, and equal to N) or N == 1;
    ("launch", N) when N > 1 and nothing launched it (bench.py spawns the N
    ranks itself).  Raises SystemExit(2) when WORLD_SIZE disagrees with
    --gpus, or when N ranks need more GPUs than the node shows -- never a
    silent one-GPU run labelled N."""
    environ = os.environ if environ is None else environ
    ws = environ.get("WORLD_SIZE")
    if gpus < 1:
        raise SystemExit("bench.py: --gpus must be >= 1 (got %d)" % gpus)
    if ws is not None and ws != "":
        if int(ws) != gpus:
            print("bench.py: --gpus %d but WORLD_SIZE=%s: the launcher and the flag disagree"
                  % (gpus, ws), file=sys.stderr)
            raise SystemExit(2)
        return "run", gpus
    if gpus == 1:
        return "run", 1
    if not shared:
        if device_count is None:
            device_count = visible_gpus(environ)         # no HIP call in the ranks' parent
        if device_count < gpus:
            print("bench.py: --gpus %d but %d GPU(s) visible" % (gpus, device_count),
                  file=sys.stderr)
            raise SystemExit(2)
    return "launch", gpus


def copy_bandwidth(dev, nbytes=1 << 30, reps=5):
    """torch's device-to-device copy rate on this GPU (read + written bytes
    over the copy's time, best of `reps` after one warmup) with 1 GiB
    tensors, far past the 256 MB Infinity Cache -- printed beside the
    guide's float4-copy figure (HBM_ACHIEVABLE_GBS) that the roofline is
    also quoted against."""
    a = torch.ones(nbytes // 4, dtype=torch.int32, device=dev)
    b = torch.empty_like(a)
    b.copy_(a)
    torch.cuda.synchronize()
    best = None
    for _ in range(reps):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        b.copy_(a)
        e1.record()
        e1.synchronize()
        ms = e0.elapsed_time(e1)
        best = ms if best is None else min(best, ms)
    del a, b
    return 2.0 * nbytes / (best / 1e3) / 1e9


def max_over_ranks(x, dev):
    """MAX of a float over the process group (the step time the job sees)."""
    import torch.distributed as dist
    t = torch.tensor([x], dtype=torch.float64, device=dev)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())


# ---------------------------------------------------------------------------
# CPU baseline (oracle, test-infrastructure C restatement of the Java scans)
# ---------------------------------------------------------------------------
def cpu_info():
    model = None
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    model = line.split(":", 1)[1].strip()
                    break
    except OSError:
        pass
    try:
        avail = len(os.sched_getaffinity(0))
    except AttributeError:
        avail = os.cpu_count() or 1
    quota = cgroup_cpu_max()
    # all host cores this process may use: the affinity
    # set, or the cgroup CPU quota when that is smaller -- threads past the
    # quota only take turns (on the GPU box 256 threads under a 16-CPU quota
    # ran the C5 sample at half the 16-thread rate).  The affinity-wide rate
    # is reported beside it (cpu_rates: `affinity_all`).
    share = avail
    if quota[1]:
        share = max(1, min(avail, int(quota[1])))
    return {"nproc": os.cpu_count(), "affinity": avail, "cpu_model": model,
            "cgroup_cpu_max": quota[0], "quota_cpus": quota[1],
            "threads_all": share}


def cgroup_cpu_max(path="/sys/fs/cgroup/cpu.max"):
    """(raw `cpu.max` text, CPUs it allows or None when unlimited/absent):
    cgroup v2 "quota period", e.g. "1600000 100000" = 16 CPUs."""
    try:
        with open(path) as f:
            raw = f.read().strip()
    except OSError:
        return None, None
    parts = raw.split()
    if len(parts) == 2 and parts[0] != "max":
        try:
            return raw, round(int(parts[0]) / int(parts[1]), 2)
        except ValueError:
            pass
    return raw, None


def cpu_rates(run, unit, budget_s, what, note=None, cap=None):
    """Time `run(n, threads) -> seconds` on a bounded sample: all-core (the
    box's CPU share) and 1 core, each sized to about `budget_s` seconds and
    at most `cap` items (the sample the caller holds)."""
    info = cpu_info()
    res = {}
    legs = [info["threads_all"], 1]
    if info["affinity"] > info["threads_all"]:
        legs.append(info["affinity"])
    for threads in legs:
        # grow the sample until it runs at least half the budget (a short
        # probe is dominated by thread start-up), or reaches the cap
        n = max(threads * 4, 64)
        while True:
            t = run(n, threads)
            if t >= 0.5 * budget_s or (cap and n >= cap):
                break
            n = int(min(n * 16, max(2 * n, n * budget_s / max(t, 1e-6))))
            if cap:
                n = min(n, cap)
        res[threads] = (n, t)
    na, ta = res[info["threads_all"]]
    n1, t1 = res[1]
    out = {"value": na / ta / 1e6, "unit": unit, "cores": info["threads_all"], "kind": "port",
           "sample": "%s; all-core: %d items in %.1f s on %d threads; 1 core: %d items in %.1f s"
                     % (what, na, ta, info["threads_all"], n1, t1),
           "one_core": {"value": n1 / t1 / 1e6, "cores": 1},
           "nproc": info["nproc"], "affinity": info["affinity"],
           "cgroup_cpu_max": info["cgroup_cpu_max"], "quota_cpus": info["quota_cpus"],
           "cpu_model": info["cpu_model"]}
    if info["affinity"] > info["threads_all"]:
        nx, tx = res[info["affinity"]]
        out["affinity_all"] = {"value": nx / tx / 1e6, "cores": info["affinity"],
                               "sample": "%d items in %.1f s" % (nx, tx)}
    if note:
        out["note"] = note
    return out


def end_to_end(fn, items, reps=3):
    """M items/s of a synchronous host-buffer call (H2D + kernels + D2H).
    VC_BENCH_NO_E2E=1 skips it (profiling passes: its chunked launches would
    mix into the per-launch averages of the device kernel)."""
    if os.environ.get("VC_BENCH_NO_E2E") == "1":
        return None
    fn()
    t0 = time.perf_counter()
    for _ in range(reps):
        fn()
    return round(items * reps / (time.perf_counter() - t0) / 1e6, 1)


def sample_blob(blob, off, idx):
    """Host blob + uint32 offsets of strings[idx] (a CPU-baseline sample)."""
    b, o, _ = gather_strings_dev(blob, off, np.asarray(idx), "cpu")
    return b.numpy(), o.numpy().view(np.uint32)


def _oracle():
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    import oracle_ffi as O
    return O


def cpu_baseline_c5(t, budget_s=8.0):
    O = _oracle()
    og = O.Groups(t.groups)
    names_blob, names_off = t.nblob, t.noff

    def run(n, threads):
        proto, src, dst, dport, hid = (x.numpy() for x in gen_packets(0, n, t, t.pool_n))
        src, dst = src.view(np.uint32), dst.view(np.uint32)
        dport = dport.view(np.uint16)
        names = [bytes(names_blob[names_off[i]:names_off[i + 1]]) for i in t.pidx[hid]]
        sub_blob, sub_off = W.pack(names)
        t0 = time.perf_counter()
        O.sg_batch_v4_np(t.tcp, t.udp, False, proto, src, dport, nthreads=threads)
        O.rt_batch_v4_np(t.v4_list, dst, nthreads=threads)
        O.hint_batch_np(og, sub_blob, sub_off, None, nthreads=threads)
        return time.perf_counter() - t0

    return cpu_rates(run, "M classifications/s", budget_s,
                     "the first packets of the same seeded C5 batch (ACL %d rules + RouteTable "
                     "%d IPv4 rules + Upstream %d groups), oracle linear scans as the Java code "
                     "does them" % (len(t.tcp) + len(t.udp), len(t.v4_list), len(t.groups)),
                     note="the CPU leg runs Upstream.searchForGroup for every packet, as the "
                          "Java path does per connection; the GPU classifies each hostname of "
                          "the 16M pool once per step and gathers the result per packet. The "
                          "restatement skips Java's per-call allocations, so it is faster than "
                          "the reference itself.")


def gather_ceiling(table_mb=64):
    """Measured random 4-byte gather rate (G gathers/s) from a table of
    `table_mb`, two independent gathers per item (tools/gather_probe.hip,
    profiles/r01_gather_probe.csv): the ceiling of the pipeline kernel,
    whose route-root and pool tables are 64 MB each."""
    import csv
    try:
        with open(os.path.join(PROFILES, "r01_gather_probe.csv")) as f:
            rows = [r for r in csv.DictReader(f) if int(r["table_MB"]) == table_mb and
                    int(r["gathers_per_item"]) == 2]
        return max(float(r["G_gathers_per_s"]) for r in rows) if rows else None
    except (OSError, ValueError, KeyError):
        return None


def fabric_ceiling():
    """Measured L2-to-fabric request rate of the two-gather probe over 64 MB
    tables (the pipeline's access pattern): the requests of that launch
    counted by the PMC method of scripts/pmc_traffic.py (FETCH_SIZE / 64 B +
    WRITE_SIZE / 64 B, profiles/r03_fetch_calibration.json launch 2) over its
    time (profiles/r01_gather_probe.csv: 64 MB, 2 gathers, 4 items per lane,
    4 workgroups per CU), in G requests/s."""
    import csv
    try:
        with open(os.path.join(PROFILES, "r03_fetch_calibration.json")) as f:
            cal = json.load(f)
        l = [x for x in cal["launches"] if x["table_bytes"] == 64 << 20 and
             x["gathers_per_item"] == 2][0]
        req = (l["fetch_bytes"] + l["write_bytes"]) / 64
        with open(os.path.join(PROFILES, "r01_gather_probe.csv")) as f:
            ms = [float(r["ms"]) for r in csv.DictReader(f) if int(r["table_MB"]) == 64 and
                  int(r["gathers_per_item"]) == 2 and int(r["items_per_lane"]) == 4 and
                  int(r["blocks_per_cu"]) == 4][0]
        return req / (ms * 1e-3) / 1e9
    except (OSError, ValueError, KeyError, IndexError):
        return None


def load_step_requests(workload):
    """L2-to-fabric requests of one whole step (profiles/pmc_traffic.json
    `step`, scripts/pmc_traffic.py --per-step) and the commit they were
    taken at."""
    try:
        with open(os.path.join(PROFILES, "pmc_traffic.json")) as f:
            d = json.load(f)[workload]
        return d["step"]["requests"], d.get("commit")
    except (OSError, ValueError, KeyError):
        return None, None


def load_traffic(workload, kernel):
    """Per-launch HBM-side bytes of `kernel` from the committed PMC passes
    (profiles/pmc_traffic.json, written by scripts/pmc_traffic.py from
    separate rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE runs of this bench),
    and the commit the passes were taken at."""
    p = os.path.join(PROFILES, "pmc_traffic.json")
    try:
        with open(p) as f:
            d = json.load(f)
        w = d[workload]
        return w["kernels"][kernel]["traffic_bytes"], w.get("commit")
    except (OSError, ValueError, KeyError):
        return None, None


# ---------------------------------------------------------------------------
def build_parser():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--workload", default="c5",
                    choices=["c5", "c1", "c2", "c2host", "c3", "c4", "c4uri", "dns", "dnsd", "sni", "http",
                             "parse", "switch", "source", "mirror", "mirroritems", "mix",
                             "mixhost"])
    ap.add_argument("--packets", type=int, default=125_000_000, help="per GPU per step (c5)")
    ap.add_argument("--pool", type=int, default=16 << 20, help="hostname pool (c5/c4)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--counters", choices=["fused", "passes", "none"], default="fused",
                    help="fused: the pipeline kernel counts ACL hits and route/group buckets "
                         "itself and the library finishes the large spaces; passes: separate "
                         "counting passes over the outputs (counters_add); none: ablation")
    ap.add_argument("--finish", choices=["stream", "inline"], default="stream",
                    help="where the library's counter finish runs: on the counting stream "
                         "(overlapping the next batch) or inline after the pipeline kernel")
    ap.add_argument("--serial", action="store_true",
                    help="ablation: one stream, no overlap between consecutive batches")
    ap.add_argument("--overlap", choices=["finish", "pipeline"], default="finish",
                    help="what the next batch's hostname-pool pass runs beside: this batch's "
                         "counter finish (it waits for this batch's pipeline kernel, which then "
                         "runs alone) or the pipeline kernel itself")
    ap.add_argument("--gate", action="store_true",
                    help="the pipeline kernel also waits for the previous batch's counter "
                         "finish (which then overlaps only the pool pass)")
    ap.add_argument("--inflight", type=int, default=3,
                    help="batches in flight (output and pool buffers)")
    ap.add_argument("--pool-stream", choices=["own", "pipe"], default="pipe",
                    help="the pool pass in order on the pipeline stream (default: no "
                         "cross-stream event wait between a step's two kernels; 6.076 against "
                         "6.115 ms, profiles/r04_ab_pool_stream.jsonl) or on its own stream")
    ap.add_argument("--pool-cus", type=int, default=0,
                    help="CU partition: the pool pass and the counter finish on this many CUs "
                         "(a CU-masked stream), the pipeline kernel on the rest (0: no masks)")
    ap.add_argument("--compact6", action="store_true",
                    help="mix / mixhost: IPv6 addresses as one row per IPv6 packet "
                         "(vc_pipeline_c6_dev / vc_pipeline_c6)")
    ap.add_argument("--v6-frac", type=float, default=0.15,
                    help="mix / mixhost: share of IPv6 packets (C3's mix is 0.15)")
    ap.add_argument("--dist", action="store_true",
                    help="use the process group and the counter all-reduce even at N = 1")
    return ap


def make_c5_steps(clf, t, packets, dev, args, bucket):
    """The C5 schedule exactly as main() times it (also run, at the timed
    size, by tests/test_gpu_c5.py::test_c5_timed_launch_exact)."""
    return C5Steps(clf, t, packets, dev, bucket=bucket, serial=args.serial,
                   counters=args.counters, finish=args.finish, inflight=args.inflight,
                   overlap=args.overlap, gate=args.gate, pool_cus=args.pool_cus,
                   pool_stream=args.pool_stream)


def main():
    args = build_parser().parse_args()

    # VC_BENCH_SHARED_GPU=1: rehearsal of the multi-rank path on a one-GPU
    # box -- every rank on cuda:0 and gloo for the collectives (RCCL refuses
    # two ranks on one device).  The timing is then not a scaling result.
    shared = os.environ.get("VC_BENCH_SHARED_GPU") == "1"
    mode, world = resolve_world(args.gpus, shared=shared)
    if mode == "launch":
        # `python bench.py --gpus N` with no launcher: spawn the N ranks here
        # (nothing above touched the GPU) and exit with their status
        log("launching %d ranks (no WORLD_SIZE in the environment)" % world)
        sys.exit(launch_ranks(world, sys.argv[1:]))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if shared:
        local = 0
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    use_dist = world > 1 or args.dist
    if use_dist:
        import torch.distributed as dist
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        os.environ.setdefault("MASTER_PORT", "29517")
        os.environ.setdefault("RANK", "0")
        os.environ.setdefault("WORLD_SIZE", "1")
        if shared:
            dist.init_process_group("gloo")
        else:
            dist.init_process_group("nccl", device_id=dev)
    clf = V.Classifier(local)

    if args.workload != "c5":
        return sub_bench(args, clf, dev, rank, world)

    t_setup = time.time()
    t = c5_tables(clf, dev, args.pool)
    log("tables built in %.1fs (acl %d+%d, routes %d+%d, groups %d, pool %d names %.0f MB)" % (
        time.time() - t_setup, len(t.tcp), len(t.udp), t.n4, t.n6, len(t.groups), args.pool,
        t.pool_bytes / 1e6))
    if use_dist:
        # summed hit counters need identical tables on every rank
        rows = check_replicated([clf.table_digest(k) for k in
                                 (V.COUNTERS_ACL, V.COUNTERS_ROUTE, V.COUNTERS_GROUP)])
        log("tables replicated: %d ranks, digests %s" % (len(rows), ["%016x" % d for d in rows[0]]))
    # this rank's shard of the global batch (weak scaling: N = packets x world)
    lo, hi = shard(args.packets * world, rank, world)
    packets = gen_packets(lo, hi - lo, t, t.pool_n, dev=dev)
    steps = make_c5_steps(clf, t, packets, dev, args, bucket=use_dist)
    torch.cuda.synchronize()
    log("packets generated (%d of %d, shard [%d, %d)), setup %.1fs" % (
        hi - lo, args.packets * world, lo, hi, time.time() - t_setup))

    steps.run(0, args.warmup, False)
    torch.cuda.synchronize()
    steps.reset_events()
    if use_dist:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    steps.run(args.warmup, args.steps, True)
    torch.cuda.synchronize()
    if use_dist:
        dist.barrier()
    torch.cuda.synchronize()
    elapsed = time.perf_counter() - t0
    if use_dist:
        elapsed = max_over_ranks(elapsed, dev)

    hint_ms, pipe_ms, count_ms = steps.span("hint"), steps.span("pipe"), steps.span("count")
    log("host ms issuing over %d steps: %s" % (args.warmup + args.steps, {
        k: round(v, 2) for k, v in steps.host_ms.items()}))
    B = hi - lo
    total = float(args.packets) * world * args.steps
    value = total / elapsed / 1e6
    # roofline of the dominant kernel, algorithmic bytes only
    if pipe_ms >= hint_ms:
        dom, per_unit, units, ms = "pipeline_v4_kernel", 27, B, pipe_ms
        unit_desc = "27 B/packet (proto 1 + src 4 + dst 4 + dport 2 + host_id 4 in; 3x int32 out)"
    else:
        dom, ms, units = "hint_kernel", hint_ms, args.pool
        per_unit = (t.pool_bytes / args.pool) + 4 + 4
        unit_desc = "%.1f B/hostname (avg bytes + 4 offset + 4 out)" % per_unit
    achieved = per_unit * units / (ms / 1e3) / 1e9
    ceil = gather_ceiling()
    g_rate = 2.0 * B / (pipe_ms / 1e3) / 1e9
    gather_bound = {"kernel": "pipeline_v4_kernel",
                    "per_packet": "2 random 4-byte gathers (route root 64 MB, pool 64 MB)",
                    "achieved_G_gathers_per_s": round(g_rate, 2),
                    "ceiling_G_gathers_per_s": ceil,
                    "frac": round(g_rate / ceil, 4) if ceil else None,
                    "ceiling_source": "tools/gather_probe.hip -> profiles/r01_gather_probe.csv"}
    traffic, t_commit = load_traffic("c5", dom)
    step_req, r_commit = load_step_requests("c5")
    fab_ceil = fabric_ceiling()
    step_ms = elapsed / args.steps * 1e3
    fabric = None
    if step_req:
        fabric = {"requests_per_step": round(step_req),
                  "achieved_G_requests_per_s": round(step_req / (step_ms / 1e3) / 1e9, 2),
                  "ceiling_G_requests_per_s": round(fab_ceil, 2) if fab_ceil else None,
                  "frac": round(step_req / (step_ms / 1e3) / 1e9 / fab_ceil, 4)
                  if fab_ceil else None,
                  "what": "every kernel of one step (pipeline, pool pass, counter finish): L2 "
                          "read + write requests to the fabric (FETCH_SIZE / 64 B + "
                          "WRITE_SIZE / 64 B per launch, rocprofv3 --pmc at commit %s) over "
                          "this run's ms_per_step, against the rate the two-gather probe over "
                          "64 MB tables reaches (tools/gather_probe.hip; the cap sits past the "
                          "CUs, tools/gather_paths.hip)" % r_commit}
    copy_gbs = copy_bandwidth(dev)
    traffic_gbs = traffic / (ms / 1e3) / 1e9 if traffic else None
    roof = {"bound": "hbm", "achieved": round(achieved, 2), "peak": HBM_PEAK_GBS, "unit": "GB/s",
            "frac": round(achieved / HBM_PEAK_GBS, 5), "traffic": traffic,
            # SURVEY.md §8(d)'s second number: the measured (PMC) bytes of the
            # kernel over its time, against the spec and this GPU's copy rate
            "traffic_GBps": round(traffic_gbs, 1) if traffic_gbs else None,
            "traffic_frac": round(traffic_gbs / HBM_PEAK_GBS, 4) if traffic_gbs else None,
            "achievable_GBps": HBM_ACHIEVABLE_GBS,
            "frac_of_achievable": round(achieved / HBM_ACHIEVABLE_GBS, 5),
            "traffic_frac_of_achievable": round(traffic_gbs / HBM_ACHIEVABLE_GBS, 4)
            if traffic_gbs else None,
            "torch_copy_GBps": round(copy_gbs, 1),
            "traffic_source": "profiles/pmc_traffic.json: rocprofv3 --pmc FETCH_SIZE + the "
                              "wide streamed reads' uncounted half (15 B/packet) + WRITE_SIZE "
                              "per launch, taken at commit %s; random-gather misses are "
                              "counted whole (profiles/r03_fetch_calibration.json)" % t_commit,
            "kernel": dom, "kernel_ms": round(ms, 4), "algorithmic_bytes": unit_desc,
            "gather_bound": gather_bound,
            "fabric_bound": fabric,
            "other_kernel_ms": {"hint_kernel": round(hint_ms, 4),
                                "pipeline_v4_kernel": round(pipe_ms, 4),
                                "kernel_end_to_counters_done": round(count_ms, 4),
                                "counting": ("in the pipeline kernel (ACL + route/group "
                                             "buckets) + library finish passes on the %s" %
                                             ("counting stream" if args.finish == "stream"
                                              else "pipeline stream")
                                             if steps.fused else args.counters)}}
    cpu = None
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        cpu = cpu_baseline_c5(t)
    if rank == 0:
        line = {"metric": METRIC, "value": round(value, 3), "unit": "M classifications/s",
                "n_gpus": world, "steps": args.steps, "warmup": args.warmup,
                "ms_per_step": round(elapsed / args.steps * 1e3, 3), "higher_is_better": True,
                "scaling": "weak", "vs_baseline": None, "dtype": "u32",
                "data": "synthetic (seeded, generated on device)",
                "config": {"workload": "C5 combined ACL->route->host pipeline, per-GPU shard of "
                                       "a seeded global batch",
                           "shard": ("weak scaling: every GPU classifies %d packets per step, "
                                     "so N = 1 runs one GPU's 125M shard of C5's 1B-packet batch "
                                     "(N = 8 classifies the whole 1B)" % args.packets
                                     if args.packets == 125_000_000 else
                                     "weak scaling: %d packets per GPU per step" % args.packets),
                           "acl_rules": int(len(t.tcp) + len(t.udp)), "routes_v4": int(t.n4),
                           "routes_v6": int(t.n6), "groups": len(t.groups),
                           "hostname_pool": args.pool, "packets_per_gpu_per_step": args.packets,
                           "global_batch": args.packets * world,
                           "parallelism": "dp%d" % world,
                           "schedule": ("serial, one stream" if args.serial else
                                        "%d batches in flight: pool pass, pipeline and counter "
                                        "finish on HIP streams (the counter finish on its own), "
                                        "next pool pass beside the %s" % (
                                            args.inflight, "counter finish" if
                                            args.overlap == "finish" else "pipeline kernel") +
                                        (", pool pass and finish on %d CUs, pipeline on the "
                                         "rest" % args.pool_cus if args.pool_cus else "") +
                                        (", pool pass in order on the pipeline stream"
                                         if args.pool_stream == "pipe" and not args.pool_cus
                                         and args.overlap == "finish" else ""))},
                "roofline": roof, "cpu_baseline": cpu}
        print(json.dumps(line), flush=True)
    clf.close()
    if use_dist:
        dist.destroy_process_group()


# ---------------------------------------------------------------------------
# sub-benchmarks (DESIGN.md / BASELINE.md numbers, not the headline)
# ---------------------------------------------------------------------------
def replicas(res, world, dev):
    """A sub-bench at N > 1: every rank runs the same workload on its own GPU
    (replicas: the classifiers share nothing, so there is no collective in
    the timed work); the line reports the slowest rank's times and the items
    all N ranks classified.  Every rank must call it (max-over-ranks)."""
    res["n_gpus"] = world
    if world > 1:
        ms = max_over_ranks(res["kernel_ms"], dev)
        res["kernel_ms"] = round(ms, 4)
        res["ms_per_step"] = round(max_over_ranks(res["ms_per_step"], dev), 3)
        res["items_per_gpu"] = res["items"]
        res["items"] = res["items"] * world
        res["M_items_per_s"] = round(res["items"] / (ms / 1e3) / 1e6, 1)
        res["scaling"] = "weak (replicas)"


def _time(fn, steps, warmup):
    for _ in range(warmup):
        fn()
    torch.cuda.synchronize()
    ev = []
    t0 = time.perf_counter()
    for _ in range(steps):
        e0 = torch.cuda.Event(enable_timing=True)
        e1 = torch.cuda.Event(enable_timing=True)
        e0.record()
        fn()
        e1.record()
        ev.append((e0, e1))
    torch.cuda.synchronize()
    el = time.perf_counter() - t0
    return el, float(np.mean([a.elapsed_time(b) for a, b in ev]))


def hosts_text(n=50_000):
    """The DNS workloads' hosts file: n lines "10.0.x.y hN.hosts.local"."""
    return "\n".join("10.0.%d.%d h%d.hosts.local" % (i >> 8 & 255, i & 255, i) for i in range(n))


def c4_workload(dns, n=16 << 20):
    """The `c4` / `dns` sub-benches' inputs (also checked whole by
    tests/test_gpu_c5.py): 100k hint-host groups, the 50k-line hosts file
    (dns), 1M distinct hostnames (DNS-flavoured with trailing dots for dns)
    and the n seeded draws from them that form the batch."""
    groups, ghosts = W.gen_groups(100_000, W.SEED + 5)
    if dns:
        names = W.gen_hostnames(ghosts, 1 << 20, W.SEED + 6, dns=True, port_frac=0)
    else:
        names = W.gen_hostnames(ghosts, 1 << 20, W.SEED + 6)
    pidx = np.random.default_rng(W.SEED + (8 if dns else 7)).integers(0, len(names), n)
    return groups, hosts_text() if dns else None, names, pidx


URI_PATHS = ["/", "/api", "/api/v1", "/api/v1/users", "/api/v2", "/static", "/static/img",
             "/static/img/a.png", "*", "/login", "/a/b/c/d/e/f"]
URI_TAILS = ["", "/", "/x", "?q=1", "/?q=2", "/users/7"]


def c4uri_workload(n=16 << 20, n_groups=100_000, n_names=1 << 20, seed_off=0):
    """The `c4uri` sub-bench's inputs (also checked whole by
    tests/test_gpu_c4uri.py): the hint the L7 callers send,
    Hint.ofHostUri(Host, uri) with port 0 (HttpContext.java:63-69,
    httpbin/Stream.java:50), scored by the whole Hint.matchLevel
    (Hint.java:100-160).  The C4 groups with a fifth carrying a hint-uri and
    200 uri-only groups (the generator of test_hint_uri_levels_at_scale), the
    n_groups / 20 path-routed groups (an earlier group's hint-host with a
    hint-uri), the C4 hostnames (n_names distinct, 10 % with ':port'), the
    66 uris of
    URI_PATHS x URI_TAILS; n seeded (name, uri) draws, 80 % with a uri.
    -> groups, names, uris, name index per hint, uri index per hint (-1 =
    null uri)."""
    groups, ghosts = W.gen_groups(n_groups, W.SEED + 5 + seed_off)
    rng = np.random.default_rng(81 + seed_off)
    for i in np.nonzero(rng.random(len(groups)) < 0.2)[0]:
        groups[i][1]["uri"] = URI_PATHS[int(rng.integers(0, len(URI_PATHS)))]
    groups += [({}, {"uri": URI_PATHS[k % len(URI_PATHS)] +
                     ("/u%d" % k if k > len(URI_PATHS) else "")}) for k in range(200)]
    # path-routed backends: n_groups / 20 more groups sharing the hint-host
    # of an earlier group, each with a hint-uri, so that for their hosts the
    # uri level picks the group
    for h in rng.integers(0, len(ghosts), n_groups // 20):
        groups.append(({}, {"host": ghosts[int(h)],
                            "uri": URI_PATHS[int(rng.integers(0, len(URI_PATHS)))]}))
    names = W.gen_hostnames(ghosts, n_names, W.SEED + 6 + seed_off)
    uris = [(p + t).encode() for p in URI_PATHS for t in URI_TAILS]
    r = np.random.default_rng(W.SEED + 24 + seed_off)
    nidx = r.integers(0, len(names), n)
    uidx = np.where(r.random(n) < 0.8, r.integers(0, len(uris), n), -1)
    return groups, names, uris, nidx, uidx


def c4uri_batch(names, uris, nidx, uidx, dev):
    """The c4uri batch on the device: host blob + offsets, uri blob +
    offsets and the null-uri flags, in the layout vc_hint_search_dev takes."""
    nblob, noff = W.pack(names)
    ublob, uoff = W.pack(uris)
    hb, ho, hbytes = gather_strings_dev(nblob, noff, nidx, dev)
    ub, uo, ubytes = gather_strings_dev(ublob, uoff, np.maximum(uidx, 0), dev)
    un = torch.from_numpy((uidx < 0).astype(np.uint8)).to(dev)
    return hb, ho, ub, uo, un, hbytes + ubytes


def http_workload(n=8 << 20, n_templates=1 << 18):
    """The `http` sub-bench's inputs (also checked whole by
    tests/test_gpu_http.py): the C4 groups, a fifth of them with a hint-uri;
    n_templates seeded HTTP/1 request heads (request line with a path and
    query, Host with 'www.' / ':port' forms on some, user agent, accept,
    optional cookie) and the n seeded draws from them that form the batch."""
    groups, ghosts = W.gen_groups(100_000, W.SEED + 5)
    paths = ["/", "/api", "/api/v1", "/api/v1/users", "/api/v2", "/static", "/static/img",
             "/static/img/a.png", "*", "/login", "/a/b/c/d/e/f"]
    rng = np.random.default_rng(W.SEED + 20)
    for i in np.nonzero(rng.random(len(groups)) < 0.2)[0]:
        groups[i][1]["uri"] = paths[int(rng.integers(0, len(paths)))]
    names = W.gen_hostnames(ghosts, n_templates, W.SEED + 21, port_frac=0.1)
    tails = ["", "/", "/x", "?q=1", "/?q=2", "/users/7", "/index.html?a=1&b=2"]
    agents = [b"curl/8.5.0", b"Mozilla/5.0 (X11; Linux x86_64; rv:128.0) Gecko/20100101 Firefox/128.0",
              b"python-requests/2.32.3", b"Go-http-client/1.1"]
    heads = []
    for k in range(n_templates):
        path = paths[int(rng.integers(0, len(paths)))] + tails[int(rng.integers(0, len(tails)))]
        h = [b"GET " + path.encode() + b" HTTP/1.1", b"Host: " + names[k],
             b"User-Agent: " + agents[int(rng.integers(0, len(agents)))], b"Accept: */*"]
        if rng.random() < 0.3:
            h.append(b"Cookie: sid=%016x" % int(rng.integers(0, 2**62)))
        heads.append(b"\r\n".join(h) + b"\r\n\r\n")
    pidx = np.random.default_rng(W.SEED + 22).integers(0, n_templates, n)
    return groups, heads, pidx


def frames_workload(n=32 << 20):
    """The frame sub-benches' inputs (`parse`, `switch`, `mirror`; also
    checked whole by tests/test_gpu_frames_scale.py): 64K seeded VXLAN
    frames and the n seeded draws from them that form the batch."""
    frames = W.gen_vxlan_frames(1 << 16, W.SEED + 12)
    pidx = np.random.default_rng(W.SEED + 13).integers(0, len(frames), n)
    return frames, pidx


def switch_senders(n, dev):
    """The `switch` sub-bench's datagram senders: n uniform IPv4 addresses."""
    g = torch.Generator(device=dev)
    g.manual_seed(19)
    return dev_u32(torch.randint(0, 2**32, (n,), generator=g, device=dev))


def compile_switch_acl(clf, t):
    """The `switch` sub-bench's bareVXLanAccess: the C5 SecurityGroup with a
    last UDP rule 0.0.0.0/0 port 4789 allow, so the senders no earlier rule
    decides reach the parse's inner route (with defaultAllow false alone the
    bench's uniform senders were nearly all denied).  Compiled into clf;
    returns the (tcp, udp) lists."""
    last = np.zeros(1, W.RULE_DT)
    last["net"] = W.v4_nets(np.array([0], np.uint32), np.array([0]))
    last["min_port"] = last["max_port"] = 4789
    last["allow"] = 1
    udp = np.concatenate([t.udp, last])
    a, na, ka = W.as_ctypes(t.tcp, V._lib.VcAclRule)
    b, nb, kb = W.as_ctypes(udp, V._lib.VcAclRule)
    V.check(V.lib().vc_compile_acl(clf.h, a, na, b, nb, 0))
    return t.tcp, udp


def mirror_items_workload(n, dev, mf_of):
    """The `mirroritems` sub-bench (Mirror.mirror over MirrorData items):
    40 seeded filters of one origin ("tcp-lb": MACs, IPv4 / IPv6 / mapped
    networks, transport and application protocols, port ranges) and n items
    drawn on the device from 64K seeded templates at every null level.
    mf_of(filters) compiles the filters and returns the MirrorFilters
    interning.  Returns (filters, mf, numpy template columns, device
    columns of the batch, template index per item)."""
    rng = np.random.default_rng(W.SEED + 41)
    pick = lambda xs: xs[int(rng.integers(0, len(xs)))]
    macs = ["0a:00:27:00:00:%02x" % i for i in range(6)]
    nets = ["10.0.0.0/8", "10.1.0.0/16", "192.168.0.0/24", "172.16.0.0/12", "fd00::/8",
            "fd00:1::/32", "::ffff:10.0.0.0/104", "2001:db8::/32", "100.64.0.0/10"]
    filters = []
    for k in range(40):
        f = {"origin": "tcp-lb", "mirror": k % 12}
        if rng.random() < 0.3:
            f["mac"] = pick(macs)
        if rng.random() < 0.8:
            f["network"] = pick(nets)
            if rng.random() < 0.4:
                f["network2"] = pick(nets)
        if rng.random() < 0.6:
            f["transportLayerProtocol"] = pick(["tcp", "udp"])
        if rng.random() < 0.6:
            a = int(rng.integers(0, 60000))
            f["port"] = [a, a + int(rng.integers(0, 2000))]
            if rng.random() < 0.3:
                b = int(rng.integers(0, 60000))
                f["port2"] = [b, b + int(rng.integers(0, 2000))]
        if rng.random() < 0.3:
            f["applicationLayerProtocol"] = pick(["http", "dns", "h2"])
        filters.append(f)
    mf = mf_of(filters)
    t = 1 << 16
    ips4 = np.concatenate([np.array([[10, 0, 0, 0], [10, 1, 0, 0], [192, 168, 0, 0], [172, 16, 0, 0],
                                     [100, 64, 0, 0], [8, 8, 0, 0]], np.uint8)[rng.integers(0, 6, t)]])
    ips4[:, 2:] = rng.integers(0, 256, (t, 2))
    cols = {"mac_src": np.array([[0x0a, 0, 0x27, 0, 0, int(x)] for x in rng.integers(0, 8, t)],
                                np.uint8).reshape(-1),
            "mac_dst": np.array([[0x0a, 0, 0x27, 0, 0, int(x)] for x in rng.integers(0, 8, t)],
                                np.uint8).reshape(-1)}
    for side, sh in (("src", 0), ("dst", 1)):
        ln = np.where(rng.random(t) < 0.7, 4, 16).astype(np.uint8)
        ip = np.zeros((t, 16), np.uint8)
        ip[:, :4] = np.roll(ips4, sh, axis=0)
        v6 = ln == 16
        kind = rng.integers(0, 3, t)
        ip[v6] = 0
        m = v6 & (kind == 0)                        # ::ffff:a.b.c.d
        ip[m, 10:12] = 0xFF
        ip[m, 12:] = np.roll(ips4, sh, axis=0)[m]
        m = v6 & (kind == 1)                        # fd00:: / fd00:1::
        ip[m, 0] = 0xFD
        ip[m, 3] = rng.integers(0, 2, int(m.sum()))
        ip[m, 8:] = rng.integers(0, 256, (int(m.sum()), 8))
        m = v6 & (kind == 2)                        # 2001:db8::
        ip[m, :4] = [0x20, 0x01, 0x0D, 0xB8]
        ip[m, 8:] = rng.integers(0, 256, (int(m.sum()), 8))
        ln[rng.random(t) < 0.05] = 0                # null IP: the Ethernet level
        cols["ip_%s_len" % side] = ln
        cols["ip_" + side] = ip
    tid = lambda s: mf.id_of(s, create=False)
    r = rng.random(t)
    cols["transport"] = np.where(r < 0.2, -1, np.where(rng.random(t) < 0.6, tid("tcp"),
                                                      tid("udp"))).astype(np.int32)
    cols["app"] = np.where((r < 0.5) | (cols["transport"] == -1), -1,
                           np.array([tid(x) for x in ("http", "dns", "h2")], np.int32)[
                               rng.integers(0, 3, t)]).astype(np.int32)
    cols["port_src"] = rng.integers(0, 65536, t).astype(np.int32)
    cols["port_dst"] = rng.integers(0, 65536, t).astype(np.int32)
    idx = torch.from_numpy(np.random.default_rng(W.SEED + 42).integers(0, t, n)).to(dev)
    dcols = {}
    for k, v in cols.items():
        d = torch.from_numpy(v).to(dev)
        if k.startswith("mac"):
            dcols[k] = d.view(-1, 6)[idx].contiguous().view(-1)
        else:
            dcols[k] = d[idx].contiguous()
    return filters, mf, cols, dcols, idx


# the `mirror` sub-bench's 17 filters (Mirror.switchPacket over the switch origin)
MIRROR_FILTERS = [{"origin": "switch", "mirror": i % 8, "network": "%d.0.0.0/8" % (i + 1),
                   "network2": "10.0.0.0/8"} for i in range(16)] + \
                 [{"origin": "switch", "mirror": 9, "mac": "0a:00:27:00:00:01"}]


def source_workload(n, dev):
    """The `source` sub-bench's inputs (also checked whole by
    tests/test_gpu_source.py): 10k groups of 1-31 IPv4 servers (90 %
    healthy), and n (group, client address) pairs generated on the device."""
    rng = np.random.default_rng(W.SEED + 14)
    groups = [[(bytes(rng.integers(0, 256, 4).astype(np.uint8)), 80, 1, rng.random() < 0.9)
               for _ in range(int(rng.integers(1, 32)))] for _ in range(10_000)]
    g = torch.Generator(device=dev)
    g.manual_seed(15)
    grp = torch.randint(0, len(groups), (n,), generator=g, device=dev, dtype=torch.int32)
    src = torch.randint(-2**31, 2**31 - 1, (n,), generator=g, device=dev, dtype=torch.int32)
    return groups, grp, src


def c3_workload(clf, dev, n=256 << 20, rank=0):
    """The `c3` sub-bench (also checked whole by tests/test_gpu_c5.py): the
    ~1M IPv4 + 200k IPv6 BGP-like prefixes through the RouteTable mirror,
    shortest first, compiled into clf; n lookups, 85 % IPv4 (90 % inside a
    prefix, generated on the device) and 15 % IPv6 (host-generated)."""
    c = types.SimpleNamespace()
    c.net, c.plen = W.gen_v4_prefixes(1_000_000, W.SEED + 3)
    c.hi, c.lo, c.p6 = W.gen_v6_prefixes(200_000, W.SEED + 4)
    c.rt = V.RouteTable()
    allnets = np.concatenate([W.v4_nets(c.net, c.plen), W.v6_nets(c.hi, c.lo, c.p6)])
    arr, n_all, keep = W.as_ctypes(allnets, V._lib.VcNet)
    c.rt.add_rules("bgp", arr, n=n_all)
    clf.compile_route_table(c.rt)
    c.n4 = int(n * 0.85)
    g = torch.Generator(device=dev)
    g.manual_seed(7 + rank)
    netd = torch.from_numpy(c.net.astype(np.int64)).to(dev)
    mkd = torch.from_numpy(W._mask32(c.plen).astype(np.int64)).to(dev)
    r = torch.randint(0, len(c.net), (c.n4,), generator=g, device=dev)
    q = torch.randint(0, 2**32, (c.n4,), generator=g, device=dev)
    c.q4 = dev_u32(torch.where(torch.rand(c.n4, generator=g, device=dev) < 0.9,
                               netd[r] | (q & (~mkd[r] & 0xFFFFFFFF)), q))
    del r, q
    c.q6h = W.v6_lookups(c.hi, c.lo, c.p6, n - c.n4, 8 + rank)
    c.q6 = torch.from_numpy(c.q6h).to(dev)
    return c


def sni_workload(n=16 << 20):
    """The `sni` sub-bench's inputs (also checked whole by
    tests/test_gpu_certs.py): 100k certificate holders, each a plain name
    and a "*." wildcard (200k names), 1M distinct SNIs from the C4 name
    generator (ports cut), and the n seeded draws that form the batch."""
    _, hosts = W.gen_groups(200_000, W.SEED + 9, wildcard=False)
    holders = [[hosts[i], "*." + hosts[i + 1]] for i in range(0, len(hosts), 2)]
    names = [x.split(b":")[0] for x in W.gen_hostnames(hosts, 1 << 20, W.SEED + 10)]
    pidx = np.random.default_rng(W.SEED + 11).integers(0, len(names), n)
    return holders, names, pidx


def dnsd_tables(clf, n_templates=1 << 20):
    """The `dnsd` workload's tables, compiled into clf: 100k hint-host
    groups, a 50k-line hosts file, a 10k-rule SecurityGroup (default allow);
    and n_templates query datagrams over the DNS-flavoured C4 hostnames (one
    A (70 %) or AAAA question, 30 % with an EDNS0 OPT record)."""
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    import dnswire as DW          # wire-format encoder (test infrastructure)
    t = types.SimpleNamespace()
    t.groups, ghosts = W.gen_groups(100_000, W.SEED + 5)
    clf.compile_upstream(t.groups)
    t.hosts = hosts_text()
    clf.compile_hosts_text(t.hosts)
    t.tcp, t.udp = W.gen_sg_rules(10000, W.SEED + 2, p_range=0.3)
    a, na, ka = W.as_ctypes(t.tcp, V._lib.VcAclRule)
    b, nb, kb = W.as_ctypes(t.udp, V._lib.VcAclRule)
    V.check(V.lib().vc_compile_acl(clf.h, a, na, b, nb, 1))
    qn = W.gen_hostnames(ghosts, n_templates, W.SEED + 6, dns=True, port_frac=0)
    trng = np.random.default_rng(W.SEED + 20)
    qt = np.where(trng.random(len(qn)) < 0.7, DW.A, DW.AAAA)
    edns = trng.random(len(qn)) < 0.3
    dgs = [DW.header(qd=1, ar=int(e), ident=i & 0xFFFF) + DW.question(q, int(qt_)) +
           (DW.opt_record() if e else b"") for i, (q, qt_, e) in enumerate(zip(qn, qt, edns))]
    t.dblob, t.doff = W.pack(dgs)
    t.qnames, t.qtypes = qn, qt
    return t


def dnsd_batch(t, n, dev):
    """n datagrams drawn from the templates (seeded), on the device, with
    random IPv4 senders and ports: (blob, off, payload bytes, remote4,
    remote_port, template index per datagram)."""
    pidx = np.random.default_rng(W.SEED + 21).integers(0, len(t.doff) - 1, n)
    blob, off, nbytes = gather_strings_dev(t.dblob, t.doff, pidx, dev)
    g = torch.Generator(device=dev)
    g.manual_seed(23)
    r4 = dev_u32(torch.randint(0, 2**32, (n,), generator=g, device=dev))
    rport = torch.randint(1024, 65536, (n,), generator=g, device=dev).to(torch.int16)
    return blob, off, nbytes, r4, rport, pidx


def sub_bench(args, clf, dev, rank, world):
    """Single-classifier benchmarks.  Each line carries `roofline` (its
    dominant kernel's algorithmic bytes over its event-timed duration) and,
    unless --no-cpu-baseline, the oracle's all-core and 1-core rates on a
    sample of the same workload."""
    O = None if args.no_cpu_baseline or rank > 0 else _oracle()
    cpu = None
    extra = {}
    S = lambda: C.c_void_p(torch.cuda.current_stream().cuda_stream)
    if args.workload in ("c1", "c2", "c2host"):
        if args.workload == "c1":
            # C1 plumbing: 64 rules + Table default 10/8 + 255 random-order CIDRs, 1M tuples
            tcp, udp = W.gen_sg_rules(64, W.SEED + 1, p_range=0.5, weighted=False)
            net, plen = W.gen_v4_prefixes(255, W.SEED + 31, dist=((8, 30, 1.0),))
            rt = V.RouteTable("10.0.0.0/8", None, 1)
            perm = np.random.default_rng(W.SEED + 32).permutation(len(net))
            for i in perm:
                s = "%d.%d.%d.%d/%d" % (net[i] >> 24, (net[i] >> 16) & 255, (net[i] >> 8) & 255,
                                        net[i] & 255, plen[i])
                try:
                    rt.add_rule("r%d" % i, s)
                except V.VcError:
                    pass                             # XException of RouteTable.addRule
            clf.compile_route_table(rt)
            a4, n4 = rt.rules_raw(4)
            rlist = np.frombuffer(bytes(a4)[:n4 * 40], W.NET_DT)
            n = 1 << 20
        else:
            tcp, udp = W.gen_sg_rules(10000, W.SEED + 2, p_range=0.3)
            n = 64 << 20
        a, na, ka = W.as_ctypes(tcp, V._lib.VcAclRule)
        b, nb, kb = W.as_ctypes(udp, V._lib.VcAclRule)
        V.check(V.lib().vc_compile_acl(clf.h, a, na, b, nb, 0))
        proto, src, port = W.gen_acl_queries(tcp, udp, n, W.SEED + 16)
        if args.workload == "c2host":
            # the plain (host-buffer) entry point over registered buffers
            out = np.empty(n, np.int32)
            allow = np.empty(n, np.uint8)
            for x in (proto, src, port, out, allow):
                V.check(V.lib().vc_host_register(C.c_void_p(x.ctypes.data), x.nbytes))
            P = lambda x: C.c_void_p(x.ctypes.data)
            fn = lambda: V.check(V.lib().vc_acl_classify_v4(clf.h, P(proto), P(src), P(port), n,
                                                              P(out), P(allow)))
            per_unit, unit, kern = 12, "B/tuple across PCIe (7 in + 5 out), kernel included", \
                "acl_v4_kernel (zero-copy over PCIe)"
        else:
            d = [torch.from_numpy(x).to(dev) for x in (proto, src, port)]
            out = torch.empty(n, dtype=torch.int32, device=dev)
            if args.workload == "c1":
                dst = W.v4_lookups(net, plen, n, W.SEED + 17)
                dd = torch.from_numpy(dst).to(dev)
                ro = torch.empty(n, dtype=torch.int32, device=dev)
                fn = lambda: (clf.acl_v4(*d, out_idx=out, want_allow=False),
                              clf.route_v4(dd, out=ro))
                per_unit, unit, kern = 19, "B/tuple (ACL 7 in + 4 out, route 4 in + 4 out)", \
                    "acl_v4_kernel + route_v4_kernel"
                # end to end from host buffers (pageable: staged copies)
                hsrc = (proto, src, port, dst)

                def e2e():
                    clf.acl_v4(*hsrc[:3], want_allow=False)
                    clf.route_v4(hsrc[3])
                e2e()
                t0 = time.perf_counter()
                for _ in range(5):
                    e2e()
                extra["end_to_end_host_buffers_M_per_s"] = round(
                    n * 5 / (time.perf_counter() - t0) / 1e6, 1)
                extra["end_to_end_note"] = ("vc_acl_classify_v4 + vc_route_lookup_v4 on pageable "
                                            "host arrays: H2D + kernel + D2H, synchronous")
            else:
                fn = lambda: clf.acl_v4(*d, out_idx=out, want_allow=False)
                per_unit, unit, kern = 11, "B/tuple (7 in + 4 out)", "acl_v4_kernel"
                extra["end_to_end_host_buffers_M_per_s"] = end_to_end(
                    lambda: clf.acl_v4(proto, src, port, want_allow=True), n)
                extra["end_to_end_note"] = ("vc_acl_classify_v4 on pageable host arrays (chunked "
                                            "DMA staging), synchronous; registered buffers: c2host")
        if O is not None:
            def run(k, threads):
                t0 = time.perf_counter()
                O.sg_batch_v4_np(tcp, udp, False, proto[:k], src[:k], port[:k], nthreads=threads)
                if args.workload == "c1":
                    O.rt_batch_v4_np(rlist, dst[:k], nthreads=threads)
                return time.perf_counter() - t0
            if args.workload == "c1":
                cpu = {}
                info = cpu_info()
                for th in (info["threads_all"], 1):     # C1 runs in full
                    tt = run(n, th)
                    cpu[th] = n / tt / 1e6
                cpu = {"value": cpu[info["threads_all"]], "unit": "M items/s",
                       "cores": info["threads_all"], "kind": "port",
                       "sample": "the full C1 batch (%d tuples, ACL + route), oracle linear "
                                 "scans" % n,
                       "one_core": {"value": cpu[1], "cores": 1}, "nproc": info["nproc"],
                       "affinity": info["affinity"], "cgroup_cpu_max": info["cgroup_cpu_max"],
                       "quota_cpus": info["quota_cpus"], "cpu_model": info["cpu_model"]}
            else:
                cpu = functools.partial(cpu_rates, run, "M items/s", 4.0, "first tuples of the C2 batch, oracle "
                                "first-match scan over 10k rules")
    elif args.workload == "c3":
        n = 256 << 20
        c3 = c3_workload(clf, dev, n, rank)
        rt, net, plen, hi, lo, p6 = c3.rt, c3.net, c3.plen, c3.hi, c3.lo, c3.p6
        q4, q6h, q6, n4 = c3.q4, c3.q6h, c3.q6, c3.n4
        o4 = torch.empty(n4, dtype=torch.int32, device=dev)
        o6 = torch.empty(n - n4, dtype=torch.int32, device=dev)
        fn = lambda: (clf.route_v4(q4, out=o4), clf.route_v6(q6, out=o6))
        per_unit, unit = (8 * 0.85 + 20 * 0.15), "B/lookup (v4 4+4, v6 16+4, 85/15 mix)"
        kern = "route_v4_kernel + route_v6_kernel_x4"
        # the split, each family timed alone
        e4, ms4 = _time(lambda: clf.route_v4(q4, out=o4), 3, 1)
        e6, ms6 = _time(lambda: clf.route_v6(q6, out=o6), 3, 1)
        extra["v4_ms"], extra["v6_ms"] = round(ms4, 4), round(ms6, 4)
        q4h_all = q4.cpu().numpy().view(np.uint32)
        extra["end_to_end_host_buffers_M_per_s"] = end_to_end(
            lambda: (clf.route_v4(q4h_all), clf.route_v6(q6h)), n)
        extra["end_to_end_note"] = ("vc_route_lookup_v4 + vc_route_lookup_v6 on pageable host "
                                    "arrays: chunked H2D + kernel + D2H, synchronous")
        del q4h_all
        extra["v4_G_per_s"] = round(n4 / ms4 / 1e6, 2)
        extra["v6_G_per_s"] = round((n - n4) / ms6 / 1e6, 2)
        if O is not None:
            a4, k4 = rt.rules_raw(4)
            a6, k6 = rt.rules_raw(6)
            v4l = np.frombuffer(bytes(a4)[:k4 * 40], W.NET_DT)
            v6l = np.frombuffer(bytes(a6)[:k6 * 40], W.NET_DT)
            q4h = W.v4_lookups(net, plen, 1 << 16, W.SEED + 33)

            def run(k, threads):
                k4_ = max(1, int(k * 0.85))
                t0 = time.perf_counter()
                O.rt_batch_v4_np(v4l, q4h[:k4_], nthreads=threads)
                O.rt_batch_v6_np(v6l, q6h[:max(1, k - k4_)], nthreads=threads)
                return time.perf_counter() - t0
            cpu = functools.partial(cpu_rates, run, "M items/s", 4.0, "85/15 v4/v6 lookups of the C3 workload, "
                            "oracle first-match scans over the RouteTable lists")
    elif args.workload in ("c4", "dns"):
        dns = args.workload == "dns"
        n = 16 << 20
        groups, hosts, names, pidx = c4_workload(dns, n)
        clf.compile_upstream(groups)
        if dns:
            clf.compile_hosts_text(hosts)
        nblob, noff = W.pack(names)
        blob, off, nbytes = gather_strings_dev(nblob, noff, pidx, dev)
        hblob, hoff = blob.cpu().numpy(), off.cpu().numpy().view(np.uint32)
        P = lambda x: C.c_void_p(x.ctypes.data)
        if dns:
            hk, hv = np.empty(n, np.uint8), np.empty(n, np.int32)
            e2e = lambda: V.check(V.lib().vc_dns_classify(clf.h, P(hblob), P(hoff), n, P(hk), P(hv)))
        else:
            ho_ = np.empty(n, np.int32)
            e2e = lambda: V.check(V.lib().vc_hint_search(clf.h, P(hblob), P(hoff), None, None, None,
                                                         None, None, n, P(ho_)))
        extra["end_to_end_host_buffers_M_per_s"] = end_to_end(e2e, n)
        extra["end_to_end_note"] = ("%s on pageable host arrays (blob + offsets in, results "
                                    "out): chunked H2D + kernel + D2H, synchronous"
                                    % ("vc_dns_classify" if dns else "vc_hint_search"))
        if dns:
            kind = torch.empty(n, dtype=torch.uint8, device=dev)
            val = torch.empty(n, dtype=torch.int32, device=dev)
            fn = lambda: V.check(V.lib().vc_dns_classify_dev(
                clf.h, C.c_void_p(blob.data_ptr()), C.c_void_p(off.data_ptr()), n,
                C.c_void_p(kind.data_ptr()), C.c_void_p(val.data_ptr()), S()))
            per_unit, unit, kern = nbytes / n + 9, "B/qname (bytes + 4 offset + 1 kind + 4 " \
                                                   "value)", "dns_kernel"
        else:
            out = torch.empty(n, dtype=torch.int32, device=dev)
            fn = lambda: V.check(V.lib().vc_hint_search_dev(
                clf.h, C.c_void_p(blob.data_ptr()), C.c_void_p(off.data_ptr()), None, None, None,
                None, None, n, C.c_void_p(out.data_ptr()), S()))
            per_unit, unit, kern = nbytes / n + 8, "B/hostname (bytes + 4 offset + 4 out)", \
                "hint_kernel"
        if O is not None:
            og = O.Groups(groups)
            oh = O.Hosts(O.hosts_parse(hosts)[0]) if dns else None

            def run(k, threads):
                sb, so = sample_blob(nblob, noff, pidx[:k])
                t0 = time.perf_counter()
                if dns:
                    O.dns_batch_np(oh, og, sb, so, nthreads=threads)
                else:
                    O.hint_batch_np(og, sb, so, None, nthreads=threads)
                return time.perf_counter() - t0
            if dns:
                cpu = functools.partial(cpu_rates, run, "M items/s", 4.0, "qnames of the DNS workload, oracle hosts "
                                "lookup (50k entries) + searchForGroup scan over 100k groups", cap=n)
            else:
                cpu = functools.partial(cpu_rates, run, "M items/s", 4.0, "hostnames of the C4 pool, oracle "
                                "searchForGroup scan over 100k groups", cap=n)
    elif args.workload == "dnsd":
        # DNSServer's drain loop per datagram: UDP SecurityGroup (10k rules)
        # -> parsePackets -> handleRequest classification over 100k groups
        # + 50k hosts; queries of one A / AAAA question, 30 % with an EDNS0
        # OPT record, from random IPv4 senders
        t = dnsd_tables(clf)
        groups, hosts, tcp, udp, dblob, doff = t.groups, t.hosts, t.tcp, t.udp, t.dblob, t.doff
        n = 16 << 20
        blob, off, nbytes, r4, rport, pidx = dnsd_batch(t, n, dev)
        res = {"status": torch.empty(n, dtype=torch.uint8, device=dev),
               "acl": torch.empty(n, dtype=torch.int32, device=dev),
               "nq": torch.empty(n, dtype=torch.uint8, device=dev),
               "qtype": torch.empty((n, V.DNSD_MAXQ), dtype=torch.int16, device=dev),
               "kind": torch.empty((n, V.DNSD_MAXQ), dtype=torch.uint8, device=dev),
               "value": torch.empty((n, V.DNSD_MAXQ), dtype=torch.int32, device=dev)}
        o = V._lib.VcDnsdOut(**{k_: v_.data_ptr() for k_, v_ in res.items()})
        fn = lambda: V.check(V.lib().vc_dns_datagrams_dev(
            clf.h, C.c_void_p(blob.data_ptr()), C.c_void_p(off.data_ptr()), n, None,
            C.c_void_p(r4.data_ptr()), None, C.c_void_p(rport.data_ptr()), C.byref(o), S()))
        # written: status 1 + acl 4 + nq 1 + one question's qtype 2 + kind 1 + value 4
        per_unit = nbytes / n + 4 + 4 + 2 + 13
        unit = ("B/datagram (payload + 4 offset + 4 sender + 2 port in; status, rule, count "
                "and one question's qtype/kind/value out)")
        kern = "dnsd_kernel"
        hb, ho = blob.cpu().numpy(), off.cpu().numpy().view(np.uint32)
        h4, hp = r4.cpu().numpy().view(np.uint32), rport.cpu().numpy().view(np.uint16)
        hres = {"status": np.empty(n, np.uint8), "kind": np.empty((n, V.DNSD_MAXQ), np.uint8),
                "value": np.empty((n, V.DNSD_MAXQ), np.int32)}
        ho_ = V._lib.VcDnsdOut(**{k_: v_.ctypes.data for k_, v_ in hres.items()})
        P = lambda x: C.c_void_p(x.ctypes.data)
        extra["end_to_end_host_buffers_M_per_s"] = end_to_end(
            lambda: V.check(V.lib().vc_dns_datagrams(clf.h, P(hb), P(ho), n, None, P(h4), None,
                                                     P(hp), C.byref(ho_))), n)
        extra["end_to_end_note"] = ("vc_dns_datagrams on pageable host arrays (payloads, "
                                    "offsets, senders in; status/kind/value out): staged H2D + "
                                    "kernel + D2H, synchronous")
        fn()
        torch.cuda.synchronize()
        st = res["status"].cpu().numpy()
        extra["status_mix"] = {nm: round(float((st == c_).mean()), 4) for c_, nm in enumerate(
            ("answer", "recursive", "response", "rejected", "empty", "malformed", "host"))}
        if O is not None:
            og = O.Groups(groups)
            oh = O.Hosts(O.hosts_parse(hosts)[0])

            def run(k, threads):
                sb, so = sample_blob(dblob, doff, pidx[:k])
                t0 = time.perf_counter()
                O.dnsd_batch_np(tcp, udp, True, oh, og, sb, so, None, h4[:k], None, hp[:k],
                                nthreads=threads)
                return time.perf_counter() - t0
            cpu = functools.partial(cpu_rates, run, "M items/s", 4.0, "datagrams of the workload, oracle UDP "
                            "SecurityGroup scan (10k rules) + parsePackets + hosts lookup and "
                            "searchForGroup scan over 100k groups", cap=n)
    elif args.workload == "sni":
        n = 16 << 20
        holders, names, pidx = sni_workload(n)
        clf.compile_certs(holders)
        nblob, noff = W.pack(names)
        blob, off, nbytes = gather_strings_dev(nblob, noff, pidx, dev)
        out = torch.empty(n, dtype=torch.int32, device=dev)
        fn = lambda: V.check(V.lib().vc_cert_choose_dev(
            clf.h, C.c_void_p(blob.data_ptr()), C.c_void_p(off.data_ptr()), None, n,
            C.c_void_p(out.data_ptr()), S()))
        per_unit, unit, kern = nbytes / n + 8, "B/SNI (bytes + 4 offset + 4 out)", "cert_kernel"
        if O is not None:
            oc = O.Certs(holders)

            def run(k, threads):
                sb, so = sample_blob(nblob, noff, pidx[:k])
                t0 = time.perf_counter()
                O.cert_batch_np(oc, sb, so, nthreads=threads)
                return time.perf_counter() - t0
            cpu = functools.partial(cpu_rates, run, "M items/s", 3.0, "SNIs of the workload, oracle "
                            "SSLContextHolder.choose scan over 100k holders (200k names)", cap=n)
    elif args.workload == "c4uri":
        n = 16 << 20
        groups, names, uris, nidx, uidx = c4uri_workload(n)
        clf.compile_upstream(groups)
        hb, ho, ub, uo, un, nbytes = c4uri_batch(names, uris, nidx, uidx, dev)
        out = torch.empty(n, dtype=torch.int32, device=dev)
        fn = lambda: V.check(V.lib().vc_hint_search_dev(
            clf.h, C.c_void_p(hb.data_ptr()), C.c_void_p(ho.data_ptr()), None, None,
            C.c_void_p(ub.data_ptr()), C.c_void_p(uo.data_ptr()), C.c_void_p(un.data_ptr()), n,
            C.c_void_p(out.data_ptr()), S()))
        per_unit = nbytes / n + 13
        unit = "B/hint (host + uri bytes + 2 x 4 offsets + 1 null + 4 out)"
        kern = "hint_kernel"
        extra["uri_fraction"] = round(float((uidx >= 0).mean()), 4)
        if O is not None:
            og = O.Groups(groups)
            nblob, noff = W.pack(names)
            ublob, uoff = W.pack(uris)

            def run(k, threads):
                sb, so = sample_blob(nblob, noff, nidx[:k])
                ubs, uos = sample_blob(ublob, uoff, np.maximum(uidx[:k], 0))
                t0 = time.perf_counter()
                O.hint_uri_batch_np(og, sb, so, ubs, uos, (uidx[:k] < 0).astype(np.uint8),
                                    nthreads=threads)
                return time.perf_counter() - t0
            cpu = functools.partial(cpu_rates, run, "M items/s", 4.0, "Hint.ofHostUri hints of the workload, oracle "
                            "searchForGroup scan (whole matchLevel) over 100,200 groups", cap=n)
    elif args.workload == "http":
        n = 8 << 20
        groups, heads, pidx = http_workload(n)
        clf.compile_upstream(groups)
        hblob_t, hoff_t = W.pack(heads)
        blob, off, nbytes = gather_strings_dev(hblob_t, hoff_t, pidx, dev)
        grp = torch.empty(n, dtype=torch.int32, device=dev)
        kind = torch.empty(n, dtype=torch.uint8, device=dev)
        fn = lambda: V.check(V.lib().vc_http_hint_dev(
            clf.h, C.c_void_p(blob.data_ptr()), nbytes, C.c_void_p(off.data_ptr()), n,
            C.c_void_p(grp.data_ptr()), C.c_void_p(kind.data_ptr()), S()))
        per_unit, unit, kern = nbytes / n + 9, "B/request head (bytes + 4 offset + 4 group + " \
                                                "1 kind)", "http_hint_kernel"
        hb, ho = blob.cpu().numpy(), off.cpu().numpy().view(np.uint32)
        P = lambda x: C.c_void_p(x.ctypes.data)
        hg, hk = np.empty(n, np.int32), np.empty(n, np.uint8)
        extra["end_to_end_host_buffers_M_per_s"] = end_to_end(
            lambda: V.check(V.lib().vc_http_hint(clf.h, P(hb), P(ho), n, P(hg), P(hk))), n)
        extra["end_to_end_note"] = ("vc_http_hint on pageable host arrays (heads + offsets in, "
                                    "group + kind out): chunked H2D + kernel + D2H, synchronous")
        del hb, ho
        if O is not None:
            og = O.Groups(groups)

            def run(k, threads):
                sb, so = sample_blob(hblob_t, hoff_t, pidx[:k])
                t0 = time.perf_counter()
                O.http_batch_np(og, sb, so, nthreads=threads)
                return time.perf_counter() - t0
            cpu = functools.partial(cpu_rates, run, "M items/s", 4.0, "request heads of the workload, oracle "
                            "HttpSubContext state machine + searchForGroup scan over 100k groups",
                            cap=n)
    elif args.workload in ("parse", "mirror", "switch"):
        n = 32 << 20
        frames, pidx = frames_workload(n)
        fblob, foff = W.pack(frames)
        blob, off, nbytes = gather_strings_dev(fblob, foff, pidx, dev)
        if args.workload == "parse":
            res = {k: torch.empty((n, w) if w > 1 else (n,), dtype={"u8": torch.uint8,
                   "u16": torch.int16, "u32": torch.int32}[t], device=dev)
                   for k, w, t in V.Classifier._PKT_FIELDS}
            o = V._lib.VcPktOut(**{k: v.data_ptr() for k, v in res.items()})
            fn = lambda: V.check(V.lib().vc_parse_packets_dev(
                clf.h, C.c_void_p(blob.data_ptr()), C.c_void_p(off.data_ptr()), n, 0,
                C.byref(o), S()))
            per_unit = nbytes / n + 4 + 54
            unit = "B/frame (frame bytes + 4 offset in; 54 B of SoA fields out)"
            kern = "packet_kernel"
            if O is not None:
                def run(k, threads):
                    sb, so = sample_blob(fblob, foff, pidx[:k])
                    t0 = time.perf_counter()
                    O.parse_batch_np(sb, so, 0, nthreads=threads)
                    return time.perf_counter() - t0
                cpu = functools.partial(cpu_rates, run, "M items/s", 3.0, "frames of the workload, oracle vpacket "
                                "parse chain (VXLAN -> Ethernet -> IPv4/IPv6 -> TCP/ICMP)", cap=1 << 22)
        elif args.workload == "switch":
            # parse + bare-VXLAN ACL on the sender + inner route, one kernel,
            # over the C5 SecurityGroup and route tables; only the route
            # index and the verdict leave the kernel
            t = c5_tables(clf, dev, 1 << 20)
            sw_tcp, sw_udp = compile_switch_acl(clf, t)
            r4 = switch_senders(n, dev)
            out_route = torch.empty(n, dtype=torch.int32, device=dev)
            out_allow = torch.empty(n, dtype=torch.uint8, device=dev)
            none = V._lib.VcPktOut()
            fn = lambda: V.check(V.lib().vc_switch_classify_dev(
                clf.h, C.c_void_p(blob.data_ptr()), C.c_void_p(off.data_ptr()), n, 0, None,
                C.c_void_p(r4.data_ptr()), None, 4789, C.byref(none), None,
                C.c_void_p(out_allow.data_ptr()), C.c_void_p(out_route.data_ptr()), S()))
            per_unit = nbytes / n + 4 + 4 + 5
            unit = ("B/datagram (frame bytes + 4 offset + 4 sender in; 4 route + 1 verdict out), "
                    "10k-rule SecurityGroup + a last allow rule for the VXLAN port, "
                    "980,848 + 200,000 routes")
            kern = "switch_kernel"
            if O is not None:
                r4h = r4[:1 << 20].cpu().numpy().view(np.uint32)

                def run(k, threads):
                    sb, so = sample_blob(fblob, foff, pidx[:k])
                    t0 = time.perf_counter()
                    O.switch_batch_np(sw_tcp, sw_udp, False, sb, so, r4h[:k], 4789, t.v4_list,
                                      t.v6_list, nthreads=threads)
                    return time.perf_counter() - t0
                cpu = functools.partial(cpu_rates, run, "M items/s", 4.0, "datagrams of the workload, oracle parse + "
                                "SecurityGroup.allow scan + RouteTable.lookup scan of the inner "
                                "destination", cap=1 << 20)
        else:
            filters = MIRROR_FILTERS
            mf = clf.compile_mirror(filters)
            out = torch.empty(n, dtype=torch.int64, device=dev)
            oid = mf.id_of("switch", create=False)
            fn = lambda: V.check(V.lib().vc_mirror_switch_dev(
                clf.h, oid, C.c_void_p(blob.data_ptr()), C.c_void_p(off.data_ptr()), n, 0,
                C.c_void_p(out.data_ptr()), S()))
            per_unit = nbytes / n + 4 + 8
            unit = "B/frame (frame bytes + 4 offset in; 8 B mirror set out), 17 filters"
            kern = "mirror_switch_kernel"
            if O is not None:
                ids = {}
                oarr = O.mirror_filters(filters, ids)

                def run(k, threads):
                    sb, so = sample_blob(fblob, foff, pidx[:k])
                    t0 = time.perf_counter()
                    O.mirror_switch_batch_np(oarr, len(filters), ids["switch"], sb, so, 0,
                                             nthreads=threads)
                    return time.perf_counter() - t0
                cpu = functools.partial(cpu_rates, run, "M items/s", 3.0, "frames of the workload, oracle "
                                "Mirror.switchPacket over the 17 filters", cap=1 << 22)
    elif args.workload == "mirroritems":
        n = 32 << 20
        from vproxy_amd.mirror import items_struct
        filters, mf, tcols, dcols, tidx = mirror_items_workload(n, dev, clf.compile_mirror)
        it = items_struct(dcols)
        out = torch.empty(n, dtype=torch.int64, device=dev)
        oid = mf.id_of("tcp-lb", create=False)
        fn = lambda: V.check(V.lib().vc_mirror_match_dev(
            clf.h, oid, C.byref(it), n, C.c_void_p(out.data_ptr()), S()))
        per_unit = 6 + 6 + 1 + 1 + 16 + 16 + 4 * 4 + 8
        unit = ("B/item (MACs 6 + 6, IP lengths 1 + 1, IP rows 16 + 16, transport, ports, app "
                "4 each in; 8 B mirror set out), 40 filters")
        kern = "mirror_match_kernel"
        if O is not None:
            ids = {}
            oarr = O.mirror_filters(filters, ids)
            assert ids == mf.ids
            ti = tidx[:1 << 22].cpu().numpy()
            scols = {}
            for k, v in tcols.items():
                scols[k] = (v.reshape(-1, 6)[ti].reshape(-1) if k.startswith("mac") else v[ti])

            def run(k, threads):
                c = {key: (v[:6 * k] if key.startswith("mac") else v[:k])
                     for key, v in scols.items()}
                t0 = time.perf_counter()
                O.mirror_match_batch_np(oarr, len(filters), ids["tcp-lb"], c, nthreads=threads)
                return time.perf_counter() - t0
            cpu = functools.partial(cpu_rates, run, "M items/s", 3.0, "items of the workload, "
                                    "oracle Mirror.mirror over the 40 filters", cap=1 << 22)
    elif args.workload == "source":
        n = 128 << 20
        groups, grp, src = source_workload(n, dev)
        clf.compile_servers(groups)
        out = torch.empty(n, dtype=torch.int32, device=dev)
        fn = lambda: V.check(V.lib().vc_source_select_v4_dev(
            clf.h, C.c_void_p(grp.data_ptr()), C.c_void_p(src.data_ptr()), n, 0,
            C.c_void_p(out.data_ptr()), S()))
        per_unit, unit, kern = 12, "B/item (group 4 + v4 source 4 in, 4 out)", "source_v4_kernel"
        if O is not None:
            gh = grp[:1 << 22].cpu().numpy()
            sh = src[:1 << 22].cpu().numpy().view(np.uint32)
            osg = O.SourceGroups(groups)

            def run(k, threads):
                t0 = time.perf_counter()
                O.source_batch_np(osg, 0, gh[:k], sh[:k], nthreads=threads)
                return time.perf_counter() - t0
            cpu = functools.partial(cpu_rates, run, "M items/s", 3.0, "clients of the workload, oracle "
                            "sourceHashGet over each group's sourceReset order (built once per "
                            "call for all 10k groups, as Java caches it per group)", cap=1 << 22)
    else:
        return mix_bench(args, clf, dev, rank, O, world)
    el, ms = _time(fn, args.steps, args.warmup)
    # the CPU baseline after the timed launches: run before them, its seconds
    # of host work left the GPU idle, and short kernels (SNI: 0.53 ms) timed
    # up to 2.3x slower right after
    if callable(cpu):
        cpu = cpu()
    gbs = per_unit * n / (ms / 1e3) / 1e9
    res = {"workload": args.workload, "items": n, "ms_per_step": round(el / args.steps * 1e3, 3),
           "kernel_ms": round(ms, 4), "M_items_per_s": round(n / (ms / 1e3) / 1e6, 1),
           "roofline": {"bound": "hbm", "achieved": round(gbs, 2), "peak": HBM_PEAK_GBS,
                        "unit": "GB/s", "frac": round(gbs / HBM_PEAK_GBS, 5), "kernel": kern,
                        "algorithmic_bytes": unit},
           "cpu_baseline": cpu}
    res.update(extra)
    replicas(res, world, dev)
    if rank == 0:
        print(json.dumps(res), flush=True)
    clf.close()


def _be_bytes(x, n):
    """int64 tensor of 64-bit values -> uint8 [n, 8] big-endian bytes."""
    return x.contiguous().view(torch.uint8).view(n, 8).flip(1)


def gen_mixed(lo, n, t, pool_n, v6_frac=0.15, seed=PACKET_SEED + 1, dev="cpu"):
    """Items [lo, lo + n) of a seeded mixed-family batch for vc_pipeline:
    gen_packets' IPv4 fields plus a family (v6_frac IPv6), IPv6 sources
    (half IPv4-mapped ::ffff:a.b.c.d forms of the IPv4 source, so the v4
    rules' v6 projections match them) and IPv6 destinations (90 % inside a
    random rulesV6 prefix).  Index-addressable like gen_packets."""
    proto, src, dst, dport, hid = gen_packets(lo, n, t, pool_n, seed=seed, dev=dev)
    idx = torch.arange(lo, lo + n, device=dev, dtype=torch.int64)
    h = lambda s: hash_u32(idx, seed, s)
    fam = torch.where(below(h(60), 1 << 20) < int(v6_frac * (1 << 20)), 6, 4).to(torch.uint8)
    # sources: ::ffff:src4 or a random 2001:db8::/32 address
    s_hi = (h(61) << 32) | h(62)
    s_hi = torch.where((h(63) & 1) == 0, torch.zeros_like(s_hi),
                       (s_hi & 0xFFFFFFFF) | (0x20010DB8 << 32))
    s_lo = torch.where(s_hi == 0, (0xFFFF << 32) | (src.to(torch.int64) & 0xFFFFFFFF),
                       (h(64) << 32) | h(65))
    # destinations: 90 % inside a random IPv6 route prefix
    hi_t = torch.from_numpy(t.hi.view(np.int64)).to(dev)
    p6 = torch.from_numpy(t.p6.astype(np.int64)).to(dev)
    r = below(h(66), len(t.hi))
    q = (h(67) << 32) | h(68)
    keep = torch.where(p6[r] >= 64, torch.full_like(q, -1),
                       (torch.full_like(q, -1) << (64 - torch.clamp(p6[r], max=63))))
    d_hi = torch.where(below(h(69), 10) < 9, (hi_t[r] & keep) | (q & ~keep), q)
    d_lo = (h(70) << 32) | h(71)
    src6 = torch.cat([_be_bytes(s_hi, n), _be_bytes(s_lo, n)], 1).contiguous()
    dst6 = torch.cat([_be_bytes(d_hi, n), _be_bytes(d_lo, n)], 1).contiguous()
    return fam, proto, src, dst, src6, dst6, dport, hid


def mix_bench(args, clf, dev, rank, O, world=1):
    """The general pipeline (vc_pipeline_dev / vc_pipeline) on the C5 tables
    over a mixed batch: 85 % IPv4 / 15 % IPv6 packets as in C3, per-packet
    family dispatch (RouteTable.java:44-58).  `mix`: device-resident
    packets, fused counters with the finish on a second stream; `mixhost`:
    the host entry point over registered host buffers (a batch with IPv6
    packets is copied through device staging in chunks by DMA: zero-copy
    reads of scattered 16-byte addresses ran at 7 GB/s)."""
    t = c5_tables(clf, dev, args.pool)
    n = args.packets if args.workload == "mix" else 32 << 20
    fam, proto, src, dst, src6, dst6, dport, hid = gen_mixed(0, n, t, t.pool_n, dev=dev,
                                                             v6_frac=args.v6_frac)
    pool = clf.hint_search((t.pool_blob, t.pool_off, None))
    torch.cuda.synchronize()
    n6 = int((fam == 6).sum())
    extra = {"ipv6_packets": n6, "ipv4_packets": n - n6}
    per_unit = ((n - n6) * 28 + n6 * 52) / n
    unit = ("B/packet: IPv4 28 (family 1 + proto 1 + src 4 + dst 4 + dport 2 + host_id 4 in, 3x "
            "int32 out), IPv6 52 (family 1 + proto 1 + src 16 + dst 16 + dport 2 + host_id 4 "
            "in, 3x int32 out); %.1f at this mix" % ((n - n6) * 28 / n + n6 * 52 / n))
    kev = []                                       # (before, after) the classify kernel
    if args.workload == "mix":
        outs = tuple(torch.empty(n, dtype=torch.int32, device=dev) for _ in range(3)) + (None,)
        s_cnt = hip_stream(dev)
        clf.counters_enable(True)

        s6, d6 = src6, dst6
        if args.compact6:                          # one row per IPv6 packet, packet order
            six = fam == 6
            s6, d6 = src6[six].contiguous(), dst6[six].contiguous()
            extra["compact6_rows"] = len(s6)

        def fn():
            k0, k1 = RawEvent(), RawEvent()
            k0.record(torch.cuda.current_stream())
            clf.pipeline(proto, src, dst, dport, hid, pool, family=fam, src6=s6, dst6=d6,
                         outs=outs, count_stream=s_cnt, kernel_done_event=k1.h.value,
                         compact6=args.compact6)
            kev.append((k0, k1))
        kern = "pipeline_mix_kernel (+ counter finish on a second stream)" + (
            ", compact IPv6 rows (vc_pipeline_c6_dev)" if args.compact6 else "")

        def fin():
            torch.cuda.current_stream().wait_stream(s_cnt)
    else:
        hs = [x.cpu().numpy() for x in (fam, proto, src, dst, src6, dst6, dport, hid)]
        hs[2], hs[3] = hs[2].view(np.uint32), hs[3].view(np.uint32)
        hs[6], hs[7] = hs[6].view(np.uint16), hs[7].view(np.uint32)
        if args.compact6:                          # one row per IPv6 packet, packet order
            six = hs[0] == 6
            hs[4], hs[5] = np.ascontiguousarray(hs[4][six]), np.ascontiguousarray(hs[5][six])
            extra["compact6_rows"] = len(hs[4])
        hpool = pool.cpu().numpy()
        houts = (np.empty(n, np.int32), np.empty(n, np.int32), np.empty(n, np.int32), None)
        reg = hs + [hpool] + list(houts[:3])
        for x in reg:
            if x.nbytes:                           # (no rows at --v6-frac 0)
                V.check(V.lib().vc_host_register(C.c_void_p(x.ctypes.data), x.nbytes))
        fn = lambda: clf.pipeline(hs[1], hs[2], hs[3], hs[6], hs[7], hpool, family=hs[0],
                                  src6=hs[4], dst6=hs[5], outs=houts, compact6=args.compact6)
        kern = ("pipeline_mix_kernel over registered host buffers, compact IPv6 rows "
                "(vc_pipeline_c6, zero-copy), synchronous" if args.compact6 else
                "pipeline_mix_kernel, inputs and outputs over PCIe (chunked DMA staging), "
                "synchronous")
        fin = None
    for _ in range(args.warmup):
        fn()
    torch.cuda.synchronize()
    ev = []
    t0 = time.perf_counter()
    for _ in range(args.steps):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        fn()
        if fin:
            fin()
        e1.record()
        ev.append((e0, e1))
    torch.cuda.synchronize()
    el = time.perf_counter() - t0
    ms = float(np.mean([a.elapsed_time(b) for a, b in ev]))
    if args.workload == "mixhost":
        ms = el / args.steps * 1e3
    else:
        # the classify kernel alone, and the IPv4 kernel (vc_pipeline_v4_dev)
        # over the same packets' IPv4 fields with the same counting: the
        # same-conditions reference for what the IPv6 share costs
        extra["kernel_only_ms"] = round(float(np.mean(
            [a.elapsed_time(b) for a, b in kev[-args.steps:]])), 4)
        ref = []
        for r in range(args.warmup + args.steps):
            k0, k1 = RawEvent(), RawEvent()
            k0.record(torch.cuda.current_stream())
            clf.pipeline_v4(proto, src, dst, dport, hid, pool, outs=outs,
                            kernel_done_event=k1.h.value, count_stream=s_cnt)
            fin()
            ref.append((k0, k1))
        torch.cuda.synchronize()
        extra["v4_kernel_same_packets_ms"] = round(float(np.mean(
            [a.elapsed_time(b) for a, b in ref[args.warmup:]])), 4)
    gbs = per_unit * n / (ms / 1e3) / 1e9
    cpu = None
    if O is not None:
        og = O.Groups(t.groups)

        def run(k, threads):
            x = [v[:k].cpu().numpy() for v in (fam, proto, src, dst, src6, dst6, dport, hid)]
            six = x[0] == 6
            names = [bytes(t.nblob[t.noff[i]:t.noff[i + 1]]) for i in t.pidx[x[7]]]
            sb, so = W.pack(names)
            t0 = time.perf_counter()
            O.sg_batch_v4_np(t.tcp, t.udp, False, x[1][~six], x[2][~six].view(np.uint32),
                             x[6][~six].view(np.uint16), nthreads=threads)
            O.sg_batch_v6_np(t.tcp, t.udp, False, x[1][six], x[4][six], x[6][six].view(np.uint16),
                             nthreads=threads)
            O.rt_batch_v4_np(t.v4_list, x[3][~six].view(np.uint32), nthreads=threads)
            O.rt_batch_v6_np(t.v6_list, x[5][six], nthreads=threads)
            O.hint_batch_np(og, sb, so, None, nthreads=threads)
            return time.perf_counter() - t0
        cpu = cpu_rates(run, "M classifications/s", 4.0, "the first packets of the mixed batch, "
                        "oracle linear scans (v4 / v6 SecurityGroup lists, rulesV4 / rulesV6, "
                        "searchForGroup per packet)")
    res = {"workload": args.workload, "items": n, "ms_per_step": round(el / args.steps * 1e3, 3),
           "kernel_ms": round(ms, 4), "M_items_per_s": round(n / (ms / 1e3) / 1e6, 1),
           "roofline": {"bound": "hbm", "achieved": round(gbs, 2), "peak": HBM_PEAK_GBS,
                        "unit": "GB/s", "frac": round(gbs / HBM_PEAK_GBS, 5), "kernel": kern,
                        "algorithmic_bytes": unit},
           "cpu_baseline": cpu}
    res.update(extra)
    res["v6_frac"] = args.v6_frac
    res["compact6"] = bool(args.compact6)
    replicas(res, world, dev)
    if rank == 0:
        print(json.dumps(res), flush=True)
    clf.close()


if __name__ == "__main__":
    main()

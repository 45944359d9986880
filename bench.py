#!/usr/bin/env python3
"""Headline benchmark: M classifications/s (ACL + route + host) per BASELINE.json.

Default workload (`--workload c5`, SURVEY.md §8(d) C5, per-GPU shard, weak
scaling): every rank holds the replicated tables
    SecurityGroup   10k rules with port ranges (C2 generator)
    RouteTable      ~1M IPv4 + 200k IPv6 prefixes inserted shortest-first (C3)
    Upstream        100k hint-host groups (C4), hostname pool of 16M
and classifies, per step, 125M IPv4 packets resident in HBM:
    1. the hostname pool once (Upstream.searchForGroup per hostname)
    2. the fused pipeline kernel per packet: SecurityGroup.allow(src, dport)
       -> RouteTable.lookup(dst) -> pool group of the packet's host id
    3. per-rule hit counters (ACL, route, group), RCCL all-reduce when N > 1.
A "classification" is one packet through all three.  Inputs are synthetic
and generated on the device; nothing is cached between steps.

Other workloads (c2, c3, c4) time one classifier alone for DESIGN.md.

Launch: python bench.py [--gpus N --steps K --warmup W]; for N > 1 under
torch.distributed.run (one rank per GPU, RCCL).
"""
import argparse
import ctypes as C
import json
import os
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

import vproxy_amd as V  # noqa: E402
from vproxy_amd import workloads as W  # noqa: E402
from vproxy_amd.dist import HitCounterBucket  # noqa: E402

METRIC = "M classifications/sec (ACL+LPM+host) at 1/2/4/8 MI355X; % HBM roofline"
HBM_PEAK_GBS = 8000.0          # MI355X_MICROARCH.md chip table (spec)
PROFILES = os.path.join(ROOT, "profiles")


def log(*a):
    if int(os.environ.get("RANK", "0")) == 0:
        print("[bench]", *a, file=sys.stderr, flush=True)


# ---------------------------------------------------------------------------
# device-side synthetic inputs
# ---------------------------------------------------------------------------
def dev_u32(x):
    """int64 tensor holding uint32 values -> int32 tensor with the same bits."""
    x = x & 0xFFFFFFFF
    return torch.where(x >= 2**31, x - 2**32, x).to(torch.int32)


def gen_packets(n, tcp, udp, net, plen, pool_n, seed, dev):
    g = torch.Generator(device=dev)
    g.manual_seed(seed)
    ri = lambda lo, hi, k: torch.randint(lo, hi, (k,), generator=g, device=dev, dtype=torch.int64)
    proto = torch.where(ri(0, 2, n) == 0, 6, 17).to(torch.uint8)
    src = ri(0, 2**32, n)
    port = ri(0, 65536, n)
    pick = ri(0, 2, n) == 0
    # half the packets hit a rule of their protocol (network + port range)
    for p, rules in ((6, tcp), (17, udp)):
        ip, mk = W.rule_v4_fields(rules)
        ipd = torch.from_numpy(ip.astype(np.int64)).to(dev)
        mkd = torch.from_numpy(mk.astype(np.int64)).to(dev)
        lo = torch.from_numpy(rules["min_port"].astype(np.int64)).to(dev)
        hi = torch.from_numpy(rules["max_port"].astype(np.int64)).to(dev)
        r = ri(0, len(rules), n)
        sel = pick & (proto == p)
        src = torch.where(sel, ipd[r] | (src & (~mkd[r] & 0xFFFFFFFF)), src)
        span = hi[r] - lo[r] + 1
        port = torch.where(sel, lo[r] + (ri(0, 2**31, n) % span), port)
        del r, span
    # 90 % of destinations inside a route prefix
    netd = torch.from_numpy(net.astype(np.int64)).to(dev)
    mkd = torch.from_numpy(W._mask32(plen).astype(np.int64)).to(dev)
    r = ri(0, len(net), n)
    dst = ri(0, 2**32, n)
    dst = torch.where(ri(0, 10, n) < 9, netd[r] | (dst & (~mkd[r] & 0xFFFFFFFF)), dst)
    hid = ri(0, pool_n, n)
    out = (proto, dev_u32(src), dev_u32(dst), port.to(torch.int32).to(torch.int16),
           hid.to(torch.int32))
    return out


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
# CPU baseline (oracle, test-infrastructure C restatement of the Java scans)
# ---------------------------------------------------------------------------
def cpu_baseline_c5(tcp, udp, v4_list, groups, names_blob, names_off, seed, threads,
                    budget_s=12.0):
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    import oracle_ffi as O
    og = O.Groups(groups)

    def run(n):
        proto, src, port = W.gen_acl_queries(tcp, udp, n, seed)
        dst = W.v4_lookups(v4_ip, v4_plen, n, seed + 1)
        hid = np.random.default_rng(seed + 2).integers(0, len(names_off) - 1, n)
        sub_blob, sub_off = W.pack([bytes(names_blob[names_off[i]:names_off[i + 1]]) for i in hid])
        t0 = time.perf_counter()
        O.sg_batch_v4_np(tcp, udp, False, proto, src, port, nthreads=threads)
        O.rt_batch_v4_np(v4_list, dst, nthreads=threads)
        O.hint_batch_np(og, sub_blob, sub_off, None, nthreads=threads)
        return time.perf_counter() - t0

    v4_ip = v4_list["ip"][:, :4].copy().view(">u4").reshape(-1).astype(np.uint32)
    v4_plen = np.array([bin(int(x)).count("1") for x in
                        v4_list["mask"][:, :4].copy().view(">u4").reshape(-1)])
    probe = max(threads * 4, 64)
    t = run(probe)
    n = int(min(65536, max(probe, probe * budget_s / max(t, 1e-6))))
    t = run(n)
    return {"value": n / t / 1e6, "unit": "M classifications/s", "cores": threads,
            "kind": "port",
            "sample": "%d packets of the same C5 workload (ACL 10k rules + RouteTable %d IPv4 "
                      "rules + Upstream %d groups), oracle linear scans as the Java code does "
                      "them, %d threads, %.1f s" % (n, len(v4_list), len(groups), threads, t)}


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


def hip_stream(dev):
    """A fresh non-blocking HIP stream wrapped for torch.  HIP spreads the
    streams a process creates round-robin over its hardware queues; three
    created back to back land on three queues, so the kernels on them can
    run concurrently (torch's pooled streams shared a queue here)."""
    hip = C.CDLL("libamdhip64.so")
    h = C.c_void_p()
    rc = hip.hipStreamCreateWithFlags(C.byref(h), C.c_uint(1))      # hipStreamNonBlocking
    assert rc == 0, rc
    return torch.cuda.ExternalStream(h.value, device=dev)


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


def load_traffic(workload, kernel):
    """Per-launch HBM-side bytes of `kernel` from the committed PMC passes
    (profiles/pmc_traffic.json, written by scripts/pmc_traffic.py from
    separate rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE runs of this bench)."""
    p = os.path.join(PROFILES, "pmc_traffic.json")
    try:
        with open(p) as f:
            d = json.load(f)
        return d[workload]["kernels"][kernel]["traffic_bytes"]
    except (OSError, ValueError, KeyError):
        return None


# ---------------------------------------------------------------------------
def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--workload", default="c5",
                    choices=["c5", "c2", "c2host", "c3", "c4", "dns", "sni", "parse", "source",
                             "mirror"])
    ap.add_argument("--packets", type=int, default=125_000_000, help="per GPU per step (c5)")
    ap.add_argument("--pool", type=int, default=16 << 20, help="hostname pool (c5/c4)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-counters", action="store_true", help="ablation: skip hit counters")
    ap.add_argument("--counters", choices=["fused", "passes"], default="fused",
                    help="fused: the pipeline kernel counts ACL hits and route/group buckets "
                         "itself and the library finishes the large spaces; passes: separate "
                         "counting passes over the outputs (counters_add)")
    ap.add_argument("--serial", action="store_true",
                    help="ablation: one stream, no overlap between consecutive batches")
    ap.add_argument("--overlap", choices=["finish", "pipeline"], default="pipeline",
                    help="what the next batch's hostname-pool pass overlaps: the counter finish "
                         "passes of this batch (it waits for this batch's pipeline kernel), or "
                         "the pipeline kernel itself (both are bound by the same random "
                         "gathers)")
    args = ap.parse_args()

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        log("note: --gpus %d but WORLD_SIZE %d; using WORLD_SIZE" % (args.gpus, world))
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    if world > 1:
        import torch.distributed as dist
        dist.init_process_group("nccl", device_id=dev)
    clf = V.Classifier(local)

    if args.workload != "c5":
        return sub_bench(args, clf, dev, rank, world)

    t_setup = time.time()
    # ---- replicated tables (same seeds on every rank) ----
    tcp, udp = W.gen_sg_rules(10000, W.SEED + 2, p_range=0.3)
    a, na, ka = W.as_ctypes(tcp, V._lib.VcAclRule)
    b, nb, kb = W.as_ctypes(udp, V._lib.VcAclRule)
    V.check(V.lib().vc_compile_acl(clf.h, a, na, b, nb, 0))
    net, plen = W.gen_v4_prefixes(1_000_000, W.SEED + 3)
    hi, lo, p6 = W.gen_v6_prefixes(200_000, W.SEED + 4)
    rt = V.RouteTable()
    allnets = np.concatenate([W.v4_nets(net, plen), W.v6_nets(hi, lo, p6)])
    arr, n_all, keep = W.as_ctypes(allnets, V._lib.VcNet)
    rt.add_rules("bgp", arr, n=n_all)
    clf.compile_route_table(rt)
    a4, n4 = rt.rules_raw(4)
    v4_list = np.frombuffer(bytes(a4)[:n4 * 40], W.NET_DT)
    groups, ghosts = W.gen_groups(100_000, W.SEED + 5)
    clf.compile_upstream(groups)
    names = W.gen_hostnames(ghosts, 1 << 20, W.SEED + 6)            # distinct pool source
    nblob, noff = W.pack(names)
    pidx = np.random.default_rng(W.SEED + 7 + rank).integers(0, len(names), args.pool)
    pool_blob, pool_off, pool_bytes = gather_strings_dev(nblob, noff, pidx, dev)
    pool_out = torch.empty(args.pool, dtype=torch.int32, device=dev)
    log("tables built in %.1fs (acl %d+%d, routes %d+%d, groups %d, pool %d names %.0f MB)" % (
        time.time() - t_setup, len(tcp), len(udp), n4, len(hi), len(groups), args.pool,
        pool_bytes / 1e6))

    B = args.packets
    proto, src, dst, dport, hid = gen_packets(B, tcp, udp, net, plen, args.pool,
                                              1234 + rank, dev)
    # Two batches in flight: outputs and pool results are double-buffered so
    # batch j's hit counters (and batch j+1's hostname pool) run on their own
    # streams while batch j+1's pipeline runs.  Every step still does all of
    # its work inside the timed region.
    nbuf = 1 if args.serial else 2
    pools = [pool_out] + [torch.empty_like(pool_out) for _ in range(nbuf - 1)]
    outsb = [tuple(torch.empty(B, dtype=torch.int32, device=dev) for _ in range(3)) + (None,)
             for _ in range(nbuf)]
    torch.cuda.synchronize()
    log("packets generated (%d per GPU), setup %.1fs" % (B, time.time() - t_setup))

    # Hit counters: the library's histogram passes over each batch's outputs,
    # scheduled explicitly (counters_add) on the counting stream.
    count = not args.no_counters
    fused = count and args.counters == "fused"
    clf.counters_enable(False)
    csrc = [clf.counters_device(k) for k in (V.COUNTERS_ACL, V.COUNTERS_ROUTE, V.COUNTERS_GROUP)]
    bucket = HitCounterBucket([n for _, n in csrc], dev) if world > 1 else None
    if args.serial:
        s_pipe = s_hint = s_cnt = torch.cuda.current_stream()
    else:
        s_pipe, s_hint, s_cnt = (hip_stream(dev) for _ in range(3))
    ev_hint, ev_pipe, ev_cnt, kdone = {}, {}, {}, {}
    timing = []                     # (hint, pipe, count) event pairs of timed steps
    TE = lambda: torch.cuda.Event(enable_timing=True)

    def hint(j, rec):
        with torch.cuda.stream(s_hint):
            if j - nbuf in ev_pipe:               # pool buffer no longer read
                s_hint.wait_event(ev_pipe[j - nbuf])
            if args.overlap == "finish" and j - 1 in kdone:
                kdone[j - 1].wait(s_hint)          # after the previous pipeline kernel
            e0, e1 = TE(), TE()
            e0.record()
            V.check(V.lib().vc_hint_search_dev(clf.h, C.c_void_p(pool_blob.data_ptr()),
                                               C.c_void_p(pool_off.data_ptr()), None, None, None,
                                               None, None, args.pool,
                                               C.c_void_p(pools[j % nbuf].data_ptr()),
                                               C.c_void_p(s_hint.cuda_stream)))
            e1.record()
            ev_hint[j] = e1
            rec["hint"] = (e0, e1)

    def pipe(j, rec):
        with torch.cuda.stream(s_pipe):
            s_pipe.wait_event(ev_hint[j])
            if j - nbuf in ev_cnt:                # output buffers counted
                s_pipe.wait_event(ev_cnt[j - nbuf])
            k0, k1 = RawEvent(), RawEvent()       # the classify kernel alone
            e1 = TE()
            k0.record(s_pipe)
            if fused:                              # count packets only, not the pool pass
                clf.counters_enable(True)
            clf.pipeline_v4(proto, src, dst, dport, hid, pools[j % nbuf], outs=outsb[j % nbuf],
                            kernel_done_event=k1.h.value)
            if fused:
                clf.counters_enable(False)
            k2 = RawEvent()                       # + in-library counter passes (fused)
            k2.record(s_pipe)
            e1.record()
            ev_pipe[j] = e1
            kdone[j] = k1
            rec["pipe"] = (k0, k1)
            rec["pipe_call"] = (k1, k2)

    def counters(j, rec):
        outs = outsb[j % nbuf]
        with torch.cuda.stream(s_cnt):
            s_cnt.wait_event(ev_pipe[j])
            e0, e1 = TE(), TE()
            e0.record()
            if count and not fused:
                clf.counters_add(V.COUNTERS_ACL, outs[0], aux=proto)
                clf.counters_add(V.COUNTERS_ROUTE, outs[1], family=4)
                clf.counters_add(V.COUNTERS_GROUP, outs[2])
            e1.record()
            if bucket is not None:                # one RCCL all-reduce per batch
                for i, cs in enumerate(csrc):
                    bucket.fill(i, cs)
                bucket.reduce()
            done = torch.cuda.Event()
            done.record()
            ev_cnt[j] = done
            rec["count"] = (e0, e1)

    def run(first, k, timed):
        """Steps first .. first+k-1; step j = hint(j), pipe(j), counters(j).
        The hostname pool of the next step is issued before this step's
        counters, so it overlaps this step's pipeline."""
        if k <= 0:
            return
        recs = [dict() for _ in range(k)]
        hint(first, recs[0])
        for i in range(k):
            j = first + i
            pipe(j, recs[i])
            if i + 1 < k:
                hint(j + 1, recs[i + 1])
            counters(j, recs[i])
        if timed:
            timing.extend(recs)

    run(0, args.warmup, False)
    torch.cuda.synchronize()
    ev_hint.clear(); ev_pipe.clear(); ev_cnt.clear(); kdone.clear()
    if world > 1:
        import torch.distributed as dist
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    run(args.warmup, args.steps, True)
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    elapsed = time.perf_counter() - t0
    if world > 1:
        t = torch.tensor([elapsed], dtype=torch.float64, device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())

    span = lambda key: float(np.mean([r[key][0].elapsed_time(r[key][1]) for r in timing]))
    hint_ms, pipe_ms = span("hint"), span("pipe")
    count_ms = span("pipe_call") if fused else span("count")
    total = float(B) * world * args.steps
    value = total / elapsed / 1e6
    # roofline of the dominant kernel, algorithmic bytes only
    if pipe_ms >= hint_ms:
        dom, per_unit, units, ms = "pipeline_v4_kernel", 27, B, pipe_ms
        unit_desc = "27 B/packet (proto 1 + src 4 + dst 4 + dport 2 + host_id 4 in; 3x int32 out)"
    else:
        dom, ms, units = "hint_kernel", hint_ms, args.pool
        per_unit = (pool_bytes / args.pool) + 4 + 4
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
    roof = {"bound": "hbm", "achieved": round(achieved, 2), "peak": HBM_PEAK_GBS, "unit": "GB/s",
            "frac": round(achieved / HBM_PEAK_GBS, 5), "traffic": load_traffic("c5", dom),
            "kernel": dom, "kernel_ms": round(ms, 4), "algorithmic_bytes": unit_desc,
            "gather_bound": gather_bound,
            "other_kernel_ms": {"hint_kernel": round(hint_ms, 4),
                                "pipeline_v4_kernel": round(pipe_ms, 4),
                                "hit_counter_passes": round(count_ms, 4),
                                "counting": ("in the pipeline kernel (ACL + route/group "
                                             "buckets) + library passes for the large spaces"
                                             if fused else "separate passes")}}
    cpu = None
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        threads = min(16, os.cpu_count() or 1)
        cpu = cpu_baseline_c5(tcp, udp, v4_list, groups, nblob, noff, 99, threads)
    if rank == 0:
        line = {"metric": METRIC, "value": round(value, 3), "unit": "M classifications/s",
                "n_gpus": world, "steps": args.steps, "warmup": args.warmup,
                "ms_per_step": round(elapsed / args.steps * 1e3, 3), "higher_is_better": True,
                "scaling": "weak", "vs_baseline": None, "dtype": "u32",
                "data": "synthetic (seeded, generated on device)",
                "config": {"workload": "C5 combined ACL->route->host pipeline, per-GPU shard",
                           "acl_rules": int(len(tcp) + len(udp)), "routes_v4": int(n4),
                           "routes_v6": int(len(hi)), "groups": len(groups),
                           "hostname_pool": args.pool, "packets_per_gpu_per_step": B,
                           "parallelism": "dp%d" % world,
                           "schedule": ("serial, one stream" if args.serial else
                                        "2 batches in flight: pool / pipeline / counters on "
                                        "3 HIP streams; the next pool pass overlaps the %s" %
                                        ("counter finish" if args.overlap == "finish"
                                         else "pipeline kernel"))},
                "roofline": roof, "cpu_baseline": cpu}
        print(json.dumps(line), flush=True)
    clf.close()
    if world > 1:
        dist.destroy_process_group()


def sub_bench(args, clf, dev, rank, world):
    """Single-classifier benchmarks (DESIGN.md numbers), not the headline."""
    res = {}
    ev = []
    if args.workload == "c2":
        tcp, udp = W.gen_sg_rules(10000, W.SEED + 2, p_range=0.3)
        a, na, ka = W.as_ctypes(tcp, V._lib.VcAclRule)
        b, nb, kb = W.as_ctypes(udp, V._lib.VcAclRule)
        V.check(V.lib().vc_compile_acl(clf.h, a, na, b, nb, 0))
        n = 64 << 20
        net, plen = W.gen_v4_prefixes(1000, 1)
        proto, src, dst, dport, hid = gen_packets(n, tcp, udp, net, plen, 1, 5 + rank, dev)
        out = torch.empty(n, dtype=torch.int32, device=dev)
        fn = lambda: clf.acl_v4(proto, src, dport, out_idx=out, want_allow=False)
        per_unit, unit = 11, "B/tuple (7 in + 4 out)"
    elif args.workload == "c3":
        net, plen = W.gen_v4_prefixes(1_000_000, W.SEED + 3)
        hi, lo, p6 = W.gen_v6_prefixes(200_000, W.SEED + 4)
        rt = V.RouteTable()
        allnets = np.concatenate([W.v4_nets(net, plen), W.v6_nets(hi, lo, p6)])
        arr, n_all, keep = W.as_ctypes(allnets, V._lib.VcNet)
        rt.add_rules("bgp", arr, n=n_all)
        clf.compile_route_table(rt)
        n = 256 << 20
        n4 = int(n * 0.85)
        g = torch.Generator(device=dev)
        g.manual_seed(7 + rank)
        netd = torch.from_numpy(net.astype(np.int64)).to(dev)
        mkd = torch.from_numpy(W._mask32(plen).astype(np.int64)).to(dev)
        r = torch.randint(0, len(net), (n4,), generator=g, device=dev)
        q = torch.randint(0, 2**32, (n4,), generator=g, device=dev)
        q4 = dev_u32(torch.where(torch.rand(n4, generator=g, device=dev) < 0.9,
                                 netd[r] | (q & (~mkd[r] & 0xFFFFFFFF)), q))
        del r, q
        q6 = torch.from_numpy(W.v6_lookups(hi, lo, p6, n - n4, 8 + rank)).to(dev)
        o4 = torch.empty(n4, dtype=torch.int32, device=dev)
        o6 = torch.empty(n - n4, dtype=torch.int32, device=dev)
        fn = lambda: (clf.route_v4(q4, out=o4), clf.route_v6(q6, out=o6))
        per_unit, unit = (8 * 0.85 + 20 * 0.15), "B/lookup (v4 4+4, v6 16+4, 85/15 mix)"
    elif args.workload == "c2host":
        # the plain (host-buffer) entry point: H2D copy + kernel + D2H copy
        # per call, from page-locked buffers (vc_host_register)
        tcp, udp = W.gen_sg_rules(10000, W.SEED + 2, p_range=0.3)
        a, na, ka = W.as_ctypes(tcp, V._lib.VcAclRule)
        b, nb, kb = W.as_ctypes(udp, V._lib.VcAclRule)
        V.check(V.lib().vc_compile_acl(clf.h, a, na, b, nb, 0))
        n = 64 << 20
        proto, src, port = W.gen_acl_queries(tcp, udp, n, W.SEED + 16)
        out = np.empty(n, np.int32)
        allow = np.empty(n, np.uint8)
        bufs = (proto, src, port, out, allow)
        for x in bufs:
            V.check(V.lib().vc_host_register(C.c_void_p(x.ctypes.data), x.nbytes))
        P = lambda x: C.c_void_p(x.ctypes.data)
        fn = lambda: V.check(V.lib().vc_acl_classify_v4(clf.h, P(proto), P(src), P(port), n,
                                                          P(out), P(allow)))
        per_unit, unit = 12, "B/tuple across PCIe (7 in + 5 out), kernel included"
    elif args.workload == "dns":
        groups, ghosts = W.gen_groups(100_000, W.SEED + 5)
        clf.compile_upstream(groups)
        hosts = "\n".join("10.0.%d.%d h%d.hosts.local" % (i >> 8 & 255, i & 255, i)
                           for i in range(50_000))
        clf.compile_hosts_text(hosts)
        names = W.gen_hostnames(ghosts, 1 << 20, W.SEED + 6, dns=True, port_frac=0)
        nblob, noff = W.pack(names)
        n = 16 << 20
        pidx = np.random.default_rng(W.SEED + 8).integers(0, len(names), n)
        blob, off, nbytes = gather_strings_dev(nblob, noff, pidx, dev)
        kind = torch.empty(n, dtype=torch.uint8, device=dev)
        val = torch.empty(n, dtype=torch.int32, device=dev)
        s = lambda: C.c_void_p(torch.cuda.current_stream().cuda_stream)
        fn = lambda: V.check(V.lib().vc_dns_classify_dev(
            clf.h, C.c_void_p(blob.data_ptr()), C.c_void_p(off.data_ptr()), n,
            C.c_void_p(kind.data_ptr()), C.c_void_p(val.data_ptr()), s()))
        per_unit, unit = nbytes / n + 9, "B/qname (bytes + 4 offset + 1 kind + 4 value)"
    elif args.workload == "sni":
        _, hosts = W.gen_groups(200_000, W.SEED + 9, wildcard=False)
        holders = [[hosts[i], "*." + hosts[i + 1]] for i in range(0, len(hosts), 2)]
        clf.compile_certs(holders)
        names = [x.split(b":")[0] for x in W.gen_hostnames(hosts, 1 << 20, W.SEED + 10)]
        nblob, noff = W.pack(names)
        n = 16 << 20
        pidx = np.random.default_rng(W.SEED + 11).integers(0, len(names), n)
        blob, off, nbytes = gather_strings_dev(nblob, noff, pidx, dev)
        out = torch.empty(n, dtype=torch.int32, device=dev)
        s = lambda: C.c_void_p(torch.cuda.current_stream().cuda_stream)
        fn = lambda: V.check(V.lib().vc_cert_choose_dev(
            clf.h, C.c_void_p(blob.data_ptr()), C.c_void_p(off.data_ptr()), None, n,
            C.c_void_p(out.data_ptr()), s()))
        per_unit, unit = nbytes / n + 8, "B/SNI (bytes + 4 offset + 4 out)"
    elif args.workload in ("parse", "mirror"):
        frames = W.gen_vxlan_frames(1 << 16, W.SEED + 12)
        fblob, foff = W.pack(frames)
        n = 32 << 20
        pidx = np.random.default_rng(W.SEED + 13).integers(0, len(frames), n)
        blob, off, nbytes = gather_strings_dev(fblob, foff, pidx, dev)
        s = lambda: C.c_void_p(torch.cuda.current_stream().cuda_stream)
        if args.workload == "parse":
            res = {k: torch.empty((n, w) if w > 1 else (n,), dtype={"u8": torch.uint8,
                   "u16": torch.int16, "u32": torch.int32}[t], device=dev)
                   for k, w, t in V.Classifier._PKT_FIELDS}
            o = V._lib.VcPktOut(**{k: v.data_ptr() for k, v in res.items()})
            fn = lambda: V.check(V.lib().vc_parse_packets_dev(
                clf.h, C.c_void_p(blob.data_ptr()), C.c_void_p(off.data_ptr()), n, 0,
                C.byref(o), s()))
            per_unit = nbytes / n + 4 + 54
            unit = "B/frame (frame bytes + 4 offset in; 54 B of SoA fields out)"
        else:
            from vproxy_amd.mirror import MirrorFilters  # noqa: F401
            filters = [{"origin": "switch", "mirror": i % 8, "network": "%d.0.0.0/8" % (i + 1),
                        "network2": "10.0.0.0/8"} for i in range(16)] + \
                      [{"origin": "switch", "mirror": 9, "mac": "0a:00:27:00:00:01"}]
            mf = clf.compile_mirror(filters)
            out = torch.empty(n, dtype=torch.int64, device=dev)
            oid = mf.id_of("switch", create=False)
            fn = lambda: V.check(V.lib().vc_mirror_switch_dev(
                clf.h, oid, C.c_void_p(blob.data_ptr()), C.c_void_p(off.data_ptr()), n, 0,
                C.c_void_p(out.data_ptr()), s()))
            per_unit = nbytes / n + 4 + 8
            unit = "B/frame (frame bytes + 4 offset in; 8 B mirror set out), 17 filters"
    elif args.workload == "source":
        rng = np.random.default_rng(W.SEED + 14)
        groups = [[(bytes(rng.integers(0, 256, 4).astype(np.uint8)), 80, 1, rng.random() < 0.9)
                   for _ in range(int(rng.integers(1, 32)))] for _ in range(10_000)]
        clf.compile_servers(groups)
        n = 128 << 20
        g = torch.Generator(device=dev)
        g.manual_seed(15)
        grp = torch.randint(0, len(groups), (n,), generator=g, device=dev, dtype=torch.int32)
        src = torch.randint(-2**31, 2**31 - 1, (n,), generator=g, device=dev, dtype=torch.int32)
        out = torch.empty(n, dtype=torch.int32, device=dev)
        s = lambda: C.c_void_p(torch.cuda.current_stream().cuda_stream)
        fn = lambda: V.check(V.lib().vc_source_select_v4_dev(
            clf.h, C.c_void_p(grp.data_ptr()), C.c_void_p(src.data_ptr()), n, 0,
            C.c_void_p(out.data_ptr()), s()))
        per_unit, unit = 12, "B/item (group 4 + v4 source 4 in, 4 out)"
    else:  # c4
        groups, ghosts = W.gen_groups(100_000, W.SEED + 5)
        clf.compile_upstream(groups)
        names = W.gen_hostnames(ghosts, 1 << 20, W.SEED + 6)
        nblob, noff = W.pack(names)
        n = 16 << 20
        pidx = np.random.default_rng(W.SEED + 7).integers(0, len(names), n)
        blob, off, nbytes = gather_strings_dev(nblob, noff, pidx, dev)
        out = torch.empty(n, dtype=torch.int32, device=dev)
        s = lambda: C.c_void_p(torch.cuda.current_stream().cuda_stream)
        fn = lambda: V.check(V.lib().vc_hint_search_dev(
            clf.h, C.c_void_p(blob.data_ptr()), C.c_void_p(off.data_ptr()), None, None, None,
            None, None, n, C.c_void_p(out.data_ptr()), s()))
        per_unit, unit = nbytes / n + 8, "B/hostname (bytes + 4 offset + 4 out)"
    for _ in range(args.warmup):
        fn()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        e0 = torch.cuda.Event(enable_timing=True)
        e1 = torch.cuda.Event(enable_timing=True)
        e0.record()
        fn()
        e1.record()
        ev.append((e0, e1))
    torch.cuda.synchronize()
    el = time.perf_counter() - t0
    ms = float(np.mean([a.elapsed_time(b) for a, b in ev]))
    gbs = per_unit * n / (ms / 1e3) / 1e9
    res = {"workload": args.workload, "items": n, "ms_per_step": round(el / args.steps * 1e3, 3),
           "kernel_ms": round(ms, 4), "M_items_per_s": round(n / (ms / 1e3) / 1e6, 1),
           "algorithmic_GBps": round(gbs, 2), "frac_of_8TBps": round(gbs / HBM_PEAK_GBS, 5),
           "bytes_per_item": unit}
    if rank == 0:
        print(json.dumps(res), flush=True)
    clf.close()


if __name__ == "__main__":
    main()

"""Design experiment (not product code): how the C5 kernels scale with the
CUs they hold, and what the pool pass costs beside the pipeline kernel when
the two hold disjoint CU sets.

tools/gather_paths.hip shows the random-gather rate of the chip capped
globally (about 56 G gathers/s, reached with 128 of 256 CUs), so a kernel
bound only by that cap should lose nothing on fewer CUs.  This script
times, on CU-masked streams (hipExtStreamCreateWithCUMask):
  - pipeline_v4_kernel (no counting) and the pool pass (hint_kernel) alone
    on k CUs, k = 64 .. 256, the k CUs chosen two ways: `blocks` (the first
    k/8 ids of each 32-id block) and `spread` (every 256/k-th id), which
    differ in XCD placement if CU ids interleave over the XCDs;
  - both kernels at once on complementary sets (pipeline on k, pool pass on
    256 - k), the wall time from the first start to the last end.

Usage (GPU box): python scripts/cu_scaling.py > gpurun_out/cu_scaling.jsonl
"""
import ctypes as C
import json
import os
import sys
import time

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))

import torch  # noqa: E402

import bench  # noqa: E402
import vproxy_amd as V  # noqa: E402


def sel(kind, k, total=256):
    if kind == "spread":
        return bench.cu_split(total, k)[0]
    if kind == "contig":                 # bits [0, k): k / 8 CUs of every XCD
        return list(range(k))
    per = k // 8
    return [b * 32 + i for b in range(total // 32) for i in range(per)]


def main():
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    clf = V.Classifier(0)
    t = bench.c5_tables(clf, dev)
    B = 125_000_000
    proto, src, dst, dport, hid = bench.gen_packets(0, B, t, t.pool_n, dev=dev)
    pool = torch.empty(t.pool_n, dtype=torch.int32, device=dev)
    outs = tuple(torch.empty(B, dtype=torch.int32, device=dev) for _ in range(3)) + (None,)
    ncu = torch.cuda.get_device_properties(dev).multi_processor_count
    clf.counters_enable(False)

    def hint(stream):
        V.check(V.lib().vc_hint_search_dev(
            clf.h, C.c_void_p(t.pool_blob.data_ptr()), C.c_void_p(t.pool_off.data_ptr()),
            None, None, None, None, None, t.pool_n, C.c_void_p(pool.data_ptr()),
            C.c_void_p(stream.cuda_stream)))

    def pipe(stream):
        with torch.cuda.stream(stream):
            clf.pipeline_v4(proto, src, dst, dport, hid, pool, outs=outs)

    def timed(fn, stream, reps=5):
        ms = []
        for _ in range(reps):
            a, b = bench.RawEvent(), bench.RawEvent()
            a.record(stream)
            fn(stream)
            b.record(stream)
            torch.cuda.synchronize()
            ms.append(a.elapsed_time(b))
        ms.sort()
        return ms[len(ms) // 2]

    hint(torch.cuda.current_stream())
    torch.cuda.synchronize()
    full = bench.hip_stream(dev)
    base = {"pipe": timed(pipe, full), "hint": timed(hint, full)}
    print(json.dumps({"probe": "alone", "cus": ncu, "sel": "all", **base}), flush=True)
    for kind in ("contig",):
        for k in (96, 160, 192, 208, 224, 240):
            s = bench.hip_stream(dev, sel(kind, k, ncu))
            r = {"pipe": timed(pipe, s), "hint": timed(hint, s)}
            if kind == "contig":     # the pool pass alone on the other CUs
                r["hint_rest"] = timed(hint, bench.hip_stream(dev, list(range(k, ncu))))
            print(json.dumps({"probe": "alone", "cus": k, "sel": kind, **r}), flush=True)
    for k in (160, 176, 192, 200, 208, 216, 224, 232, 240):
        mine = sel("contig", k, ncu)
        rest = [c for c in range(ncu) if c not in set(mine)]
        sp, sh = bench.hip_stream(dev, mine), bench.hip_stream(dev, rest)
        walls, pms, hms = [], [], []
        for _ in range(5):
            torch.cuda.synchronize()
            a0, a1, b0, b1 = (bench.RawEvent() for _ in range(4))
            t0 = time.perf_counter()
            a0.record(sp)
            pipe(sp)
            a1.record(sp)
            b0.record(sh)
            hint(sh)
            b1.record(sh)
            torch.cuda.synchronize()
            walls.append((time.perf_counter() - t0) * 1e3)
            pms.append(a0.elapsed_time(a1))
            hms.append(b0.elapsed_time(b1))
        med = lambda x: sorted(x)[len(x) // 2]
        print(json.dumps({"probe": "together", "pipe_cus": k, "hint_cus": ncu - k,
                          "pipe": med(pms), "hint": med(hms), "wall_host": med(walls),
                          "serial_full": base["pipe"] + base["hint"]}), flush=True)
    clf.close()


if __name__ == "__main__":
    main()

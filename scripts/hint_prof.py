"""Phase breakdown of the hint and DNS kernels (profiling build).

Build the profiling library first (on the CPU side):
    make -C vproxy_amd/csrc OUT=../../build/prof/libvclassify.so \
         BUILD=../../build/objprof EXTRA=-DVC_HINT_PROF
then on the GPU box:
    python scripts/hint_prof.py
Prints, per kernel, the per-wave cycles of each phase (clock64 marks in
hint.hip / hint_dev.h) over the C4 and DNS sub-bench workloads, and the
wave-level name-length statistics that set the scan's trip count.
"""
import ctypes as C
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
os.environ.setdefault("VCLASSIFY_LIB", os.path.join(ROOT, "build", "prof", "libvclassify.so"))
sys.path.insert(0, ROOT)

import numpy as np  # noqa: E402
import torch  # noqa: E402

import bench  # noqa: E402
import vproxy_amd as V  # noqa: E402
from vproxy_amd import workloads as W  # noqa: E402

PHASES = ["stage", "scan", "tag_groups", "records", "dns_hosts", "output"]


def read_prof():
    buf = (C.c_ulonglong * 7)()
    fn = V.lib().vc_debug_hint_prof
    fn.argtypes = [C.c_void_p]
    fn.restype = C.c_int
    assert fn(C.cast(buf, C.c_void_p)) == 0
    return list(buf)


def wave_stats(off):
    lens = np.diff(off.astype(np.int64))
    n = len(lens) // 64 * 64
    w = lens[:n].reshape(-1, 64)
    words = (w + 3) // 4
    return {"mean_len": float(lens.mean()), "mean_wave_max_len": float(w.max(1).mean()),
            "mean_words": float(words.mean()), "mean_wave_max_words": float(words.max(1).mean())}


def main():
    dev = torch.device("cuda:0")
    torch.cuda.set_device(dev)
    for wl in ("c4", "dns"):
        clf = V.Classifier()
        groups, ghosts = W.gen_groups(100_000, W.SEED + 5)
        clf.compile_upstream(groups)
        dns = wl == "dns"
        if dns:
            clf.compile_hosts_text("\n".join("10.0.%d.%d h%d.hosts.local" % (i >> 8 & 255, i & 255, i)
                                             for i in range(50_000)))
            names = W.gen_hostnames(ghosts, 1 << 20, W.SEED + 6, dns=True, port_frac=0)
        else:
            names = W.gen_hostnames(ghosts, 1 << 20, W.SEED + 6)
        nblob, noff = W.pack(names)
        n = 16 << 20
        pidx = np.random.default_rng(W.SEED + (8 if dns else 7)).integers(0, len(names), n)
        blob, off, _ = bench.gather_strings_dev(nblob, noff, pidx, dev)
        S = C.c_void_p(torch.cuda.current_stream().cuda_stream)
        if dns:
            kind = torch.empty(n, dtype=torch.uint8, device=dev)
            val = torch.empty(n, dtype=torch.int32, device=dev)
            fn = lambda: V.check(V.lib().vc_dns_classify_dev(
                clf.h, C.c_void_p(blob.data_ptr()), C.c_void_p(off.data_ptr()), n,
                C.c_void_p(kind.data_ptr()), C.c_void_p(val.data_ptr()), S))
        else:
            out = torch.empty(n, dtype=torch.int32, device=dev)
            fn = lambda: V.check(V.lib().vc_hint_search_dev(
                clf.h, C.c_void_p(blob.data_ptr()), C.c_void_p(off.data_ptr()), None, None, None,
                None, None, n, C.c_void_p(out.data_ptr()), S))
        fn()
        torch.cuda.synchronize()
        read_prof()
        reps = 5
        ev = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
        ev[0].record()
        for _ in range(reps):
            fn()
        ev[1].record()
        torch.cuda.synchronize()
        p = read_prof()
        waves = p[6]
        tot = sum(p[:6])
        print("%s: %.3f ms/launch (profiling build), %d waves" %
              (wl, ev[0].elapsed_time(ev[1]) / reps, waves // reps), flush=True)
        print("  cycles per wave (all its chunks):", {k: round(p[i] / waves) for i, k in enumerate(PHASES)})
        print("  share:", {k: round(p[i] / tot, 3) for i, k in enumerate(PHASES)})
        print("  names:", wave_stats(off.cpu().numpy().view(np.uint32)[: n + 1]), flush=True)
        clf.close()


if __name__ == "__main__":
    main()

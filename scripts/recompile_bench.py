"""Control-plane cost on one MI355X: how long a recompile takes at C5
scale, and whether it stalls classify calls running on other threads.

  1. vc_compile_acl (10k rules) and vc_compile_routes (980,848 + 200,000
     rules, the C3/C5 tables) with the device idle: host build + upload.
  2. A classify thread issues vc_acl_classify_v4_dev calls (1M tuples) on
     its own stream and waits for each (launch + kernel); a load thread
     keeps a second stream busy with 256M-lookup route batches (~5 ms
     kernels), as event-loop traffic on other streams would.  Per-call
     host latency of the classify thread is recorded while the control
     thread is idle, then while it recompiles the ACL and the routes over
     and over.  A snapshot release or recompile that waits for the device
     shows up as classify calls stalled for the length of the load's
     kernels.
Prints one JSON line.
"""
import ctypes as C
import json
import os
import sys
import threading
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import bench  # noqa: E402
import vproxy_amd as V  # noqa: E402
from vproxy_amd import workloads as W  # noqa: E402


def pct(x, q):
    return round(float(np.percentile(x, q)), 3) if len(x) else None


def main():
    dev = torch.device("cuda:0")
    clf = V.Classifier(0)
    t = bench.c5_rule_tables(groups=1000)
    sets = [W.gen_sg_rules(10000, W.SEED + 2 + k, p_range=0.3) for k in range(2)]
    acl_c = []
    for tcp, udp in sets:
        a, na, ka = W.as_ctypes(tcp, V._lib.VcAclRule)
        b, nb, kb = W.as_ctypes(udp, V._lib.VcAclRule)
        acl_c.append((a, na, b, nb, ka, kb))
    nets4 = W.v4_nets(t.net, t.plen)
    nets6 = W.v6_nets(t.hi, t.lo, t.p6)
    r4, n4, k4 = W.as_ctypes(nets4, V._lib.VcNet)
    r6, n6, k6 = W.as_ctypes(nets6, V._lib.VcNet)
    L = V.lib()

    def compile_acl(k):
        a, na, b, nb, _, _ = acl_c[k]
        V.check(L.vc_compile_acl(clf.h, a, na, b, nb, 0))

    def compile_routes():
        V.check(L.vc_compile_routes(clf.h, r4, n4, r6, n6))

    res = {"workload": "recompile"}
    ta, tr = [], []
    for k in range(5):
        t0 = time.perf_counter()
        compile_acl(k & 1)
        ta.append((time.perf_counter() - t0) * 1e3)
    for k in range(3):
        t0 = time.perf_counter()
        compile_routes()
        tr.append((time.perf_counter() - t0) * 1e3)
    res["compile_acl_10k_ms"] = {"median": pct(ta, 50), "max": round(max(ta), 3)}
    res["compile_routes_1180848_ms"] = {"median": pct(tr, 50), "max": round(max(tr), 3)}

    # classify thread + load thread
    n = 1 << 20
    proto, src, port = W.gen_acl_queries(sets[0][0], sets[0][1], n, 5)
    T = lambda x: torch.from_numpy(x).to(dev)
    dp, ds, dq = T(proto), T(src.view(np.int32)), T(port.view(np.int16))
    out = torch.empty(n, dtype=torch.int32, device=dev)
    nl = 256 << 20
    dst = torch.randint(-2**31, 2**31 - 1, (nl,), dtype=torch.int32, device=dev)
    rout = torch.empty(nl, dtype=torch.int32, device=dev)
    s_cls, s_load = bench.hip_stream(dev), bench.hip_stream(dev)
    hip = C.CDLL("libamdhip64.so")
    hip.hipStreamSynchronize.argtypes = [C.c_void_p]
    stop = threading.Event()
    phase = ["quiet"]
    lat = {"quiet": [], "recompile": []}
    loads = [0]

    def classify():
        P = lambda x: C.c_void_p(x.data_ptr())
        while not stop.is_set():
            t0 = time.perf_counter()
            V.check(L.vc_acl_classify_v4_dev(clf.h, P(dp), P(ds), P(dq), n, P(out), None,
                                             C.c_void_p(s_cls.cuda_stream)))
            hip.hipStreamSynchronize(C.c_void_p(s_cls.cuda_stream))
            lat[phase[0]].append((time.perf_counter() - t0) * 1e3)

    def load():
        P = lambda x: C.c_void_p(x.data_ptr())
        while not stop.is_set():
            V.check(L.vc_route_lookup_v4_dev(clf.h, P(dst), nl, P(rout),
                                             C.c_void_p(s_load.cuda_stream)))
            hip.hipStreamSynchronize(C.c_void_p(s_load.cuda_stream))
            loads[0] += 1

    th = [threading.Thread(target=classify), threading.Thread(target=load)]
    for x in th:
        x.start()
    time.sleep(2.0)
    phase[0] = "recompile"
    t_re = time.perf_counter()
    nre = 0
    for k in range(8):
        compile_acl(k & 1)
        nre += 1
        if k % 4 == 3:
            compile_routes()
            nre += 1
    t_re = time.perf_counter() - t_re
    phase[0] = "after"
    lat["after"] = []
    time.sleep(0.5)
    stop.set()
    for x in th:
        x.join()
    for ph in ("quiet", "recompile"):
        v = lat[ph]
        res["classify_call_ms_" + ph] = {"calls": len(v), "p50": pct(v, 50), "p99": pct(v, 99),
                                         "max": round(max(v), 3) if v else None}
    res["recompiles"] = nre
    res["recompile_phase_s"] = round(t_re, 2)
    res["load_batches"] = loads[0]
    clf.close()
    print(json.dumps(res))


if __name__ == "__main__":
    main()

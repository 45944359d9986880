"""Where the mirror_switch_kernel's time goes: the bench's 32M frames through
vc_mirror_switch_dev with different filter lists, beside the parse kernel on
the same frames.  Prints one JSON line per variant (median of 20 launches,
torch events on the launch stream)."""
import ctypes as C
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

import bench as B  # noqa: E402
import vproxy_amd as V  # noqa: E402
from vproxy_amd import workloads as W  # noqa: E402


def timed(fn, reps=20):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    ms = []
    for _ in range(reps):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        fn()
        e1.record()
        e1.synchronize()
        ms.append(e0.elapsed_time(e1))
    ms.sort()
    return ms[len(ms) // 2]


def main():
    dev = torch.device("cuda", 0)
    clf = V.Classifier(0)
    n = 32 << 20
    frames, pidx = B.frames_workload(n)
    fblob, foff = W.pack(frames)
    blob, off, nbytes = B.gather_strings_dev(fblob, foff, pidx, dev)
    S = lambda: C.c_void_p(torch.cuda.current_stream().cuda_stream)
    out = torch.empty(n, dtype=torch.int64, device=dev)
    other = [{"origin": "other", "mirror": 1, "network": "%d.0.0.0/8" % (i + 1)}
             for i in range(16)]
    variants = {
        "bench17": B.MIRROR_FILTERS,
        "one_net": [{"origin": "switch", "mirror": 0, "network": "1.0.0.0/8"}],
        "one_mac": [{"origin": "switch", "mirror": 9, "mac": "0a:00:27:00:00:01"}],
        "skip16_plus_mac": other + [{"origin": "switch", "mirror": 9,
                                     "mac": "0a:00:27:00:00:01"}],
        "four_nets": [{"origin": "switch", "mirror": i, "network": "%d.0.0.0/8" % (i + 1)}
                      for i in range(4)],
        "net_x_only16": [{"origin": "switch", "mirror": i % 8, "network": "%d.0.0.0/8" % (i + 1)}
                         for i in range(16)],
    }
    for name, filters in variants.items():
        res = {}
        for sw in ("0", "1", "2"):     # per-filter kernel / bit-set image / + IPv4 table in LDS
            os.environ["VC_MIRROR_SW"] = sw
            mf = clf.compile_mirror(filters)
            oid = mf.id_of("switch", create=False)
            fn = lambda: V.check(V.lib().vc_mirror_switch_dev(
                clf.h, oid, C.c_void_p(blob.data_ptr()), C.c_void_p(off.data_ptr()), n, 0,
                C.c_void_p(out.data_ptr()), S()))
            ms = timed(fn)
            res[sw] = out.clone()
            print(json.dumps({"variant": name, "filters": len(filters),
                              "path": {"0": "per_filter", "1": "bitsets_global",
                                       "2": "bitsets_lds4"}[sw],
                              "ms": round(ms, 4)}), flush=True)
        assert torch.equal(res["0"], res["1"]) and torch.equal(res["0"], res["2"]), name
        del res
    os.environ.pop("VC_MIRROR_SW")
    res = {k: torch.empty((n, w) if w > 1 else (n,), dtype={"u8": torch.uint8,
           "u16": torch.int16, "u32": torch.int32}[t], device=dev)
           for k, w, t in V.Classifier._PKT_FIELDS}
    o = V._lib.VcPktOut(**{k: v.data_ptr() for k, v in res.items()})
    fn = lambda: V.check(V.lib().vc_parse_packets_dev(
        clf.h, C.c_void_p(blob.data_ptr()), C.c_void_p(off.data_ptr()), n, 0, C.byref(o), S()))
    print(json.dumps({"variant": "parse_all_fields", "ms": round(timed(fn), 4)}), flush=True)
    st = V._lib.VcPktOut(status=res["status"].data_ptr())
    fn = lambda: V.check(V.lib().vc_parse_packets_dev(
        clf.h, C.c_void_p(blob.data_ptr()), C.c_void_p(off.data_ptr()), n, 0, C.byref(st), S()))
    print(json.dumps({"variant": "parse_status_only", "ms": round(timed(fn), 4)}), flush=True)
    clf.close()


if __name__ == "__main__":
    main()

"""Mirror.mirror over MirrorData items (vc_mirror_match_dev): 32M device-
resident items drawn from 64K seeded templates (tests/cases.py
gen_mirror_case: every null level, IPv4 / IPv6 / mapped addresses), 40
filters of one origin with MACs, networks, protocols and port ranges;
per-filter kernel (VC_MIRROR_SW=0) against the bit-set image, median of 20
launches, outputs compared."""
import ctypes as C
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "tests")]
import numpy as np  # noqa: E402
import torch  # noqa: E402

import vproxy_amd as V  # noqa: E402
from cases import gen_mirror_case, mirror_columns  # noqa: E402
from vproxy_amd.mirror import items_struct  # noqa: E402
from mirror_probe import timed  # noqa: E402


def main():
    n = 32 << 20
    rng = np.random.default_rng(91)
    filters, items = gen_mirror_case(rng, 40, 1 << 16, origins=("switch",))
    clf = V.Classifier(0)
    res = {}
    for sw in ("0", "1", "2"):
        os.environ["VC_MIRROR_SW"] = sw
        mf = clf.compile_mirror(filters)
        if sw == "0":
            cols = mirror_columns(items, lambda s: mf.id_of(s, create=False), V.parse_ip)
            idx = torch.from_numpy(np.random.default_rng(92).integers(0, len(items), n)).cuda()
            dcols = {}
            for k, v in cols.items():
                t = torch.from_numpy(v).cuda()
                w = 6 if k.startswith("mac") else 1
                if w > 1:
                    t = t.view(-1, w)
                dcols[k] = t[idx].contiguous().view(-1) if w > 1 else t[idx].contiguous()
            it = items_struct(dcols)
            out = torch.empty(n, dtype=torch.int64, device="cuda")
        oid = mf.id_of("switch", create=False)
        fn = lambda: V.check(V.lib().vc_mirror_match_dev(
            clf.h, oid, C.byref(it), n, C.c_void_p(out.data_ptr()),
            C.c_void_p(torch.cuda.current_stream().cuda_stream)))
        ms = timed(fn)
        res[sw] = out.clone()
        print(json.dumps({"workload": "mirror items", "items": n, "filters": len(filters),
                          "path": {"0": "per_filter", "1": "bitsets_global",
                                   "2": "bitsets_lds"}[sw], "ms": round(ms, 4)}),
              flush=True)
    assert torch.equal(res["0"], res["1"]) and torch.equal(res["0"], res["2"])
    clf.close()


if __name__ == "__main__":
    main()

#!/usr/bin/env python3
"""FETCH_SIZE calibration for random 4-byte gathers (MI355X_MICROARCH.md:
"other access widths are uncalibrated: calibrate on a known byte count in
your own access pattern").

    scripts/fetch_calibration.py CAL_FETCH CAL_L2 CAL_WRITE [--out profiles/r03_fetch_calibration.json]

Input: the rocprofv3 --pmc FETCH_SIZE / TCC_HIT_sum TCC_MISS_sum /
WRITE_SIZE passes of `tools/gather_probe cal`, whose five gather launches
(in dispatch order) stream n = 124,999,992 keys (4 B, 16-B loads) in and
results (4 B, 16-B stores) out, and gather G times per item from a table:
4 KiB (L2-resident: the streams alone), 64 MiB (G = 1, 2), 1 GiB (G = 1, 2).
Per launch: the stream's FETCH (launch 0) against its byte count gives the
stream factor; (FETCH - stream FETCH) / (TCC misses - stream misses) gives
the counted bytes per gather miss.
"""
import argparse
import csv
import json
import os
import re
from collections import defaultdict

N = 125000000 // 8 * 8
LAUNCHES = [(4 << 10, 1), (64 << 20, 1), (64 << 20, 2), (1 << 30, 1), (1 << 30, 2)]
# launch 5 (round 4): the 4 KiB table again, keys read with 4-byte loads
# (one item per lane) -- the dword-stream width of the string kernels


def per_dispatch(d, counter):
    path = None
    for root, _, files in os.walk(d):
        for f in files:
            if f.endswith("counter_collection.csv"):
                path = os.path.join(root, f)
    out = defaultdict(float)
    with open(path) as f:
        for r in csv.DictReader(f):
            if r["Counter_Name"] == counter and re.search(r"\bgather<", r["Kernel_Name"]):
                out[int(r["Dispatch_Id"])] += float(r["Counter_Value"])
    return [out[k] for k in sorted(out)]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("fetch")
    ap.add_argument("l2")
    ap.add_argument("write")
    ap.add_argument("--out", default=None)
    a = ap.parse_args()
    fetch = [x * 1024 for x in per_dispatch(a.fetch, "FETCH_SIZE")]
    miss = per_dispatch(a.l2, "TCC_MISS_sum")
    hit = per_dispatch(a.l2, "TCC_HIT_sum")
    write = [x * 1024 for x in per_dispatch(a.write, "WRITE_SIZE")]
    assert len(fetch) == len(miss) == len(write) in (5, 6), (len(fetch), len(miss), len(write))
    stream = 4 * N
    rows = []
    dword = None
    if len(fetch) == 6:
        dword = {"fetch_bytes": fetch[5], "write_bytes": write[5], "tcc_miss": miss[5],
                 "tcc_hit": hit[5], "stream_fetch_factor": fetch[5] / stream}
    for (tb, g), fr, m, h, w in zip(LAUNCHES, fetch, miss, hit, write):
        gm = m - miss[0]
        rows.append({"table_bytes": tb, "gathers_per_item": g, "items": N,
                     "fetch_bytes": fr, "write_bytes": w, "tcc_miss": m, "tcc_hit": h,
                     "gather_misses": gm if tb > 4096 else 0,
                     "gather_miss_rate": gm / (g * N) if tb > 4096 else 0.0,
                     "fetch_bytes_per_gather_miss": (fr - fetch[0]) / gm if tb > 4096 else None})
    res = {"source": "tools/gather_probe cal under rocprofv3 --pmc (three separate passes)",
           "stream_read_bytes": stream, "stream_fetch_bytes": fetch[0],
           "stream_fetch_factor": fetch[0] / stream,
           "stream_write_factor": write[0] / stream,
           "launches": rows,
           "dword_stream": dword,
           "conclusion": ("a wide (16-B/lane) streamed read is counted at %.3f of its bytes; a "
                          "random 4-byte gather miss is counted at %.1f bytes (one 64-B request); "
                          "streamed stores are counted exactly" % (
                              fetch[0] / stream,
                              sum(r["fetch_bytes_per_gather_miss"] for r in rows[1:]) / 4)) +
                         ("; a 4-byte-per-lane streamed read at %.3f" % dword["stream_fetch_factor"]
                          if dword else "")}
    print(json.dumps(res, indent=1))
    if a.out:
        with open(a.out, "w") as f:
            json.dump(res, f, indent=1)


if __name__ == "__main__":
    main()

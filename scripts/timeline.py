#!/usr/bin/env python3
"""Print the dispatch timeline of a rocprofv3 --kernel-trace CSV.

    scripts/timeline.py KERNEL_TRACE.csv [--last MS] [--match SUBSTR]

One line per dispatch in start order over the last MS milliseconds of the
trace: start offset, duration, queue and a short kernel name, plus the
per-kernel average and how much of each kernel's time overlapped another
queue's kernels (the concurrency the multi-stream schedule buys).
"""
import argparse
import csv
import re
from collections import defaultdict


def short(name):
    name = re.sub(r"\(.*", "", name)
    name = re.sub(r"<.*>", "", name)
    return name.split("::")[-1][:40]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("csv")
    ap.add_argument("--last", type=float, default=30.0)
    ap.add_argument("--match", default="")
    a = ap.parse_args()
    rows = []
    with open(a.csv) as f:
        for r in csv.DictReader(f):
            name = r.get("Kernel_Name") or r.get("KernelName") or ""
            if a.match and a.match not in name:
                continue
            s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
            q = r.get("Queue_Id") or r.get("Stream_Id") or "?"
            rows.append((s, e, q, short(name)))
    rows.sort()
    if not rows:
        print("no dispatches")
        return
    t_end = max(e for _, e, _, _ in rows)
    t0 = t_end - a.last * 1e6
    sel = [r for r in rows if r[1] >= t0]
    base = sel[0][0]
    for s, e, q, n in sel:
        print("%9.3f ms  %8.3f ms  q%-3s %s" % ((s - base) / 1e6, (e - s) / 1e6, q, n))
    tot = defaultdict(float)
    cnt = defaultdict(int)
    ovl = defaultdict(float)
    for i, (s, e, q, n) in enumerate(sel):
        tot[n] += (e - s) / 1e6
        cnt[n] += 1
        # time of [s, e) covered by a dispatch on another queue
        segs = sorted((max(s, s2), min(e, e2)) for s2, e2, q2, _ in sel
                      if q2 != q and s2 < e and e2 > s)
        cov, cur = 0, s
        for x, y in segs:
            x = max(x, cur)
            if y > x:
                cov += y - x
                cur = y
        ovl[n] += cov / 1e6
    print("\nkernel                                     n    avg ms   overlapped")
    for n in sorted(tot, key=lambda k: -tot[k]):
        print("%-40s %4d  %8.3f   %5.1f %%" % (n, cnt[n], tot[n] / cnt[n], 100 * ovl[n] / tot[n]))
    span = (sel[-1][1] - base) / 1e6
    print("\nspan %.3f ms" % span)


if __name__ == "__main__":
    main()

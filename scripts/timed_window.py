#!/usr/bin/env python3
"""Cut the timed steps out of a rocprofv3 --kernel-trace CSV of a C5 bench
run and summarise them.

    scripts/timed_window.py KERNEL_TRACE.csv --warmup W --steps K [--out PREFIX]

bench.py synchronises the device between the warmup and the timed steps,
and the first kernel of the timed region is the hostname-pool pass
(hint_kernel) of batch W.  The window runs from that launch's start to the
end of the last classifier kernel; torch generator kernels and the
warmup's kernels fall outside it.  Prints (and writes PREFIX_stats.csv /
PREFIX_timeline.txt): per kernel the launches, average / min / max
duration and total time in the window; the window's wall time per step;
per queue the busy time; and the dispatch timeline of two timed steps.
"""
import argparse
import csv
import re
from collections import defaultdict


def short(name):
    name = re.sub(r"\(.*", "", name)
    name = re.sub(r"<.*>", "", name)
    return name.replace("void ", "").split("::")[-1].strip()


def load(path):
    rows = []
    with open(path) as f:
        for r in csv.DictReader(f):
            rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]),
                         r.get("Queue_Id") or r.get("Stream_Id") or "?", short(r["Kernel_Name"])))
    rows.sort()
    return rows


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("csv")
    ap.add_argument("--warmup", type=int, required=True)
    ap.add_argument("--steps", type=int, required=True)
    ap.add_argument("--out", default=None)
    a = ap.parse_args()
    rows = load(a.csv)
    hints = [r for r in rows if r[3] == "hint_kernel"]
    pipes = [r for r in rows if r[3].startswith("pipeline_")]
    assert len(pipes) >= a.warmup + a.steps, (len(pipes), a.warmup + a.steps)
    t0 = hints[a.warmup][0] if len(hints) > a.warmup else pipes[a.warmup][0]
    # the window ends with the last classifier kernel: bench.py measures its
    # copy rate (torch copies) after the timed region
    ours = ("hint_", "pipeline_", "bucket_", "counter", "acl_", "route_", "dns", "cert_",
            "packet", "switch", "mirror", "source")
    t1 = max(r[1] for r in rows if r[0] >= t0 and r[3].startswith(ours))
    mine = [r for r in rows if t0 <= r[0] < t1]
    wall = (t1 - t0) / 1e6
    per = defaultdict(list)
    busy = defaultdict(float)
    for s, e, q, n in mine:
        per[n].append((e - s) / 1e6)
        busy[q] += (e - s) / 1e6
    lines = ["timed window: %d steps, %.3f ms wall = %.3f ms per step (first timed kernel start "
             "to last kernel end)" % (a.steps, wall, wall / a.steps)]
    lines.append("%-32s %7s %9s %9s %9s %10s %8s" % ("kernel", "count", "avg_ms", "min_ms",
                                                     "max_ms", "total_ms", "per_step"))
    stats = []
    for n, v in sorted(per.items(), key=lambda kv: -sum(kv[1])):
        stats.append((n, len(v), sum(v) / len(v), min(v), max(v), sum(v)))
        lines.append("%-32s %7d %9.4f %9.4f %9.4f %10.3f %8.3f" % (
            n, len(v), sum(v) / len(v), min(v), max(v), sum(v), sum(v) / a.steps))
    lines.append("queue busy per step: " + ", ".join(
        "q%s %.3f ms" % (q, b / a.steps) for q, b in sorted(busy.items())))
    # timeline of two timed steps (from the second timed pool pass)
    tl = []
    th = [r for r in mine if r[3] == "hint_kernel"]
    if len(th) >= 3:
        lo, hi = th[1][0], th[3][0] if len(th) > 3 else t1
        for s, e, q, n in mine:
            if lo <= s < hi:
                tl.append("%9.3f ms  %8.3f ms  q%-3s %s" % ((s - lo) / 1e6, (e - s) / 1e6, q, n))
    print("\n".join(lines))
    print("\n".join(tl))
    if a.out:
        with open(a.out + "_stats.csv", "w", newline="") as f:
            w = csv.writer(f)
            w.writerow(["kernel", "count", "avg_ms", "min_ms", "max_ms", "total_ms"])
            for r in stats:
                w.writerow([r[0], r[1]] + ["%.5f" % x for x in r[2:]])
        with open(a.out + "_timeline.txt", "w") as f:
            f.write("\n".join(lines) + "\n\n" + "\n".join(tl) + "\n")


if __name__ == "__main__":
    main()

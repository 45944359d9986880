#!/usr/bin/env python3
"""Summarise rocprofv3 CSV outputs into profiles/ (run on this side, after
gpurun merged gpurun_out/ back).

    scripts/pmc_traffic.py STATS_DIR FETCH_DIR WRITE_DIR [--tag r01] [--workload c5]

STATS_DIR: `rocprofv3 --kernel-trace --stats --output-format csv` output
FETCH_DIR / WRITE_DIR: `rocprofv3 --pmc FETCH_SIZE` / `--pmc WRITE_SIZE`
(separate passes, as MI355X_MICROARCH.md §rocprofv3 PMC slots requires).

Per kernel it writes the average per-launch HBM-side bytes.  FETCH_SIZE and
WRITE_SIZE are in KiB.  On gfx950 FETCH_SIZE counts half the bytes of a
wide coalesced stream (MI355X_MICROARCH.md §HBM) and, by this repo's own
calibration (scripts/fetch_calibration.py -> profiles/r03_fetch_calibration.json:
tools/gather_probe cal, known gathers into known tables), one L2 miss of a
random 4-byte gather as 64 bytes -- the full line request.  So the
correction applies only to the wide streamed reads: with
--stream KERNEL=BYTES (the kernel's algorithmic 16-B-per-lane streamed read
bytes per launch), `traffic` = FETCH + BYTES / 2 + WRITE.  Kernels without
--stream keep the guide's upper estimate 2 x FETCH + WRITE.
"""
import argparse
import csv
import glob
import json
import os
import shutil
from collections import defaultdict

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def kname(s):
    """'void vcd::pipeline_v4_kernel<true, true>(AclImage, ...)' -> 'pipeline_v4_kernel'"""
    s = s.split("(")[0]
    if s.startswith("void "):
        s = s[5:]
    return s.split("<")[0].split("::")[-1].strip()


def _find(d, pattern):
    hits = sorted(glob.glob(os.path.join(d, "**", pattern), recursive=True))
    if not hits:
        raise SystemExit("no %s under %s" % (pattern, d))
    return hits[0]


def counter_avg(d, name):
    """kernel -> (launches, mean counter value per launch)."""
    path = _find(d, "*counter_collection.csv")
    per = defaultdict(lambda: defaultdict(float))
    with open(path) as f:
        for row in csv.DictReader(f):
            if row.get("Counter_Name") != name:
                continue
            k = kname(row["Kernel_Name"])
            per[k][row.get("Dispatch_Id") or row.get("Correlation_Id")] += float(row["Counter_Value"])
    return {k: (len(v), sum(v.values()) / len(v)) for k, v in per.items()}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("stats")
    ap.add_argument("fetch")
    ap.add_argument("write")
    ap.add_argument("--tag", default="r01")
    ap.add_argument("--workload", default="c5")
    ap.add_argument("--kernels", default="pipeline_v4_kernel,hint_kernel")
    ap.add_argument("--l2", default=None, help="rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum output")
    ap.add_argument("--commit", default=None, help="git commit the passes were taken at")
    ap.add_argument("--stream", action="append", default=[],
                    help="KERNEL=BYTES: wide streamed read bytes per launch (see module doc)")
    ap.add_argument("--per-step", action="append", default=[],
                    help="KERNEL=COUNT: launches of KERNEL in one bench step; with it the "
                         "entry gets `step`: the L2-to-fabric requests of one whole step "
                         "(FETCH_SIZE / 64 B = TCC_EA0_RDREQ, WRITE_SIZE / 64 B = write "
                         "requests), the quantity tools/gather_paths.hip finds capped")
    a = ap.parse_args()
    prof = os.path.join(ROOT, "profiles")
    stats = _find(a.stats, "*kernel_stats.csv")
    shutil.copy(stats, os.path.join(prof, "%s_%s_kernel_stats.csv" % (a.tag, a.workload)))
    avg_ns = {}
    with open(stats) as f:
        for row in csv.DictReader(f):
            avg_ns[kname(row["Name"])] = float(row["AverageNs"])
    fetch = counter_avg(a.fetch, "FETCH_SIZE")
    write = counter_avg(a.write, "WRITE_SIZE")
    l2 = {}
    if a.l2:
        hits, miss = counter_avg(a.l2, "TCC_HIT_sum"), counter_avg(a.l2, "TCC_MISS_sum")
        l2 = {k: (hits[k][1], miss[k][1]) for k in hits if k in miss}
    stream = {kv.split("=")[0]: float(kv.split("=")[1]) for kv in a.stream}
    out = {}
    for k in a.kernels.split(","):
        if k not in fetch or k not in write:
            continue
        fr, wr = fetch[k][1] * 1024, write[k][1] * 1024
        if k in stream:
            traffic = fr + stream[k] / 2 + wr
            method = ("FETCH_SIZE + streamed reads / 2 (%.4g B, counted at half) + WRITE_SIZE; "
                      "gather misses counted whole (profiles/r03_fetch_calibration.json)"
                      % stream[k])
        else:
            traffic = 2 * fr + wr
            method = "2 x FETCH_SIZE + WRITE_SIZE (the guide's stream correction on every read)"
        ns = avg_ns.get(k)
        out[k] = {"launches_fetch_pass": fetch[k][0], "fetch_bytes_raw": fr,
                  "fetch_bytes_x2": 2 * fr, "write_bytes": wr, "traffic_bytes": traffic,
                  "traffic_method": method, "avg_ns_kernel_trace": ns,
                  "traffic_GBps": traffic / ns if ns else None}
        if k in l2:
            out[k]["tcc_hit"], out[k]["tcc_miss"] = l2[k]
    step = None
    if a.per_step:
        kinds = {}
        for kv in a.per_step:
            k, cnt = kv.split("=")
            if k in fetch and k in write:
                req = (fetch[k][1] * 1024 + write[k][1] * 1024) / 64
                kinds[k] = {"launches": int(cnt), "requests_per_launch": req}
        step = {"requests": sum(v["launches"] * v["requests_per_launch"] for v in kinds.values()),
                "kernels": kinds,
                "method": "per launch FETCH_SIZE / 64 B (read requests, a wide stream's 128-B "
                          "request counted once) + WRITE_SIZE / 64 B, times launches per step"}
    path = os.path.join(prof, "pmc_traffic.json")
    try:
        with open(path) as f:
            allw = json.load(f)
    except (OSError, ValueError):
        allw = {}
    allw[a.workload] = {"tag": a.tag, "commit": a.commit, "kernels": out,
                        "note": "per launch; FETCH_SIZE/WRITE_SIZE KiB x 1024; traffic_method "
                                "per kernel"}
    if step:
        allw[a.workload]["step"] = step
    with open(path, "w") as f:
        json.dump(allw, f, indent=1)
    for src, name in ((a.fetch, "fetch"), (a.write, "write")):
        p = _find(src, "*counter_collection.csv")
        rows = [r for r in csv.DictReader(open(p))
                if kname(r["Kernel_Name"]) in a.kernels.split(",")]
        if rows:
            with open(os.path.join(prof, "%s_%s_pmc_%s.csv" % (a.tag, a.workload, name)), "w",
                      newline="") as f:
                w = csv.DictWriter(f, fieldnames=list(rows[0].keys()))
                w.writeheader()
                w.writerows(rows)
    print(json.dumps(allw[a.workload], indent=1))


if __name__ == "__main__":
    main()

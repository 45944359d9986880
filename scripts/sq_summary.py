#!/usr/bin/env python3
"""Per-dispatch SQ issue counters of scripts/prof.sh (PASSES=sq), for the
dispatches of one kernel at its largest grid: instructions per wave, and the
VALU issue share of the kernel's own cycles.  GRBM_GUI_ACTIVE is summed over
the 8 XCDs (MI355X_MICROARCH.md), so cycles = GRBM_GUI_ACTIVE / 8; a CU
issues at most two wave64 VALU instructions per cycle (four SIMDs, two
cycles each).
    scripts/sq_summary.py DIR KERNEL [CUS]"""
import csv
import glob
import sys
from collections import defaultdict

d, kern = sys.argv[1], sys.argv[2]
cus = int(sys.argv[3]) if len(sys.argv) > 3 else 256
rows = defaultdict(dict)
meta = {}
for r in csv.DictReader(open(glob.glob(d + "/*counter_collection.csv")[0])):
    if kern not in r["Kernel_Name"]:
        continue
    k = r["Dispatch_Id"]
    rows[k][r["Counter_Name"]] = float(r["Counter_Value"])
    meta[k] = int(r["Grid_Size"])
big = max(meta.values())
sel = [rows[k] for k in rows if meta[k] == big]
avg = {c: sum(x[c] for x in sel) / len(sel) for c in sel[0]}
cyc = avg["GRBM_GUI_ACTIVE"] / 8
waves = avg["SQ_WAVES"]
out = {"kernel": kern, "dispatches": len(sel), "grid_threads": big, "waves": waves,
       "kernel_cycles": round(cyc)}
for c in ("SQ_INSTS_VALU", "SQ_INSTS_SALU", "SQ_INSTS_LDS", "SQ_INSTS_VMEM_RD"):
    out[c + "_per_wave"] = round(avg[c] / waves, 1)
out["valu_issue_share"] = round(avg["SQ_INSTS_VALU"] / (cus * 2 * cyc), 3)
out["salu_per_cu_cycle"] = round(avg["SQ_INSTS_SALU"] / (cus * cyc), 3)
out["wave_cycles_per_wave"] = round(avg["SQ_WAVE_CYCLES"] * 4 / waves)
print(out)

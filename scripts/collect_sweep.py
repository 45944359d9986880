"""Gathers the JSON lines of gpurun_out/sweep_<w>.log (scripts/sweep.sh)
into one file keyed by workload: python scripts/collect_sweep.py OUT.json"""
import glob
import json
import os
import sys

out = {}
if os.path.exists(sys.argv[1]):
    out = json.load(open(sys.argv[1]))
for f in sorted(glob.glob("gpurun_out/sweep_*.log")):
    w = os.path.basename(f)[len("sweep_"):-len(".log")]
    lines = [l for l in open(f) if l.startswith("{")]
    if lines:
        out[w] = json.loads(lines[-1])
json.dump(out, open(sys.argv[1], "w"), indent=1)
print(sorted(out))

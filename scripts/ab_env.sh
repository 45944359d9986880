#!/bin/bash
# A/B of C5 schedule / library knobs on the GPU box, two interleaved rounds:
#   bash scripts/ab_env.sh "name|ENV=V ENV2=V|bench args" ...
# One JSON line per run in gpurun_out/ab_env.jsonl.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
OUT=gpurun_out/ab_env.jsonl
: > $OUT
B="python3 bench.py --steps ${STEPS:-20} --warmup 3 --no-cpu-baseline"
for round in 1 2; do
  for cfg in "$@"; do
    IFS='|' read -r name envs args <<< "$cfg"
    echo "=== $round $name [$envs] $args"
    env $envs timeout -k 10 120 $B $args > gpurun_out/ab_one.log 2>&1
    rc=$?
    if [ $rc -ne 0 ]; then echo "rc=$rc"; tail -5 gpurun_out/ab_one.log; exit $rc; fi
    python3 - "$name" "$round" <<'PY' >> $OUT
import json, sys
line = [l for l in open("gpurun_out/ab_one.log") if l.startswith("{")][-1]
d = json.loads(line)
o = d["roofline"].get("other_kernel_ms", {})
sub = "config" not in d          # a sub-bench line (bench.py run_sub)
print(json.dumps({"cfg": sys.argv[1], "round": int(sys.argv[2]),
                  "workload": d["workload"] if sub else d["config"]["workload"],
                  "ms_per_step": d["ms_per_step"], "value": d["M_items_per_s"] if sub else d["value"],
                  "kernel_ms": d["kernel_ms"] if sub else d["roofline"].get("kernel_ms"),
                  "pipe_ms": o.get("pipeline_v4_kernel"),
                  "hint_ms": o.get("hint_kernel"), "count_ms": o.get("kernel_end_to_counters_done"),
                  "kernel_only_ms": d.get("kernel_only_ms"), "v4_ms": d.get("v4_ms"),
                  "v6_ms": d.get("v6_ms"), "v4_same_ms": d.get("v4_kernel_same_packets_ms")}))
PY
    tail -1 $OUT
  done
done

#!/bin/bash
# A/B on the GPU box: the C5 schedule with the next pool pass beside the
# counter finish (default) against the pool pass beside the pipeline kernel
# with the pool pass capped at K workgroups per CU (VC_HINT_WG_PER_CU, a knob of the
# library at b2524f6, since removed), so
# the VALU-bound pool pass shares the CUs of the gather-bound pipeline
# kernel.  Two interleaved rounds; one JSON line per run in gpurun_out/ab_overlap.jsonl.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
OUT=gpurun_out/ab_overlap.jsonl
: > $OUT
B="python3 bench.py --steps ${STEPS:-20} --warmup 3 --no-cpu-baseline"
for round in 1 2; do
  for cfg in "base::" "pipe::--overlap pipeline" "pipe1:1:--overlap pipeline" "pipe2:2:--overlap pipeline" "pipe3:3:--overlap pipeline" "fin1:1:"; do
    name=${cfg%%:*}; rest=${cfg#*:}; cap=${rest%%:*}; args=${rest#*:}
    echo "=== $round $name cap=$cap $args"
    if [ -n "$cap" ]; then export VC_HINT_WG_PER_CU=$cap; else unset VC_HINT_WG_PER_CU; fi
    timeout -k 10 120 $B $args > gpurun_out/ab_one.log 2>&1
    rc=$?
    if [ $rc -ne 0 ]; then echo "rc=$rc"; tail -5 gpurun_out/ab_one.log; exit $rc; fi
    python3 - "$name" "$round" "$cap" <<'PY' >> $OUT
import json, sys
line = [l for l in open("gpurun_out/ab_one.log") if l.startswith("{")][-1]
d = json.loads(line)
o = d["roofline"]["other_kernel_ms"]
print(json.dumps({"cfg": sys.argv[1], "round": int(sys.argv[2]), "cap": sys.argv[3],
                  "ms_per_step": d["ms_per_step"], "value": d["value"],
                  "pipe_ms": o["pipeline_v4_kernel"], "hint_ms": o["hint_kernel"],
                  "count_ms": o["kernel_end_to_counters_done"]}))
PY
    tail -1 $OUT
  done
done

#!/bin/bash
# A/B of library builds on one GPU box, interleaved rounds:
#   scripts/ab_libs.sh "<workloads>" <lib dir>...
# Workloads are separated by ';': a bench.py --workload name, or
# "tag|bench args" for any other argument set, e.g.
#   scripts/ab_libs.sh "c5;mix15c|--workload mix --compact6" build/a build/b  Each build
# runs every workload ROUNDS times (default 2); one JSON line per run in
# gpurun_out/ab/ab.jsonl.  Builds:
#   make -C vproxy_amd/csrc OUT=../../build/<x>/libvclassify.so BUILD=../../build/obj_<x> EXTRA=...
set -o pipefail
wls=$1; shift
mkdir -p gpurun_out/ab
for rep in $(seq 1 ${ROUNDS:-2}); do
  IFS=';' read -r -a wlist <<< "$wls"
  for wl in "${wlist[@]}"; do
    if [[ "$wl" == *"|"* ]]; then tagw=${wl%%|*}; args=${wl#*|}; else tagw=$wl; args="--workload $wl"; fi
    for d in "$@"; do
      tag=$(basename $d)
      f=gpurun_out/ab/$tag.$tagw.$rep
      VCLASSIFY_LIB=$d/libvclassify.so timeout -k 10 240 python -u bench.py $args --steps ${STEPS:-20} --warmup 5 \
        --no-cpu-baseline > $f.json 2> $f.err || { echo "FAIL $tag $tagw"; tail -5 $f.err; exit 1; }
      python - $f.json $tag $tagw $rep <<'PY' | tee -a gpurun_out/ab/ab.jsonl
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
sub = "config" not in d
r = d.get("roofline", {})
print(json.dumps({"lib": sys.argv[2], "wl": sys.argv[3], "rep": int(sys.argv[4]),
                  "value": d.get("M_items_per_s") if sub else d["value"],
                  "ms_per_step": d["ms_per_step"],
                  "kernel_ms": d.get("kernel_only_ms") or d.get("kernel_ms") or r.get("kernel_ms"),
                  "v4_ms": d.get("v4_kernel_same_packets_ms"),
                  "other": r.get("other_kernel_ms")}))
PY
    done
  done
done

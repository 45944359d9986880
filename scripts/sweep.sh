#!/bin/bash
# Runs bench.py workloads one after another on the GPU box (each a step of
# gpu_steps.sh, so a failure stops the sweep), CPU baselines included:
#   bash scripts/sweep.sh c5 c1 c2 "mixc6|--workload mix --compact6" ...
#   -> gpurun_out/sweep_<name>.log   (a plain name w runs --workload w)
# Collect with scripts/collect_sweep.py.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
steps=()
for w in "$@"; do
    if [[ "$w" == *"|"* ]]; then name=${w%%|*}; args=${w#*|}; else name=$w; args="--workload $w"; fi
    steps+=("sweep_$name:240:python bench.py $args --steps ${STEPS:-10}")
done
bash scripts/gpu_steps.sh "${steps[@]}"

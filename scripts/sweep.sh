#!/bin/bash
# Runs bench.py workloads one after another on the GPU box (each a step of
# gpu_steps.sh, so a failure stops the sweep), CPU baselines included:
#   bash scripts/sweep.sh c5 c1 c2 ...   -> gpurun_out/sweep_<w>.log
# Collect with scripts/collect_sweep.py.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
steps=()
for w in "$@"; do
    steps+=("sweep_$w:240:python bench.py --workload $w --steps ${STEPS:-10}")
done
bash scripts/gpu_steps.sh "${steps[@]}"

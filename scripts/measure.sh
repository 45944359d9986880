#!/bin/bash
# One round's measurement at one commit, on the GPU box:
#   bash scripts/measure.sh TAG suite     GPU suite, the driver's C5 command, the default line
#   bash scripts/measure.sh TAG sweep W.. sub-benches (scripts/sweep.sh), CPU baselines included
#   bash scripts/measure.sh TAG prof      C5 timed-window trace + PMC passes of c5 / c3 / c4 / dns / mix
# Outputs under gpurun_out/; scripts/collect_sweep.py, pmc_traffic.py and
# timed_window.py summarise them into profiles/ on this side.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
tag=$1; what=$2; shift 2
mkdir -p gpurun_out
case $what in
  suite)
    bash scripts/gpu_steps.sh \
      "${tag}_gpu_tests:900:python -u -m pytest -x -v --timeout 300 --timeout-method thread tests -m gpu" \
      "${tag}_bench_c5:300:python bench.py --gpus 1 --steps 20 --warmup 5" \
      "${tag}_bench_default:300:python bench.py" ;;
  sweep)
    rm -f gpurun_out/sweep_*.log
    bash scripts/sweep.sh "$@" ;;
  prof)
    bash scripts/prof.sh "$tag" "c5|" "c3|--workload c3" "c4|--workload c4" "dns|--workload dns" \
      "mix|--workload mix --compact6" ;;
  *) echo "usage: measure.sh TAG suite|sweep W...|prof"; exit 2 ;;
esac

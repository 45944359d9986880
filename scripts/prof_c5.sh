#!/bin/bash
# The C5 profile passes of scripts/prof_r03.sh alone (no gather calibration),
# for re-taking the pipeline's kernel trace and PMC traffic at HEAD:
# kernel trace of the run (scripts/timed_window.py cuts the timed steps),
# then FETCH_SIZE, WRITE_SIZE and TCC hit/miss, each --pmc pass its own run.
# Summaries: scripts/timed_window.py, scripts/pmc_traffic.py --stream.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
export TMPDIR=/tmp
O=gpurun_out/p3
B="python3 bench.py --steps ${STEPS:-5} --warmup 2 --no-cpu-baseline"
bash scripts/gpu_steps.sh \
  "c5_trace:240:rocprofv3 --kernel-trace --stats --output-format csv -d $O/c5_trace -o run -- $B" \
  "c5_fetch:240:timeout -s KILL 220 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/c5_fetch -o run -- $B" \
  "c5_write:240:timeout -s KILL 220 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/c5_write -o run -- $B" \
  "c5_l2:240:timeout -s KILL 220 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum --output-format csv -d $O/c5_l2 -o run -- $B"

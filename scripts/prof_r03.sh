#!/bin/bash
# Round-3 profile passes on the GPU box: the C5 bench (kernel trace of the
# whole run -- scripts/timed_window.py cuts the timed steps out of it -- and
# FETCH_SIZE / WRITE_SIZE / TCC hit-miss passes), then the FETCH_SIZE
# calibration of random 4-byte gathers (tools/gather_probe cal).  Each --pmc
# pass is a run of its own (MI355X_MICROARCH.md).  Summaries on this side:
# scripts/timed_window.py, scripts/pmc_traffic.py.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
export TMPDIR=/tmp
O=gpurun_out/p3
B="python3 bench.py --steps ${STEPS:-5} --warmup 2 --no-cpu-baseline"
G="tools/gather_probe cal"
bash scripts/gpu_steps.sh \
  "c5_trace:240:rocprofv3 --kernel-trace --stats --output-format csv -d $O/c5_trace -o run -- $B" \
  "c5_fetch:240:timeout -s KILL 220 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/c5_fetch -o run -- $B" \
  "c5_write:240:timeout -s KILL 220 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/c5_write -o run -- $B" \
  "c5_l2:240:timeout -s KILL 220 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum --output-format csv -d $O/c5_l2 -o run -- $B" \
  "cal_trace:120:rocprofv3 --kernel-trace --stats --output-format csv -d $O/cal_trace -o run -- $G" \
  "cal_fetch:120:timeout -s KILL 100 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/cal_fetch -o run -- $G" \
  "cal_write:120:timeout -s KILL 100 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/cal_write -o run -- $G" \
  "cal_l2:120:timeout -s KILL 100 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum --output-format csv -d $O/cal_l2 -o run -- $G"
bash scripts/gpu_steps.sh "gather_mix:300:tools/gather_probe mix"

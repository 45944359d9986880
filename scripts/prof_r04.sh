#!/bin/bash
# Round-4 profile passes on the GPU box, one workload set per call:
#   bash scripts/prof_r04.sh c5 c3 ...   (c5 c3 c4 dns mix c2, or cal)
# Per workload: a kernel-trace --stats pass and separate --pmc passes for
# FETCH_SIZE, WRITE_SIZE and TCC_HIT_sum TCC_MISS_sum (MI355X_MICROARCH.md:
# counters in their own runs, no tracing beside them).  `cal`: the FETCH_SIZE
# calibration launches of tools/gather_probe (incl. the 4-byte-load stream).
# Summaries on this side: scripts/pmc_traffic.py, scripts/fetch_calibration.py.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
export TMPDIR=/tmp
export VC_BENCH_NO_E2E=1
O=gpurun_out/p4
steps=()
for w in "$@"; do
  if [ "$w" = cal ]; then
    C="tools/gather_probe cal"
  else
    C="python3 bench.py --workload $w --steps ${STEPS:-5} --warmup 2 --no-cpu-baseline"
  fi
  steps+=("${w}_trace:300:rocprofv3 --kernel-trace --stats --output-format csv -d $O/${w}_trace -o run -- $C"
          "${w}_fetch:300:timeout -s KILL 280 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/${w}_fetch -o run -- $C"
          "${w}_write:300:timeout -s KILL 280 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/${w}_write -o run -- $C"
          "${w}_l2:300:timeout -s KILL 280 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum --output-format csv -d $O/${w}_l2 -o run -- $C")
done
bash scripts/gpu_steps.sh "${steps[@]}"

#!/bin/bash
# rocprofv3 passes of one bench workload on the GPU box (round 2): kernel
# stats, then FETCH_SIZE, WRITE_SIZE and TCC hit/miss, each a pass of its own
# (MI355X_MICROARCH.md: separate --pmc passes).  Usage: prof_r02.sh WORKLOAD
# [bench args].  Summarise with scripts/pmc_traffic.py afterwards.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
export TMPDIR=/tmp
W=$1; shift
O=gpurun_out/p_$W
B="python3 bench.py --workload $W --steps ${STEPS:-3} --warmup 1 --no-cpu-baseline $*"
bash scripts/gpu_steps.sh \
  "${W}_stats:200:rocprofv3 --kernel-trace --stats --output-format csv -d $O/stats -o run -- $B" \
  "${W}_fetch:200:timeout -s KILL 180 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/fetch -o run -- $B" \
  "${W}_write:200:timeout -s KILL 180 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/write -o run -- $B" \
  "${W}_l2:200:timeout -s KILL 180 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum --output-format csv -d $O/l2 -o run -- $B"

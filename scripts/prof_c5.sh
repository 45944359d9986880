#!/bin/bash
# rocprofv3 passes for the C5 bench (run on the GPU box via gpurun):
# kernel-trace stats, then FETCH_SIZE, WRITE_SIZE and L2 hit/miss each in a
# pass of its own.  Summarise afterwards with scripts/pmc_traffic.py.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
export TMPDIR=/tmp
O=gpurun_out
B="python3 bench.py --steps ${STEPS:-3} --warmup 1 --no-cpu-baseline $*"
bash scripts/gpu_steps.sh \
  "stats:200:rocprofv3 --kernel-trace --stats --output-format csv -d $O/p_stats -o run -- $B" \
  "fetch:200:timeout -s KILL 180 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/p_fetch -o run -- $B" \
  "write:200:timeout -s KILL 180 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/p_write -o run -- $B" \
  "l2:200:timeout -s KILL 180 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum --output-format csv -d $O/p_l2 -o run -- $B"
[ -n "$SQ" ] && bash scripts/gpu_steps.sh \
  "sq:200:timeout -s KILL 180 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_WAVES --output-format csv -d $O/p_sq -o run -- $B" \
  "list:60:timeout -s KILL 50 rocprofv3 -L > $O/counters_list.txt"
true

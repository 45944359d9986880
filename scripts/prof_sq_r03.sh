#!/bin/bash
# SQ issue counters with the kernel's own cycle count (GRBM_GUI_ACTIVE), per
# dispatch, for the C2 ACL kernel and the C4 hint kernel: is the VALU the
# bound?  Summary: scripts/sq_summary.py.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
export TMPDIR=/tmp
O=gpurun_out/sq3
C="SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_WAVE_CYCLES GRBM_GUI_ACTIVE"
bash scripts/gpu_steps.sh \
  "c2_sq:200:timeout -s KILL 180 rocprofv3 --pmc $C --output-format csv -d $O/c2 -o run -- python3 bench.py --workload c2 --steps 3 --warmup 1 --no-cpu-baseline" \
  "c4_sq:200:timeout -s KILL 180 rocprofv3 --pmc $C --output-format csv -d $O/c4 -o run -- python3 bench.py --workload c4 --steps 3 --warmup 1 --no-cpu-baseline"

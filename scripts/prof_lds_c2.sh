#!/bin/bash
# LDS and wait counters of the C2 ACL kernel (lockstep search): is the LDS
# array (bank conflicts) or the wait on it what bounds C2?
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
export TMPDIR=/tmp
O=gpurun_out/lds_c2
C="SQ_WAVES SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_WAVE_CYCLES GRBM_GUI_ACTIVE"
bash scripts/gpu_steps.sh \
  "c2_lds:200:timeout -s KILL 180 rocprofv3 --pmc $C --output-format csv -d $O -o run -- python3 bench.py --workload c2 --steps 3 --warmup 1 --no-cpu-baseline"

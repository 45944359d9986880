#!/bin/bash
# SQ counter passes of the C2 ACL kernel (acl_v4_kernel) and of the C5
# pipeline kernel: where their cycles go (VALU / LDS / VMEM issue and waits,
# LDS bank conflicts).  One --pmc pass per counter group.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
export TMPDIR=/tmp
O=gpurun_out/sq
B2="python3 bench.py --workload c2 --steps 3 --warmup 1 --no-cpu-baseline"
B5="python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline"
timeout -k 10 60 rocprofv3 --list-avail > $O.avail.txt 2>&1 || true
bash scripts/gpu_steps.sh \
  "c2_sq1:200:timeout -s KILL 180 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD --output-format csv -d $O/c2_sq1 -o run -- $B2" \
  "c2_sq2:200:timeout -s KILL 180 rocprofv3 --pmc SQ_INSTS_SALU SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VMEM SQ_INST_CYCLES_VMEM SQ_LDS_BANK_CONFLICT SQ_INSTS_SMEM SQ_ACTIVE_INST_ANY --output-format csv -d $O/c2_sq2 -o run -- $B2" \
  "c5_sq1:200:timeout -s KILL 180 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD --output-format csv -d $O/c5_sq1 -o run -- $B5" \
  "c5_sq2:200:timeout -s KILL 180 rocprofv3 --pmc SQ_INSTS_SALU SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VMEM SQ_INST_CYCLES_VMEM SQ_LDS_BANK_CONFLICT SQ_INSTS_SMEM SQ_ACTIVE_INST_ANY --output-format csv -d $O/c5_sq2 -o run -- $B5"

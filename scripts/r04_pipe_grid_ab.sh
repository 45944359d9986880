#!/bin/bash
# C5: the IPv4 pipeline kernel's grid (VC_PIPE_GRID workgroups, one per CU)
# with the round-4 pool pass: 224 (default) / 216 / 232 / 240
cd "$(dirname "$0")/.."
STEPS=20 bash scripts/ab_env.sh "g224||" "g216|VC_PIPE_GRID=216|" "g232|VC_PIPE_GRID=232|" "g240|VC_PIPE_GRID=240|" > gpurun_out/pipe_grid.txt 2>&1

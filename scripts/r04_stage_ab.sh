#!/bin/bash
# A/B of the per-wave stage copy: dword loop (sq0), 16-byte pieces (sq1),
# 16-byte pieces with every load issued before the writes (sq2)
cd "$(dirname "$0")/.."
bash scripts/ab_libs.sh "c4 dns switch" build/sq0 build/sq1 build/sq2 > gpurun_out/stage_ab.txt 2>&1

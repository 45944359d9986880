#!/bin/bash
# frame kernels on the static split: every nwaves-th chunk (pc0) or one
# contiguous run of chunks per wave (pc1)
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
bash scripts/ab_libs.sh "parse switch" build/pc0 build/pc1 > gpurun_out/contig_ab.txt 2>&1

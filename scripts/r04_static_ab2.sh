#!/bin/bash
# static share of the chunks per wave before the work tickets: 0 / 25 / 40 /
# 50 / 60 %, on every kernel that takes tickets and the C5 step
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
bash scripts/ab_libs.sh "c4 dns sni mirror dnsd c5" build/st0 build/st25 build/st40 build/st50 build/st60 > gpurun_out/static_ab2.txt 2>&1

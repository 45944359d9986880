#!/bin/bash
# a static share of the chunks per wave before the work tickets (0 / 50 / 75 %)
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
bash scripts/ab_libs.sh "c4 dns c5" build/st0 build/st50 build/st75 > gpurun_out/static_ab.txt 2>&1

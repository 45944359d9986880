#!/bin/bash
# the "*" record's meta in the image (no dependent load for a miss) vs loaded
# from the table: pre2 (loaded) vs wild (in the image), C4, DNS and the C5 step
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
bash scripts/ab_libs.sh "c4 dns c5" build/pre2 build/wild > gpurun_out/wild_ab.txt 2>&1

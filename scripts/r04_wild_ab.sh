#!/bin/bash
# hint pass A/B: pre2 (offset pairs up front, "*" meta loaded from the table),
# wild ("*" meta in the image), pre3 / pre3w6 (and the next pair's offsets
# prefetched, at 7 and 6 waves per SIMD)
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
bash scripts/ab_libs.sh "c4 dns" build/pre2 build/wild build/pre3 build/pre3w6 > gpurun_out/wild_ab.txt 2>&1

#!/bin/bash
# occupancy of the call-free hint / DNS kernels: d1 (hint 7, DNS 6 waves per
# SIMD), dns7 (DNS 7: 72 VGPRs, no spills), h8 (hint 8: 64 VGPRs, 20 spilled)
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
bash scripts/ab_libs.sh "c4 dns" build/d1 build/dns7 build/h8 > gpurun_out/minw_ab.txt 2>&1

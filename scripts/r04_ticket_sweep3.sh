#!/bin/bash
# third sweep around 24 / 8 / 1 work tickets, and the next-pair offset
# prefetch at 6 waves per SIMD; C4, DNS, SNI
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
bash scripts/ab_libs.sh "c4 dns sni" build/s_base build/s_pre3w6 build/s_t20 build/s_t28 build/s_tl6 build/s_tl12 > gpurun_out/ticket_sweep3.txt 2>&1

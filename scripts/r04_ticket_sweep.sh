#!/bin/bash
# work-ticket layout for the call-free string kernels: chunks per big ticket,
# tail ticket size, tail rounds (base 16 / 4 / 2); C4 and DNS
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
bash scripts/ab_libs.sh "c4 dns" build/abl_base build/tk_16_4_1 build/tk_16_8_1 build/tk_24_4_2 build/tk_12_4_2 build/tk_16_2_2 build/tk_16_0 > gpurun_out/ticket_sweep.txt 2>&1

#!/bin/bash
# work-ticket layout, second sweep around 16 / 8 / 1 (chunks per big ticket,
# tail ticket size, tail rounds); the string and frame kernels that take tickets
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
bash scripts/ab_libs.sh "c4 dns sni mirror" build/abl_base build/tk_16_8_1 build/tk_24_8_1 build/tk_32_8_1 build/tk_16_16_1 build/tk_32_16_1 build/tk_16_8_2 > gpurun_out/ticket_sweep2.txt 2>&1

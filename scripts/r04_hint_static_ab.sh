#!/bin/bash
# hint_kernel's static share with the pair lane swap: 50 / 60 (default) / 70 %
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
bash scripts/ab_libs.sh "c4 c5" build/hs50 build/hs60 build/hs70 > gpurun_out/hint_static_ab.txt 2>&1

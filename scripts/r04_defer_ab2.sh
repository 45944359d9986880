#!/bin/bash
# second half of the deferral A/B: the DNS drain loop and the C5 step
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
bash scripts/ab_libs.sh "dnsd c5" build/base build/d1 > gpurun_out/defer_ab2.txt 2>&1

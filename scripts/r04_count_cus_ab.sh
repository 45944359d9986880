#!/bin/bash
# C5: the counter finish on all CUs (default) or CU-masked to 32 / 64
cd "$(dirname "$0")/.."
STEPS=20 bash scripts/ab_env.sh "all||" "c32||--count-cus 32" "c64||--count-cus 64" > gpurun_out/count_cus.txt 2>&1

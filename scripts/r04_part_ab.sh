#!/bin/bash
# partitioned work tickets for the deferring hint kernel: GPU tests (hint,
# DNS, C5) at the default build, then C4 / C5: the single counter (abl_base)
# vs 8 partitions at 16 / 32 chunks per big ticket
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests -m gpu \
    -k "hint or dns or c5 or pipeline or threads" > gpurun_out/part_tests.log 2>&1 || exit $?
bash scripts/ab_libs.sh "c4 c5" build/abl_base build/p16 build/p32 > gpurun_out/part_ab.txt 2>&1

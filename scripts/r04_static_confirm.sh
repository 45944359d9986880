#!/bin/bash
# per-kernel static shares (hint 60 %, DNS 50 %, SNI / mirror 25 %, drain loop
# 60 %): the GPU suite at the default build, then against no static share
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests -m gpu \
    > gpurun_out/static_tests.log 2>&1 || exit $?
bash scripts/ab_libs.sh "c4 dns sni mirror dnsd c5" build/st0 build/snew > gpurun_out/static_confirm.txt 2>&1

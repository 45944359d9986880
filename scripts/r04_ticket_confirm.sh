#!/bin/bash
# 24 / 8 / 1 work tickets (tnew, the default) against 16 / 4 / 2 (abl_base)
# on the DNS drain loop, the C5 step and C4; then the GPU tests that take
# tickets
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
bash scripts/ab_libs.sh "dnsd c5 c4" build/abl_base build/tnew > gpurun_out/ticket_confirm.txt 2>&1 || exit 1
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests -m gpu \
    -k "hint or dns or c5 or sni or cert or mirror or switch or parse or ticket" > gpurun_out/ticket_tests.log 2>&1

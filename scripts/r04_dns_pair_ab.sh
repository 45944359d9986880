#!/bin/bash
# the DNS kernel on chunk pairs: sw1 (one chunk per stage, the default),
# dp1 (pairs at 7 waves: 72 VGPRs, 11 spilled), dq1 (6 waves: 80, 1 spilled),
# dq5 (5 waves: 90 VGPRs, no scratch); the string parity tests on dq5 first
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
VCLASSIFY_LIB=build/dq5/libvclassify.so timeout -k 10 300 python -u -m pytest -x -q --timeout 200 \
    --timeout-method thread tests/test_gpu_00_parity.py tests/test_gpu_static_chunks.py -m gpu \
    > gpurun_out/dnspair_tests.log 2>&1 || exit $?
bash scripts/ab_libs.sh "dns" build/sw1 build/dp1 build/dq1 build/dq5 > gpurun_out/dns_pair_ab.txt 2>&1

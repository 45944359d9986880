#!/bin/bash
# the DNS kernel on chunk pairs (chunk_loop) with and without the lane swap:
# sw0 (neither), sw1 (swap in hint / cert), dp1 (swap + DNS pairs, 72 VGPRs: 11 spilled), dq1 (dp1 at 6 waves, 80 VGPRs: 1 spilled);
# the GPU suite at the default build, then the string parity tests on dp1 first
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests -m gpu \
    > gpurun_out/swap2_suite.log 2>&1 || exit $?
VCLASSIFY_LIB=build/dp1/libvclassify.so timeout -k 10 300 python -u -m pytest -x -q --timeout 200 \
    --timeout-method thread tests/test_gpu_00_parity.py tests/test_gpu_static_chunks.py -m gpu \
    > gpurun_out/swap2_tests.log 2>&1 || exit $?
bash scripts/ab_libs.sh "dns c4" build/sw0 build/sw1 build/dp1 build/dq1 > gpurun_out/swap_ab2.txt 2>&1

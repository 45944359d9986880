#!/bin/bash
# pair lane swap (each lane's shorter item in the pair's first body call):
# sw0 (off) against sw1 (hint + cert kernels), after the string parity tests
# on sw1
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
VCLASSIFY_LIB=build/sw1/libvclassify.so timeout -k 10 300 python -u -m pytest -x -q --timeout 200 \
    --timeout-method thread tests/test_gpu_00_parity.py tests/test_gpu_static_chunks.py -m gpu \
    > gpurun_out/swap_tests.log 2>&1 || exit $?
bash scripts/ab_libs.sh "c4 sni c5" build/sw0 build/sw1 > gpurun_out/swap_ab.txt 2>&1

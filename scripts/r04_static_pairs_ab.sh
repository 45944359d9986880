#!/bin/bash
# the static share as one contiguous block per wave (sp0) or as chunk pairs
# interleaved over the waves (sp1): tests of the interleaved build, then A/B
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
VCLASSIFY_LIB=build/sp1/libvclassify.so timeout -k 10 400 python -u -m pytest -x -q --timeout 300 \
    --timeout-method thread tests/test_gpu_static_chunks.py -m gpu > gpurun_out/sp_tests.log 2>&1 || exit $?
bash scripts/ab_libs.sh "c4 dns sni c5" build/sp0 build/sp1 > gpurun_out/sp_ab.txt 2>&1

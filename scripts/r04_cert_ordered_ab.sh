#!/bin/bash
# cert_kernel's results stored in item order after a pair's two body calls
# (co1) against in each call (co0, the default); string parity tests on co1
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
VCLASSIFY_LIB=build/co1/libvclassify.so timeout -k 10 300 python -u -m pytest -x -q --timeout 200 \
    --timeout-method thread tests/test_gpu_00_parity.py tests/test_gpu_static_chunks.py -m gpu \
    > gpurun_out/certord_tests.log 2>&1 || exit $?
bash scripts/ab_libs.sh "sni" build/co0 build/co1 > gpurun_out/cert_ordered_ab.txt 2>&1
bash scripts/ab_libs.sh "sni" build/co0 build/co1 >> gpurun_out/cert_ordered_ab.txt 2>&1

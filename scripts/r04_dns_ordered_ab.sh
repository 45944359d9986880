#!/bin/bash
# dns_kernel's results stored in item order after a pair's two body calls
# (do1) against in each call (do0, the default); string parity tests on do1
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
VCLASSIFY_LIB=build/do1/libvclassify.so timeout -k 10 300 python -u -m pytest -x -q --timeout 200 \
    --timeout-method thread tests/test_gpu_00_parity.py tests/test_gpu_static_chunks.py tests/test_gpu_c5.py -m gpu \
    > gpurun_out/dnsord_tests.log 2>&1 || exit $?
bash scripts/ab_libs.sh "dns" build/do0 build/do1 > gpurun_out/dns_ordered_ab.txt 2>&1
bash scripts/ab_libs.sh "dns" build/do0 build/do1 >> gpurun_out/dns_ordered_ab.txt 2>&1

#!/bin/bash
# hint / DNS / dnsd kernels without calls in their loops (deferred lanes and
# follow-up kernels) and the 16-byte-piece stage copy: GPU tests at the
# default build, then A/B
#   base: neither; q1: stage pieces; d0: deferral; d1: both (the default)
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests -m gpu \
    > gpurun_out/defer_tests.log 2>&1 || exit $?
bash scripts/ab_libs.sh "c4 dns" build/base build/q1 build/d0 build/d1 > gpurun_out/defer_ab.txt 2>&1

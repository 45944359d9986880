#!/bin/bash
# hint pool pass without calls in its loop (deferred lanes, hint_defer_kernel)
# and the 16-byte-piece stage copy: GPU tests at the default build, then A/B
#   base: neither; q1: stage pieces; d0: deferral; d1: both (the default)
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests -m gpu \
    > gpurun_out/defer_tests.log 2>&1 || exit $?
bash scripts/ab_libs.sh "c4 dns c5" build/base build/q1 build/d0 build/d1 > gpurun_out/defer_ab.txt 2>&1 || exit $?


#!/bin/bash
# switch kernel: the route root entry loaded before the ACL -- parity, then A/B against HEAD
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_frames_scale.py \
  tests/test_gpu_switch_loop.py tests/test_gpu_switch.py > gpurun_out/r06_switch_tests.log 2>&1 \
  || { tail -30 gpurun_out/r06_switch_tests.log; exit 1; }
tail -3 gpurun_out/r06_switch_tests.log
rm -f gpurun_out/ab/ab.jsonl
ROUNDS=3 bash scripts/ab_libs.sh "switch;c3" build/ab_head build/ab_pre

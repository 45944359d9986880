#!/bin/bash
# source kernels: lists in LDS -- parity, then A/B of the block size against the global table
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_source.py \
  > gpurun_out/r06_source_tests.log 2>&1 || { tail -30 gpurun_out/r06_source_tests.log; exit 1; }
tail -3 gpurun_out/r06_source_tests.log
rm -f gpurun_out/ab/ab.jsonl
ROUNDS=3 bash scripts/ab_libs.sh "source" build/ab_nolds build/ab_lds256 build/ab_lds512 build/ab_lds1024

#!/bin/bash
# hint follow-up kernel: wider scan -- parity, then A/B against HEAD
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_c4uri.py tests/test_gpu_00_parity.py tests/test_gpu_static_chunks.py tests/test_gpu_edges.py \
  > gpurun_out/r06_defer_tests.log 2>&1 || { tail -30 gpurun_out/r06_defer_tests.log; exit 1; }
tail -3 gpurun_out/r06_defer_tests.log
rm -f gpurun_out/ab/ab.jsonl
ROUNDS=3 bash scripts/ab_libs.sh "c4uri;c4" build/ab_head build/ab_scan1 build/ab_scan4 build/ab_scan8

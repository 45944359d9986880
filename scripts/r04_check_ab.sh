#!/bin/bash
# Round 4: GPU parity of the touched modules, then A/B of build/old vs build/new
# (scripts/ab_libs.sh) on the ACL and mixed-family sub-benches.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu \
  tests/test_gpu_00_parity.py tests/test_gpu_c5.py tests/test_gpu_pipeline.py tests/test_gpu_dnsd.py \
  tests/test_gpu_switch.py tests/test_gpu_acl_large.py tests/test_gpu_dnsd_loop.py \
  > gpurun_out/r04_tests_b.log 2>&1 || { tail -30 gpurun_out/r04_tests_b.log; exit 1; }
tail -2 gpurun_out/r04_tests_b.log
bash scripts/ab_libs.sh "${AB_WL:-c2 mix}" build/old build/new

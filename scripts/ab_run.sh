#!/bin/bash
# Round 5: host-entry mixed batches stage compact rows -- parity of every
# host-path pipeline test, then mixhost (row per packet) and mixhost
# --compact6 (caller-compacted rows), 32M packets at 15 % IPv6.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread \
  tests/test_gpu_pipeline.py tests/test_gpu_abi_c.py tests/test_gpu_hostpath.py > gpurun_out/r05_host_tests.log 2>&1 \
  || { tail -30 gpurun_out/r05_host_tests.log; exit 1; }
tail -1 gpurun_out/r05_host_tests.log
STEPS=5 bash scripts/ab_env.sh "mixhost||--workload mixhost" "mixhost_c6||--workload mixhost --compact6"

#!/bin/bash
# Round 5: the IPv6 wide root -- route / mixed-pipeline parity, then the C3
# and mix (compact and sparse) sub-benches with and without it
# (VC_ROUTE6_WIDE=0), two interleaved rounds.  -> gpurun_out/ab_env.jsonl
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread \
  tests/test_gpu_00_parity.py -k "route" tests/test_gpu_pipeline.py \
  tests/test_gpu_c5.py::test_mix_bench_batch_vs_oracle tests/test_gpu_switch.py > gpurun_out/r05_wide_tests.log 2>&1 \
  || { tail -30 gpurun_out/r05_wide_tests.log; exit 1; }
tail -1 gpurun_out/r05_wide_tests.log
STEPS=10 bash scripts/ab_env.sh "wide||--workload c3" "root|VC_ROUTE6_WIDE=0|--workload c3" \
  "wide_mix15c||--workload mix --compact6" "root_mix15c|VC_ROUTE6_WIDE=0|--workload mix --compact6" \
  "wide_mix15||--workload mix" "root_mix15|VC_ROUTE6_WIDE=0|--workload mix"

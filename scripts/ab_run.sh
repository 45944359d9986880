#!/bin/bash
# Round 5: one-step lookahead of the compact rows (pipe_mix_c6) -- parity,
# then mix --compact6 at 15 % and 50 % IPv6 against the previous build.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread \
  tests/test_gpu_pipeline.py tests/test_gpu_c5.py::test_mix_bench_batch_vs_oracle > gpurun_out/r05_la_tests.log 2>&1 \
  || { tail -30 gpurun_out/r05_la_tests.log; exit 1; }
tail -1 gpurun_out/r05_la_tests.log
ROUNDS=2 STEPS=10 bash scripts/ab_libs.sh "mix15c|--workload mix --compact6;mix50c|--workload mix --compact6 --v6-frac 0.5" build/head vproxy_amd

#!/bin/bash
# vc_pipeline_c6 (host compact rows): GPU tests, then mixhost with and without compact rows
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -v --timeout 200 --timeout-method thread \
    tests/test_gpu_pipeline.py -m gpu -k "host_entry_small" > gpurun_out/c6host_tests.log 2>&1 || exit $?
for c in "--compact6" "--compact6 --v6-frac 0" "--compact6 --v6-frac 0.5" "--v6-frac 0.5"; do
    timeout -k 10 300 python -u bench.py --workload mixhost --steps 10 --warmup 3 \
        --no-cpu-baseline $c >> gpurun_out/c6host_bench.jsonl 2> gpurun_out/c6host_bench.err || exit $?
done

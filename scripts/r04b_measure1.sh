#!/bin/bash
# Round-4 re-measurement at one commit, part 1: the GPU suite, the driver's
# C5 command and the first half of the sub-benches.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
mkdir -p gpurun_out
rm -f gpurun_out/sweep_*.log
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests -m gpu \
  > gpurun_out/r04_gpu_tests.log 2>&1 || { tail -30 gpurun_out/r04_gpu_tests.log; exit 1; }
tail -1 gpurun_out/r04_gpu_tests.log
timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/r04_bench_c5.json \
  2> gpurun_out/r04_bench_c5.err || { tail gpurun_out/r04_bench_c5.err; exit 1; }
tail -c 400 gpurun_out/r04_bench_c5.json
bash scripts/sweep.sh c1 c2 c2host c3 c4 dns dnsd

set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread -s \
    tests/test_gpu_pin_loop.py tests/test_gpu_zy_bench_ranks.py \
    > gpurun_out/r06_tests2.log 2>&1 || { echo TESTS FAILED; tail -30 gpurun_out/r06_tests2.log; exit 1; }
timeout -k 10 300 python -u bench.py --workload c4uri --steps 10 --warmup 3 \
    > gpurun_out/r06_c4uri.json 2> gpurun_out/r06_c4uri.err
timeout -k 10 300 python -u bench.py --steps 10 --warmup 3 \
    > gpurun_out/r06_c5.json 2> gpurun_out/r06_c5.err

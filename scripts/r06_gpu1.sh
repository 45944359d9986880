# round 6, first GPU pass: environment facts, the new tests, the c4uri and C5 lines
set -o pipefail
mkdir -p gpurun_out
bash scripts/r06_probe_env.sh > gpurun_out/r06_probe.txt 2>&1
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread \
    tests/test_gpu_pins.py tests/test_gpu_c4uri.py tests/test_gpu_pin_loop.py \
    "tests/test_gpu_00_parity.py" -k "pin or uri or hint or c4uri" -s \
    > gpurun_out/r06_tests1.log 2>&1 || { echo TESTS FAILED; tail -30 gpurun_out/r06_tests1.log; exit 1; }
timeout -k 10 300 python -u bench.py --workload c4uri --steps 10 --warmup 3 \
    > gpurun_out/r06_c4uri.json 2> gpurun_out/r06_c4uri.err
timeout -k 10 300 python -u bench.py --steps 10 --warmup 3 \
    > gpurun_out/r06_c5.json 2> gpurun_out/r06_c5.err

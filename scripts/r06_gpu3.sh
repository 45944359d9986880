# dnsd in place: its tests, then the dnsd / c4uri / c5 lines
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest -x -v --timeout 600 --timeout-method thread \
    tests/test_gpu_dnsd.py tests/test_gpu_dnsd_loop.py "tests/test_gpu_c5.py::test_dnsd_bench_workload" \
    tests/test_gpu_edges.py > gpurun_out/r06_tests3.log 2>&1 || { echo TESTS FAILED; tail -30 gpurun_out/r06_tests3.log; exit 1; }
for w in dnsd c4uri; do
  timeout -k 10 300 python -u bench.py --workload $w --steps 10 --warmup 3 --no-cpu-baseline \
      > gpurun_out/r06_${w}_d.json 2> gpurun_out/r06_${w}_d.err || exit 1
done
timeout -k 10 300 python -u bench.py --steps 10 --warmup 3 --no-cpu-baseline > gpurun_out/r06_c5_d.json 2> gpurun_out/r06_c5_d.err

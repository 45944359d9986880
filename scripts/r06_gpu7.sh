set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest -x -v --timeout 600 --timeout-method thread \
    tests/test_gpu_c4uri.py tests/test_gpu_00_parity.py tests/test_gpu_edges.py tests/test_gpu_http.py \
    > gpurun_out/r06_tests7.log 2>&1 || { echo TESTS FAILED; tail -30 gpurun_out/r06_tests7.log; exit 1; }
tail -2 gpurun_out/r06_tests7.log
for w in c4uri c4; do
  timeout -k 10 300 python -u bench.py --workload $w --steps 10 --warmup 3 --no-cpu-baseline \
      > gpurun_out/r06_${w}_g.json 2> gpurun_out/r06_${w}_g.err || exit 1
done
PASSES=trace bash scripts/prof.sh r06e "c4uri|--workload c4uri" > /dev/null 2>&1

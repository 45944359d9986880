# switch kernel with the bind port's ACL image: GPU tests, then the sub-bench
# A/B (VC_ACL_PORT=0: the general image) interleaved, then a kernel trace
set -o pipefail
mkdir -p gpurun_out
tag=${1:-r06s}
timeout -k 10 500 python -u -m pytest tests/test_gpu_switch.py tests/test_gpu_frames_scale.py tests/test_gpu_switch_loop.py tests/test_gpu_mirror.py -x -v -m gpu --timeout 300 --timeout-method thread > gpurun_out/${tag}_tests.log 2>&1 || { echo TESTS FAILED; tail -30 gpurun_out/${tag}_tests.log; exit 1; }
tail -2 gpurun_out/${tag}_tests.log
for r in 1 2; do
  for v in 1 0; do
    VC_ACL_PORT=$v timeout -k 10 200 python -u bench.py --workload switch --no-cpu-baseline > gpurun_out/${tag}_ab_${v}_${r}.json 2>> gpurun_out/${tag}_ab.err || exit 1
    echo "VC_ACL_PORT=$v run $r: $(python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(d['kernel_ms'], d['roofline']['frac'])" gpurun_out/${tag}_ab_${v}_${r}.json)"
  done
done
timeout -k 10 300 python -u bench.py --workload switch > gpurun_out/${tag}_bench.json 2> gpurun_out/${tag}_bench.err || exit 1
PASSES="trace" bash scripts/prof.sh ${tag}p "switch|--workload switch" > /dev/null 2>&1 || exit 1
grep -h switch_kernel gpurun_out/${tag}p/switch_trace/*kernel_stats.csv | cut -c1-220

set -o pipefail
mkdir -p gpurun_out
tag=${1:-r06mi}
timeout -k 10 400 python -u -m pytest tests/test_gpu_mirror.py -x -v -m gpu --timeout 300 --timeout-method thread > gpurun_out/${tag}_tests.log 2>&1 || { echo TESTS FAILED; tail -30 gpurun_out/${tag}_tests.log; exit 1; }
tail -2 gpurun_out/${tag}_tests.log
timeout -k 10 300 python -u bench.py --workload mirroritems > gpurun_out/${tag}_bench.json 2> gpurun_out/${tag}_bench.err || { tail -20 gpurun_out/${tag}_bench.err; exit 1; }
cut -c1-600 gpurun_out/${tag}_bench.json
PASSES="trace fetch write" bash scripts/prof.sh ${tag}p "mirroritems|--workload mirroritems" > /dev/null 2>&1 || exit 1
grep -h mirror_match gpurun_out/${tag}p/mirroritems_trace/*kernel_stats.csv | cut -c1-200

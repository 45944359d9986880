set -o pipefail
mkdir -p gpurun_out
tag=${1:-r06m2}
timeout -k 10 400 python -u -m pytest tests/test_gpu_mirror.py tests/test_gpu_frames_scale.py tests/test_gpu_edges.py -x -v -m gpu --timeout 300 --timeout-method thread > gpurun_out/${tag}_tests.log 2>&1 || { echo TESTS FAILED; tail -30 gpurun_out/${tag}_tests.log; exit 1; }
tail -2 gpurun_out/${tag}_tests.log
timeout -k 10 300 python -u scripts/mirror_items_probe.py > gpurun_out/${tag}_items.jsonl 2> gpurun_out/${tag}_items.err || { tail -20 gpurun_out/${tag}_items.err; exit 1; }
cat gpurun_out/${tag}_items.jsonl

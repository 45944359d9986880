# round-end rehearsal at head (after the container was re-created): the whole
# GPU suite + smoke, the driver's C5 command, then the mirror-kernel probe
set -o pipefail
mkdir -p gpurun_out
bash scripts/r06_suite.sh r06k || exit 1
timeout -k 10 300 python -u bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/r06k_bench_c5.json 2> gpurun_out/r06k_bench_c5.err || exit 1
cat gpurun_out/r06k_bench_c5.json
timeout -k 10 300 python -u scripts/mirror_probe.py > gpurun_out/r06k_mirror_probe.jsonl 2> gpurun_out/r06k_mirror_probe.err || exit 1
cat gpurun_out/r06k_mirror_probe.jsonl

# round-end rehearsal at head: the whole GPU suite + smoke, then the driver's C5 command
set -o pipefail
mkdir -p gpurun_out
bash scripts/r06_suite.sh r06f || exit 1
timeout -k 10 300 python -u bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/r06f_bench_c5.json 2> gpurun_out/r06f_bench_c5.err || exit 1
cat gpurun_out/r06f_bench_c5.json

# the round's last rehearsal: GPU suite + smoke, the driver's C5 command, and
# the mirror sub-bench after the lockstep searches
set -o pipefail
mkdir -p gpurun_out
bash scripts/r06_suite.sh r06z || exit 1
timeout -k 10 300 python -u bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/r06z_bench_c5.json 2> gpurun_out/r06z_bench_c5.err || exit 1
cut -c1-200 gpurun_out/r06z_bench_c5.json
timeout -k 10 300 python -u bench.py --workload mirror > gpurun_out/r06z_mirror.json 2> gpurun_out/r06z_mirror.err || exit 1
cut -c1-300 gpurun_out/r06z_mirror.json

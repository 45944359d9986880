# checkpoint at head: suite + smoke, the driver's C5 command, PMC passes of the round-6 kernels
set -o pipefail
mkdir -p gpurun_out
bash scripts/r06_suite.sh r06d || exit 1
timeout -k 10 300 python -u bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/r06_bench_c5_driver.json 2> gpurun_out/r06_bench_c5_driver.err || exit 1
PASSES="fetch write" bash scripts/prof.sh r06p "c4uri|--workload c4uri" "dnsd|--workload dnsd"

set -o pipefail
mkdir -p gpurun_out
bash scripts/r06_suite.sh r06b || exit 1
for w in dnsd c4uri; do
  timeout -k 10 300 python -u bench.py --workload $w --steps 10 --warmup 3 --no-cpu-baseline \
      > gpurun_out/r06_${w}_e.json 2> gpurun_out/r06_${w}_e.err || exit 1
done
timeout -k 10 300 python -u bench.py --steps 10 --warmup 3 --no-cpu-baseline > gpurun_out/r06_c5_e.json 2> gpurun_out/r06_c5_e.err

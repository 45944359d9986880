set -o pipefail
mkdir -p gpurun_out
bash scripts/r06_suite.sh r06c || exit 1
for w in dnsd c4uri http; do
  timeout -k 10 300 python -u bench.py --workload $w --steps 10 --warmup 3 --no-cpu-baseline \
      > gpurun_out/r06_${w}_f.json 2> gpurun_out/r06_${w}_f.err || exit 1
done
timeout -k 10 300 python -u bench.py --steps 10 --warmup 3 --no-cpu-baseline > gpurun_out/r06_c5_f.json 2> gpurun_out/r06_c5_f.err || exit 1
ROUNDS=2 STEPS=10 bash scripts/ab_libs.sh "dnsd" build/head build/dnsd5

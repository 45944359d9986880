set -o pipefail
mkdir -p gpurun_out
rm -f gpurun_out/ab/ab.jsonl
ROUNDS=3 STEPS=20 bash scripts/ab_libs.sh "c5|" build/r05 build/head || exit 1
cp gpurun_out/ab/ab.jsonl gpurun_out/r06_ab_c5_vs_r05.jsonl
PASSES=trace bash scripts/prof.sh r06d "c4uri|--workload c4uri" "dnsd|--workload dnsd" "http|--workload http" "c5|"

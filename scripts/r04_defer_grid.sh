#!/bin/bash
# grid of the deferred-lane kernels: 64 / 128 / 512 workgroups (kernel trace
# of C4 for the follow-up kernel's own time, then C4 / C5 A/B)
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp VC_BENCH_NO_E2E=1
for g in 64 512; do
  VCLASSIFY_LIB=build/g$g/libvclassify.so timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv \
    -d gpurun_out/dgrid_$g -o run -- python3 bench.py --workload c4 --steps 10 --warmup 2 --no-cpu-baseline \
    > gpurun_out/dgrid_$g.log 2>&1 || exit 1
done
bash scripts/ab_libs.sh "c4 c5" build/g64 build/g128 build/g512 > gpurun_out/dgrid_ab.txt 2>&1

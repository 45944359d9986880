#!/bin/bash
# call-free hint kernel: phase profile, then offset prefetch A/B (VC_HINT_PRE 0/1/2)
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
timeout -k 10 300 python -u scripts/hint_prof.py > gpurun_out/hint_prof.txt 2>&1 || exit $?
bash scripts/ab_libs.sh "c4" build/cur build/pre1 build/pre2 > gpurun_out/pre_ab.txt 2>&1

#!/bin/bash
# where the hint pass's time goes (timing only for the VC_ABL builds, which
# give wrong results): the work-ticket counter (16 / 32 / 64 chunks per ticket,
# or the static split) with and without the scan
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
bash scripts/ab_libs.sh "c4" build/abl_base build/abl_t32 build/abl_t64 build/abl_static build/abl_noscan build/abl_ns_t64 build/abl_ns_static > gpurun_out/hint_ablation2.txt 2>&1

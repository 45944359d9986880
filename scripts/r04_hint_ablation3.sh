#!/bin/bash
# the hint pass without its scan (timing-only builds): with / without the
# blob copy into LDS, on the work tickets / the static split
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
bash scripts/ab_libs.sh "c4" build/abl_ns build/abl_ns_nst build/abl_ns_static build/abl_ns_nst_static > gpurun_out/hint_ablation3.txt 2>&1

#!/bin/bash
# dns_kernel's static share on chunk pairs: 35 / 50 (default) / 65 / 80 %
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
bash scripts/ab_libs.sh "dns" build/ds35 build/ds50 build/ds65 build/ds80 > gpurun_out/dns_static_ab.txt 2>&1

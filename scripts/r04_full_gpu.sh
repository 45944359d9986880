#!/bin/bash
# the whole GPU suite at this tree
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
timeout -k 10 1000 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests -m gpu \
    > gpurun_out/full_gpu.log 2>&1

#!/bin/bash
# dnsd: ACL cost (timing-only ablation) and the UDP ACL as its own pass --
# the pass variant's parity first, then the interleaved A/B
set -o pipefail
mkdir -p gpurun_out
VCLASSIFY_LIB=build/ab_aclpass/libvclassify.so timeout -k 10 400 python -u -m pytest -x -v --timeout 300 \
  --timeout-method thread tests/test_gpu_dnsd.py tests/test_gpu_dnsd_loop.py > gpurun_out/r06_aclpass_tests.log 2>&1 \
  || { tail -30 gpurun_out/r06_aclpass_tests.log; exit 1; }
tail -3 gpurun_out/r06_aclpass_tests.log
rm -f gpurun_out/ab/ab.jsonl
ROUNDS=3 bash scripts/ab_libs.sh "dnsd" build/ab_head build/ab_noacl build/ab_aclpass
export TMPDIR=/tmp
VCLASSIFY_LIB=build/ab_aclpass/libvclassify.so timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv \
  -d gpurun_out/r06acl/trace2 -o run -- python3 bench.py --workload dnsd --steps 5 --warmup 2 --no-cpu-baseline \
  > gpurun_out/r06acl_b2.log 2>&1

#!/bin/bash
# Round 4: compact IPv6 rows -- GPU parity, then the mix bench sparse vs
# compact at 15 % and 50 % IPv6 (interleaved), then the C5 line three times.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu \
  tests/test_gpu_pipeline.py tests/test_gpu_c5.py > gpurun_out/r04_tests_c6.log 2>&1 \
  || { tail -30 gpurun_out/r04_tests_c6.log; exit 1; }
tail -1 gpurun_out/r04_tests_c6.log
: > gpurun_out/r04_c6_ab.jsonl
for rep in 1 2; do
  for f in 0.15 0.5; do
    for c in "" "--compact6"; do
      timeout -k 10 240 python3 bench.py --workload mix --v6-frac $f $c --steps 10 --warmup 3 \
        --no-cpu-baseline > gpurun_out/c6.log 2>&1 || { tail gpurun_out/c6.log; exit 1; }
      grep '^{' gpurun_out/c6.log | tail -1 >> gpurun_out/r04_c6_ab.jsonl
      python3 -c "import json,sys; d=json.loads(open('gpurun_out/r04_c6_ab.jsonl').read().splitlines()[-1]); print(d['v6_frac'], d['compact6'], d['kernel_only_ms'], d['v4_kernel_same_packets_ms'], d['kernel_ms'])"
    done
  done
done
for rep in 1 2 3; do
  timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/c5_rep$rep.json 2>/dev/null \
    || exit 1
  python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print('c5', d['value'], d['ms_per_step'])" gpurun_out/c5_rep$rep.json
done

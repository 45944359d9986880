#!/bin/bash
# Round 4: compact rows with the first round's rows issued before the IPv4
# gathers (build/new) against without (build/old), mix bench, interleaved.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
mkdir -p gpurun_out
: > gpurun_out/r04_c6_pf.jsonl
for rep in 1 2; do
  for f in 0.15 0.5; do
    for b in old new; do
      VCLASSIFY_LIB=build/$b/libvclassify.so timeout -k 10 240 python3 bench.py --workload mix \
        --v6-frac $f --compact6 --steps 10 --warmup 3 --no-cpu-baseline > gpurun_out/c6.log 2>&1 \
        || { tail gpurun_out/c6.log; exit 1; }
      grep '^{' gpurun_out/c6.log | tail -1 | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); d['build']='$b'; print(json.dumps(d))" >> gpurun_out/r04_c6_pf.jsonl
      python3 -c "import json; d=json.loads(open('gpurun_out/r04_c6_pf.jsonl').read().splitlines()[-1]); print(d['build'], d['v6_frac'], d['kernel_only_ms'], d['v4_kernel_same_packets_ms'])"
    done
  done
done

#!/bin/bash
# C5 schedule variants on one GPU box: scripts/ab_c5.sh "<args>" "<args>" ...
# Each argument string is one bench.py variant; all run twice, interleaved.
set -o pipefail
mkdir -p gpurun_out/abc5
k=0
for rep in 1 2; do
  k=0
  for a in "$@"; do
    k=$((k+1))
    timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline $a \
      > gpurun_out/abc5/v$k.$rep.json 2> gpurun_out/abc5/v$k.$rep.err || { echo "FAIL v$k [$a]"; tail -5 gpurun_out/abc5/v$k.$rep.err; exit 1; }
    python -c "
import json,sys
d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
print('v%s rep%s %-45s %9.1f  %.3f ms  pipe %.3f' % (sys.argv[2], sys.argv[3], sys.argv[4], d['value'], d['ms_per_step'], d['roofline'].get('kernel_ms', float('nan'))))
" gpurun_out/abc5/v$k.$rep.json $k $rep "$a"
  done
done

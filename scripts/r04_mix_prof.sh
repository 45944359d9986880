#!/bin/bash
# Round 4: the mixed-family pipeline at 0 / 15 / 50 % IPv6 (kernel alone and
# the IPv4 kernel over the same packets), then PMC passes of the FETCH
# calibration, C5 and the 15 % mix (scripts/prof_r04.sh).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
mkdir -p gpurun_out
for f in 0 0.15 0.5; do
  timeout -k 10 240 python3 bench.py --workload mix --v6-frac $f --steps 10 --warmup 3 --no-cpu-baseline \
    > gpurun_out/mix_f$f.log 2>&1 || { tail gpurun_out/mix_f$f.log; exit 1; }
  grep '^{' gpurun_out/mix_f$f.log | tail -1
done
bash scripts/prof_r04.sh cal c5 mix

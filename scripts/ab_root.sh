#!/bin/bash
# Route-root A/B (DESIGN.md §2 "Could a smaller route root move the ceiling?"):
# parity at a 20-bit root first, then the C5 step and the C3 route kernels
# with 24- vs 20-bit roots (two interleaved rounds), then TCC hits/misses per
# pipeline launch for each.  Results: gpurun_out/ab_env.jsonl, gpurun_out/rootpmc/
# (committed as profiles/r03_ab_root.jsonl).  The VC_ROUTE_ROOT_BITS_V4/V6
# knob it sets existed at commit 660aa3a only (compile.cpp default_root_bits).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
R20="VC_ROUTE_ROOT_BITS_V4=20 VC_ROUTE_ROOT_BITS_V6=20"
T="python -u -m pytest -x -v --timeout 240 --timeout-method thread"
PMC="timeout -s KILL 90 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum --output-format csv"
bash scripts/gpu_steps.sh \
  "root20_parity:600:$R20 $T tests/test_gpu_c5.py tests/test_gpu_00_parity.py -k 'route or c5 or mix or pipeline'" \
  "root_ab:600:bash scripts/ab_env.sh 'rb24||' 'rb20|$R20|' 'c3_rb24||--workload c3' 'c3_rb20|$R20|--workload c3'" \
  "pmc24:120:$PMC -d gpurun_out/rootpmc/rb24 -o run -- python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline" \
  "pmc20:120:$R20 $PMC -d gpurun_out/rootpmc/rb20 -o run -- python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline"

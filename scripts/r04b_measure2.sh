#!/bin/bash
# Round-4 re-measurement at one commit, part 2: the other sub-benches and the
# trace / PMC passes of c5, c4 and dns.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
mkdir -p gpurun_out
rm -f gpurun_out/sweep_*.log
bash scripts/sweep.sh sni parse switch source mirror mix mixhost || exit 1
bash scripts/prof_r04.sh c5 c4 dns

#!/bin/bash
# Round 5: the pool pass without its record loads (timing-only ablation
# VC_ABL_NOREC: every tag hit taken as a match) against the real kernel, on
# C4 and the C5 step: the most a smaller / denser record layout can give.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
mkdir -p build/head && cp vproxy_amd/libvclassify.so build/head/
ROUNDS=2 bash scripts/ab_libs.sh "c4;c5" build/head build/norec

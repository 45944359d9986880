#!/bin/bash
# Round 5: the frame kernels (parse, mirror, switch, dnsd) with the staged
# copy's nontemporal loads (base, the default) against plain loads; interleaved.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
ROUNDS=2 bash scripts/ab_libs.sh "parse;mirror;switch;dnsd" build/base build/plain

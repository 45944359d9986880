#!/bin/bash
# Round 5: the string kernels' chunk-loop offset loads nontemporal (VC_OFF_NT)
# against plain loads (both with the nontemporal staged copy); interleaved.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
ROUNDS=2 bash scripts/ab_libs.sh "c4;dns;sni;c5" build/base build/offnt

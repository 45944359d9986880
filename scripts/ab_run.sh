#!/bin/bash
# Round 5: the source-hash kernel through the per-position pick table with
# four items per lane (the tree) against the probing kernel (build/base).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
mkdir -p build/head && cp vproxy_amd/libvclassify.so build/head/
ROUNDS=2 bash scripts/ab_libs.sh "source" build/base build/head

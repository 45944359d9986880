#!/bin/bash
# Round 5: the compact mixed-family kernel overlapping its single IPv6
# round's root gathers with the IPv4 ACL searches (the tree) against the
# round-then-ACL order (build/base, VC_MIX_OVERLAP=0).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
mkdir -p build/head && cp vproxy_amd/libvclassify.so build/head/
ROUNDS=2 bash scripts/ab_libs.sh "mixc6|--workload mix --compact6" build/base build/head

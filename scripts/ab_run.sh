#!/bin/bash
# Round 5: the switch kernel with the inner IPv4 route's root entry loaded
# before the bare-VXLAN ACL (the tree) against the serial chain (build/base).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
mkdir -p build/head && cp vproxy_amd/libvclassify.so build/head/
ROUNDS=2 bash scripts/ab_libs.sh "switch" build/base build/head

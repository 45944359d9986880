#!/bin/bash
# Round 5: the deferring DNS drain-loop kernel with 96-char qname buffers
# (longer names deferred; seven workgroups per CU) against 128-char ones.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
mkdir -p build/head && cp vproxy_amd/libvclassify.so build/head/
ROUNDS=2 bash scripts/ab_libs.sh "dnsd" build/base build/head

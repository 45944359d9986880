#!/bin/bash
# Round 5: the DNS drain loop without its UDP ACL search (timing-only
# ablation VC_ABL_NOACL) against the real kernel: the ACL chain's share.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
ROUNDS=2 bash scripts/ab_libs.sh "dnsd" build/base build/noacl

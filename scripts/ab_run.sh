#!/bin/bash
# Round 5: C2 with the ACL interval search removed (timing-only ablation,
# VC_ABL_NOSEARCH) against the real kernel: the most any faster search can gain.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
ROUNDS=2 bash scripts/ab_libs.sh "c2" build/base build/nosearch

#!/bin/bash
# full check of the tree (tests, smoke, bench) + the GroupNorm apply and attention A/Bs
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
SKIP_PROF=1 bash tools/gpu/full_check.sh ${1:-r4b} || exit 1
bash tools/gpu/gn_ab.sh || exit 1
bash tools/gpu/attn_ab.sh

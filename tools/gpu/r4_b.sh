#!/bin/bash
# full check of the tree (tests, smoke, bench, profiles) + the GroupNorm apply A/B
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
SKIP_PROF=${SKIP_PROF:-0} bash tools/gpu/full_check.sh ${1:-r4b} || exit 1
bash tools/gpu/gn_ab.sh

#!/bin/bash
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
bash tools/gpu/r6_n.sh && bash tools/gpu/r6_o.sh

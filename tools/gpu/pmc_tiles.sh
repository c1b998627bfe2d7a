#!/bin/bash
# PMC of the 8-wave deep-ring tiles (configs 26 / 27) against the 4-wave tiles they replaced
# (3 = 128x64 4-wave, 12 = 128x128 4-wave deep ring), forced on the level-3 shapes they serve
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
for arm in "g26:26:gemm 2048 1280 1280" "g27:27:gemm 2048 1280 1280" "g3:3:gemm 2048 1280 1280" "g12:12:gemm 2048 1280 1280" \
           "c26:26:conv 8 16 640 1280" "c3:3:conv 8 16 640 1280"; do
  name=${arm%%:*}; rest=${arm#*:}; cfg=${rest%%:*}; op=${rest#*:}
  CASSMANTLE_GEMM_CFG=$cfg ITERS=10 TOP=2 CFG_NOTE="cfg $cfg: " CMD="python tools/one_op.py $op" bash tools/gpu/pmc_table.sh tiles_$name || exit 1
done

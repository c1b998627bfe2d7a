#!/bin/bash
# PMC of the producer-wave deep rings (configs 31 / 33: 8 MFMA + 8 LDS-DMA-only waves) against the
# tiles they replaced on the shapes they serve: level-3 projection (26: 8-wave 128x80), level-2
# 3x3 conv (8: ping-pong 256x160) and level-2 projection (20: ping-pong 128x160)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
for arm in "g31:31:gemm 2048 1280 1280" "g26:26:gemm 2048 1280 1280" \
           "c33:33:conv 8 32 640 640" "c8:8:conv 8 32 640 640" \
           "l33:33:gemm 8192 640 2560" "l20:20:gemm 8192 640 2560"; do
  name=${arm%%:*}; rest=${arm#*:}; cfg=${rest%%:*}; op=${rest#*:}
  CASSMANTLE_GEMM_CFG=$cfg ITERS=10 TOP=2 CFG_NOTE="cfg $cfg: " CMD="python tools/one_op.py $op" bash tools/gpu/pmc_table.sh ptiles_$name || exit 1
done

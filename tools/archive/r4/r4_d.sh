#!/bin/bash
# GroupNorm apply variants and the attention micro-changes, each measured alone (same box)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
bash tools/gpu/so_ab.sh gnv shape us "python tools/bench_membound.py --gn-only" gn_v0 tree gn_v1 gn_v3 gn_v4 || exit 1
bash tools/gpu/so_ab.sh atv shape us.bf16 "python tools/bench_attn.py --rounds 3 --iters 10" tree at_perm at_bl at_prio || exit 1

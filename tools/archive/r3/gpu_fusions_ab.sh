#!/bin/bash
# same-box A/B of the round-3 launch fusions, all off vs all on (LayerNorm row statistics from producer
# epilogues, GroupNorm folded into proj_in), SD-1.5 and SDXL
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
for r in 1 2; do
  for e in "CASSMANTLE_LN_ROWSTATS=0 CASSMANTLE_GN_FOLD=0" "CASSMANTLE_X=1"; do
    env $e timeout -k 10 300 python -u bench.py --steps 4 --warmup 2 --no-score --no-batch1 > gpurun_out/ab_one.log 2>&1 || { tail -5 gpurun_out/ab_one.log; exit 1; }
    echo "sd15 $e | $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/ab_one.log) $(grep -o '"stage_mean_ms": {[^}]*}' gpurun_out/ab_one.log)" | tee -a gpurun_out/fusions_ab3.txt
  done
done
for r in 1 2; do
  for e in "CASSMANTLE_LN_ROWSTATS=0 CASSMANTLE_GN_FOLD=0" "CASSMANTLE_X=1"; do
    env $e timeout -k 10 400 python -u bench.py --model sdxl --batch 1 --fp8-attention --steps 2 --warmup 1 --no-score --no-batch1 \
      > gpurun_out/ab_one.log 2>&1 || { tail -5 gpurun_out/ab_one.log; exit 1; }
    echo "sdxl $e | $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/ab_one.log) $(grep -o '"stage_mean_ms": {[^}]*}' gpurun_out/ab_one.log)" | tee -a gpurun_out/fusions_ab3.txt
  done
done

#!/bin/bash
# SDXL config 4 (1024^2, 30 Euler steps, batch 1, fp8 attention): UNet batch branches 1 vs 2
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
for r in 1 2; do
  for b in 1 2; do
    timeout -k 10 400 python -u bench.py --model sdxl --batch 1 --fp8-attention --steps 2 --warmup 1 --no-score --no-batch1 \
      --branches $b > gpurun_out/sx.log 2>&1 || { tail -5 gpurun_out/sx.log; exit 1; }
    echo "sdxl branches=$b | $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/sx.log) $(grep -o '"stage_mean_ms": {[^}]*}' gpurun_out/sx.log)" | tee -a gpurun_out/sdxl_branch_ab.txt
  done
done

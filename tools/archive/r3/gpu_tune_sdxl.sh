#!/bin/bash
# in-situ re-tune of the SDXL shapes over all tile configs, then SDXL config-4 A/B old vs new table
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
cp cassmantle_amd/ops/gemm_tuning.json gpurun_out/tune_sdxl.json
timeout -k 10 1000 python -u tools/autotune_gemm.py --models sdxl --batch 1 --merge --out gpurun_out/tune_sdxl.json \
  > gpurun_out/autotune_sdxl.log 2>&1 || { tail -5 gpurun_out/autotune_sdxl.log; exit 1; }
tail -1 gpurun_out/autotune_sdxl.log
for r in 1 2; do
  for t in old new; do
    if [ $t = new ]; then e=CASSMANTLE_GEMM_TUNE_PATH=gpurun_out/tune_sdxl.json; else e=X=0; fi
    env $e timeout -k 10 400 python -u bench.py --model sdxl --batch 1 --fp8-attention --steps 2 --warmup 1 --no-score --no-batch1 \
      > gpurun_out/ab_one.log 2>&1 || { tail -5 gpurun_out/ab_one.log; exit 1; }
    echo "sdxl table=$t | $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/ab_one.log) $(grep -o '"stage_mean_ms": {[^}]*}' gpurun_out/ab_one.log)" | tee -a gpurun_out/tune_sdxl_ab.txt
  done
done

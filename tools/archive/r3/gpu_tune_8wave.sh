#!/bin/bash
# in-situ tune of the 8-wave deep-ring tiles (configs 26 / 27) against the current table plans
# (SD-1.5 batch 4 and SDXL batch 1 shapes), then same-box A/B old vs new table on both models
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
cp cassmantle_amd/ops/gemm_tuning.json gpurun_out/tune_8w.json
timeout -k 10 600 python -u tools/autotune_gemm.py --models sd15 --merge --cfgs 26,27 --out gpurun_out/tune_8w.json \
  > gpurun_out/autotune_8w_sd15.log 2>&1 || { tail -5 gpurun_out/autotune_8w_sd15.log; exit 1; }
tail -1 gpurun_out/autotune_8w_sd15.log
timeout -k 10 600 python -u tools/autotune_gemm.py --models sdxl --batch 1 --merge --cfgs 26,27 --out gpurun_out/tune_8w.json \
  > gpurun_out/autotune_8w_sdxl.log 2>&1 || { tail -5 gpurun_out/autotune_8w_sdxl.log; exit 1; }
tail -1 gpurun_out/autotune_8w_sdxl.log
for r in 1 2; do
  for t in old new; do
    if [ $t = new ]; then e=CASSMANTLE_GEMM_TUNE_PATH=gpurun_out/tune_8w.json; else e=X=0; fi
    env $e timeout -k 10 400 python -u bench.py --steps 3 --warmup 1 --no-score --no-batch1 \
      > gpurun_out/ab_one.log 2>&1 || { tail -5 gpurun_out/ab_one.log; exit 1; }
    echo "sd15 table=$t | $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/ab_one.log)" | tee -a gpurun_out/tune_8w_ab.txt
    env $e timeout -k 10 400 python -u bench.py --model sdxl --batch 1 --fp8-attention --steps 2 --warmup 1 --no-score --no-batch1 \
      > gpurun_out/ab_one.log 2>&1 || { tail -5 gpurun_out/ab_one.log; exit 1; }
    echo "sdxl table=$t | $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/ab_one.log)" | tee -a gpurun_out/tune_8w_ab.txt
  done
done

#!/bin/bash
# SDXL: full in-situ re-tune (every live config x split) merged into the table, then a same-box
# bench A/B of the tables (SDXL fp8 attention, and SD-1.5 to check nothing regressed)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
cp cassmantle_amd/ops/gemm_tuning.json gpurun_out/tune_prev.json
cp cassmantle_amd/ops/gemm_tuning.json gpurun_out/tune_new.json
timeout -k 10 800 python tools/autotune_gemm.py --models sdxl --batch 1 --merge --out gpurun_out/tune_new.json > gpurun_out/tune_full_sdxl.log 2>&1 || { tail -20 gpurun_out/tune_full_sdxl.log; exit 1; }
tail -1 gpurun_out/tune_full_sdxl.log
for rep in 1 2; do
  for v in prev new; do
    CASSMANTLE_GEMM_TUNE_PATH=gpurun_out/tune_$v.json timeout -k 10 300 python bench.py --model sdxl --batch 1 --fp8-attention --steps 3 --warmup 1 --no-score --no-batch1 > gpurun_out/fullx_ab_${v}_$rep.json 2> gpurun_out/fullx_ab_${v}_$rep.err || { tail -5 gpurun_out/fullx_ab_${v}_$rep.err; exit 1; }
    echo "sdxl $v $rep $(python -c "import json;print(json.load(open('gpurun_out/fullx_ab_${v}_$rep.json'))['ms_per_step'])")"
  done
done

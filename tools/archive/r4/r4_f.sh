#!/bin/bash
# Re-tune the GEMM/conv plan table on the current kernels (every live config x split, in situ,
# existing plans kept as arms), then A/B the SD-1.5 bench step on the old vs new table (same box)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
cp cassmantle_amd/ops/gemm_tuning.json gpurun_out/tune_prev.json
cp cassmantle_amd/ops/gemm_tuning.json gpurun_out/tune_new.json
timeout -k 10 600 python tools/autotune_gemm.py --models sd15 --batch 4 --merge --out gpurun_out/tune_new.json > gpurun_out/tune_sd15.log 2>&1 || { tail -20 gpurun_out/tune_sd15.log; exit 1; }
tail -2 gpurun_out/tune_sd15.log
timeout -k 10 600 python tools/autotune_gemm.py --models sdxl --batch 1 --merge --out gpurun_out/tune_new.json > gpurun_out/tune_sdxl.log 2>&1 || { tail -20 gpurun_out/tune_sdxl.log; exit 1; }
tail -2 gpurun_out/tune_sdxl.log
for rep in 1 2; do
  for v in prev new; do
    CASSMANTLE_GEMM_TUNE_PATH=gpurun_out/tune_$v.json timeout -k 10 300 python bench.py --steps 6 --warmup 2 --no-score --no-batch1 > gpurun_out/tune_ab_${v}_$rep.json 2> gpurun_out/tune_ab_${v}_$rep.err || { tail -5 gpurun_out/tune_ab_${v}_$rep.err; exit 1; }
    echo "$v $rep $(python -c "import json;print(json.load(open('gpurun_out/tune_ab_${v}_$rep.json'))['ms_per_step'])")"
  done
done

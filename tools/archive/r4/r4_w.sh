#!/bin/bash
# cold-weight in-situ tune (every arm timed with its weight read from HBM on every call) of the
# SD-1.5 shapes, then a same-box bench A/B of the tables
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
cp cassmantle_amd/ops/gemm_tuning.json gpurun_out/tune_prev.json
cp cassmantle_amd/ops/gemm_tuning.json gpurun_out/tune_new.json
timeout -k 10 800 python tools/autotune_gemm.py --models sd15 --batch 4 --merge --cold 512 --out gpurun_out/tune_new.json > gpurun_out/tune_cold_sd15.log 2>&1 || { tail -20 gpurun_out/tune_cold_sd15.log; exit 1; }
tail -1 gpurun_out/tune_cold_sd15.log
for rep in 1 2; do
  for v in prev new; do
    CASSMANTLE_GEMM_TUNE_PATH=gpurun_out/tune_$v.json timeout -k 10 300 python bench.py --steps 6 --warmup 2 --no-score --no-batch1 > gpurun_out/cold_ab_${v}_$rep.json 2> gpurun_out/cold_ab_${v}_$rep.err || { tail -5 gpurun_out/cold_ab_${v}_$rep.err; exit 1; }
    echo "sd15 $v $rep $(python -c "import json;print(json.load(open('gpurun_out/cold_ab_${v}_$rep.json'))['ms_per_step'])")"
  done
done

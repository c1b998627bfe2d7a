#!/bin/bash
# producer-wave deep rings (configs 23 / 24 (ping-pong 128x160 / 128x128 with 8 producer waves)): forced-config numerics, in-situ tune of those configs
# against the current table's plans (SD-1.5 and SDXL shapes), then a same-box bench A/B of the tables
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_kernels_gpu.py -x -q -m gpu -k "pp or conv or geglu" --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/r4v_tests.log 2>&1 || { tail -30 gpurun_out/r4v_tests.log; exit 1; }
tail -1 gpurun_out/r4v_tests.log
cp cassmantle_amd/ops/gemm_tuning.json gpurun_out/tune_prev.json
cp cassmantle_amd/ops/gemm_tuning.json gpurun_out/tune_new.json
timeout -k 10 500 python tools/autotune_gemm.py --models sd15 --batch 4 --merge --cfgs 23,24 --out gpurun_out/tune_new.json > gpurun_out/tune_pppw_sd15.log 2>&1 || { tail -20 gpurun_out/tune_pppw_sd15.log; exit 1; }
tail -3 gpurun_out/tune_pppw_sd15.log
timeout -k 10 500 python tools/autotune_gemm.py --models sdxl --batch 1 --merge --cfgs 23,24 --out gpurun_out/tune_new.json > gpurun_out/tune_pppw_sdxl.log 2>&1 || { tail -20 gpurun_out/tune_pppw_sdxl.log; exit 1; }
tail -3 gpurun_out/tune_pppw_sdxl.log
for rep in 1 2; do
  for v in prev new; do
    CASSMANTLE_GEMM_TUNE_PATH=gpurun_out/tune_$v.json timeout -k 10 300 python bench.py --steps 6 --warmup 2 --no-score --no-batch1 > gpurun_out/pppw_ab_${v}_$rep.json 2> gpurun_out/pppw_ab_${v}_$rep.err || { tail -5 gpurun_out/pppw_ab_${v}_$rep.err; exit 1; }
    echo "sd15 $v $rep $(python -c "import json;print(json.load(open('gpurun_out/pppw_ab_${v}_$rep.json'))['ms_per_step'])")"
  done
done
for rep in 1 2; do
  for v in prev new; do
    CASSMANTLE_GEMM_TUNE_PATH=gpurun_out/tune_$v.json timeout -k 10 300 python bench.py --model sdxl --batch 1 --fp8-attention --steps 3 --warmup 1 --no-score --no-batch1 > gpurun_out/pppwx_ab_${v}_$rep.json 2> gpurun_out/pppwx_ab_${v}_$rep.err || { tail -5 gpurun_out/pppwx_ab_${v}_$rep.err; exit 1; }
    echo "sdxl $v $rep $(python -c "import json;print(json.load(open('gpurun_out/pppwx_ab_${v}_$rep.json'))['ms_per_step'])")"
  done
done

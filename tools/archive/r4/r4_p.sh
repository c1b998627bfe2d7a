#!/bin/bash
# hybrid producer-wave tiles (34-36: 31-33 with the MFMA waves staging too): numerics, the probe
# (warm / cold weights) against 31-33, in-situ tune of 34-36 and a same-box bench A/B of the tables
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_kernels_gpu.py -x -q -m gpu -k "pp or conv or producer_wave" --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/r4p_tests.log 2>&1 || { tail -30 gpurun_out/r4p_tests.log; exit 1; }
tail -1 gpurun_out/r4p_tests.log
timeout -k 10 300 python tools/cold_weight_probe.py --arms 31:1,34:1,32:1,35:1,33:1,36:1 --iters 40 > gpurun_out/r4p_probe.jsonl 2> gpurun_out/r4p_probe.err || { tail -20 gpurun_out/r4p_probe.err; exit 1; }
cat gpurun_out/r4p_probe.jsonl
cp cassmantle_amd/ops/gemm_tuning.json gpurun_out/tune_prev.json
cp cassmantle_amd/ops/gemm_tuning.json gpurun_out/tune_new.json
timeout -k 10 500 python tools/autotune_gemm.py --models sd15 --batch 4 --merge --cfgs 34,35,36 --out gpurun_out/tune_new.json > gpurun_out/tune_mix_sd15.log 2>&1 || { tail -20 gpurun_out/tune_mix_sd15.log; exit 1; }
tail -1 gpurun_out/tune_mix_sd15.log
timeout -k 10 500 python tools/autotune_gemm.py --models sdxl --batch 1 --merge --cfgs 34,35,36 --out gpurun_out/tune_new.json > gpurun_out/tune_mix_sdxl.log 2>&1 || { tail -20 gpurun_out/tune_mix_sdxl.log; exit 1; }
tail -1 gpurun_out/tune_mix_sdxl.log
for rep in 1 2; do
  for v in prev new; do
    CASSMANTLE_GEMM_TUNE_PATH=gpurun_out/tune_$v.json timeout -k 10 300 python bench.py --steps 6 --warmup 2 --no-score --no-batch1 > gpurun_out/mix_ab_${v}_$rep.json 2> gpurun_out/mix_ab_${v}_$rep.err || { tail -5 gpurun_out/mix_ab_${v}_$rep.err; exit 1; }
    echo "sd15 $v $rep $(python -c "import json;print(json.load(open('gpurun_out/mix_ab_${v}_$rep.json'))['ms_per_step'])")"
  done
done
for rep in 1 2; do
  for v in prev new; do
    CASSMANTLE_GEMM_TUNE_PATH=gpurun_out/tune_$v.json timeout -k 10 300 python bench.py --model sdxl --batch 1 --fp8-attention --steps 3 --warmup 1 --no-score --no-batch1 > gpurun_out/mixx_ab_${v}_$rep.json 2> gpurun_out/mixx_ab_${v}_$rep.err || { tail -5 gpurun_out/mixx_ab_${v}_$rep.err; exit 1; }
    echo "sdxl $v $rep $(python -c "import json;print(json.load(open('gpurun_out/mixx_ab_${v}_$rep.json'))['ms_per_step'])")"
  done
done

#!/bin/bash
# fp8 K/V from the QKV epilogue: kernel + model tests, SDXL bf16 vs fp8 bench (x2 interleaved),
# SD-1.5 bench (epilogue change must not cost the headline), decode-graph A/B
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_kernels_gpu.py -x -q --timeout 120 --timeout-method thread -k "fp8 or qkv_epilogue or ln_linear or gemm" > gpurun_out/r3_kv8_tests.txt 2>&1
rc=$?; tail -3 gpurun_out/r3_kv8_tests.txt; [ $rc -ne 0 ] && { grep -E "Error|assert" gpurun_out/r3_kv8_tests.txt | head; exit $rc; }
timeout -k 10 400 python -u -m pytest tests/test_models_gpu.py -x -q --timeout 200 --timeout-method thread -k "sdxl or fp8" > gpurun_out/r3_kv8_mtests.txt 2>&1
rc=$?; tail -3 gpurun_out/r3_kv8_mtests.txt; [ $rc -ne 0 ] && exit $rc
for r in 1 2; do
  for arm in bf16 fp8; do
    extra=""; [ $arm = fp8 ] && extra="--fp8-attention"
    timeout -k 10 300 python -u bench.py --model sdxl --batch 1 --steps 3 --warmup 1 --denoise-steps 10 --no-score --no-batch1 $extra > gpurun_out/sdxl_ab.log 2>&1 || { tail -5 gpurun_out/sdxl_ab.log; exit 1; }
    echo "sdxl $arm | $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/sdxl_ab.log) $(grep -o '"stage_mean_ms": {[^}]*}' gpurun_out/sdxl_ab.log)" | tee -a gpurun_out/r3_sdxl_fp8_ab.txt
  done
done
for r in 1 2; do
  for vg in 1 0; do
    CASSMANTLE_VAE_GRAPH=$vg timeout -k 10 200 python -u bench.py --steps 5 --warmup 2 --no-score --no-batch1 > gpurun_out/sd15_ab.log 2>&1 || { tail -5 gpurun_out/sd15_ab.log; exit 1; }
    echo "sd15 vae_graph=$vg | $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/sd15_ab.log) $(grep -o '"stage_mean_ms": {[^}]*}' gpurun_out/sd15_ab.log)" | tee -a gpurun_out/r3_sd15_vaegraph_ab.txt
  done
done

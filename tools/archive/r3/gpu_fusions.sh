#!/bin/bash
# Round-3 launch fusions (LayerNorm row statistics from producer epilogues, GroupNorm folded into proj_in,
# graph-captured text encoders): numerics and model parity, then same-box A/B all-off vs all-on, SD-1.5 and SDXL
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_kernels_gpu.py tests/test_models_gpu.py -x -q \
  -k "row_stats or gn_linear or ln_ or layer_norm or full_size or sdxl or end_to_end or graph_replay or deterministic or clip_encode" \
  --timeout 300 --timeout-method thread > gpurun_out/fusions_tests.txt 2>&1
rc=$?; tail -2 gpurun_out/fusions_tests.txt; [ $rc -ne 0 ] && { grep -E "FAIL|Error|assert" gpurun_out/fusions_tests.txt | head -30; exit $rc; }
for r in 1 2; do
  for e in "CASSMANTLE_LN_ROWSTATS=0 CASSMANTLE_GN_FOLD=0 CASSMANTLE_TEXT_GRAPH=0" "CASSMANTLE_X=1"; do
    env $e timeout -k 10 300 python -u bench.py --steps 4 --warmup 2 --no-score --no-batch1 > gpurun_out/ab_one.log 2>&1 || { tail -5 gpurun_out/ab_one.log; exit 1; }
    echo "sd15 $e | $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/ab_one.log) $(grep -o '"stage_mean_ms": {[^}]*}' gpurun_out/ab_one.log)" | tee -a gpurun_out/fusions_ab.txt
  done
done
for r in 1 2; do
  for e in "CASSMANTLE_LN_ROWSTATS=0 CASSMANTLE_GN_FOLD=0 CASSMANTLE_TEXT_GRAPH=0" "CASSMANTLE_X=1"; do
    env $e timeout -k 10 400 python -u bench.py --model sdxl --batch 1 --fp8-attention --steps 2 --warmup 1 --no-score --no-batch1 \
      > gpurun_out/ab_one.log 2>&1 || { tail -5 gpurun_out/ab_one.log; exit 1; }
    echo "sdxl $e | $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/ab_one.log) $(grep -o '"stage_mean_ms": {[^}]*}' gpurun_out/ab_one.log)" | tee -a gpurun_out/fusions_ab.txt
  done
done

#!/bin/bash
# staggered-wave attention (CASSMANTLE_ATTN_DB=3) and 4-wave blocks (CASSMANTLE_ATTN_NW=4) vs the
# double-buffered default: numerics under each knob, microbenchmark, then the bench A/B
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
for e in CASSMANTLE_ATTN_DB=3 CASSMANTLE_ATTN_NW=4; do
  env $e timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -x -q -k "attention or attn" --timeout 120 \
    --timeout-method thread > gpurun_out/attn_tests.txt 2>&1
  rc=$?; echo "$e: $(tail -1 gpurun_out/attn_tests.txt)"; [ $rc -ne 0 ] && { grep -E "FAIL|Error|assert" gpurun_out/attn_tests.txt | head -20; exit $rc; }
done
for r in 1 2; do
  for e in X=0 CASSMANTLE_ATTN_DB=3 CASSMANTLE_ATTN_NW=4; do
    env $e timeout -k 10 200 python -u tools/bench_attn.py --rounds 3 --iters 20 > gpurun_out/ba.log 2>&1 || { tail -5 gpurun_out/ba.log; exit 1; }
    echo "$e | $(head -3 gpurun_out/ba.log | cut -c1-160 | tr '\n' ' ')" | tee -a gpurun_out/attn_stag_ab.txt
  done
done
for r in 1 2; do
  for e in X=0 CASSMANTLE_ATTN_DB=3; do
    env $e timeout -k 10 300 python -u bench.py --steps 4 --warmup 2 --no-score --no-batch1 > gpurun_out/ab_one.log 2>&1 || { tail -5 gpurun_out/ab_one.log; exit 1; }
    echo "$e | $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/ab_one.log) $(grep -o '"stage_mean_ms": {[^}]*}' gpurun_out/ab_one.log)" | tee -a gpurun_out/attn_stag_ab.txt
  done
done

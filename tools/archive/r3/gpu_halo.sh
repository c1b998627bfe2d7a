#!/bin/bash
# halo-staged conv: numerics tests, then the per-shape microbenchmark
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -x -q -k "halo" --timeout 120 --timeout-method thread \
  > gpurun_out/halo_tests.txt 2>&1
rc=$?; tail -3 gpurun_out/halo_tests.txt; [ $rc -ne 0 ] && { grep -E "FAIL|Error|assert" gpurun_out/halo_tests.txt | head -30; exit $rc; }
timeout -k 10 400 python -u tools/bench_halo.py > gpurun_out/bench_halo.jsonl 2>&1 || { tail -5 gpurun_out/bench_halo.jsonl; exit 1; }
cut -c1-400 gpurun_out/bench_halo.jsonl
# in-situ autotune with the halo configs (batch-4 room = the bench's shapes), then same-box A/B
cp cassmantle_amd/ops/gemm_tuning.json gpurun_out/tune_halo.json
timeout -k 10 900 python -u tools/autotune_gemm.py --batch 4 --merge --out gpurun_out/tune_halo.json \
  > gpurun_out/autotune_halo.log 2>&1 || { tail -5 gpurun_out/autotune_halo.log; exit 1; }
tail -1 gpurun_out/autotune_halo.log
grep -c '"best": \[2[45],' gpurun_out/autotune_halo.log
for r in 1 2; do
  for t in old new; do
    if [ $t = new ]; then e=CASSMANTLE_GEMM_TUNE_PATH=gpurun_out/tune_halo.json; else e=X=0; fi
    env $e timeout -k 10 300 python -u bench.py --steps 4 --warmup 2 --no-score --no-batch1 > gpurun_out/ab_one.log 2>&1 \
      || { tail -5 gpurun_out/ab_one.log; exit 1; }
    echo "table=$t | $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/ab_one.log) $(grep -o '"stage_mean_ms": {[^}]*}' gpurun_out/ab_one.log)" | tee -a gpurun_out/halo_ab.txt
  done
done

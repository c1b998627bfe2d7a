#!/bin/bash
# UNet batch branches (pipeline branches=N): branch tests, same-box interleaved bench A/B of 1 / 2 / 4
# branches, tuning-table entries for the half-batch shapes, A/B again with them.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
out=gpurun_out/branch_ab.txt
timeout -k 10 600 python -u -m pytest tests/test_models_gpu.py -x -q -k "branches or graph_replay" --timeout 300 \
  --timeout-method thread > gpurun_out/branch_tests.txt 2>&1
rc=$?; tail -3 gpurun_out/branch_tests.txt; [ $rc -ne 0 ] && { grep -E "FAIL|Error|assert" gpurun_out/branch_tests.txt | head -20; exit $rc; }
ab() {   # ab LABEL [env...]
  for r in 1 2; do
    for b in 1 2 4; do
      env "$@" timeout -k 10 300 python -u bench.py --steps 4 --warmup 2 --no-score --no-batch1 --branches $b \
        > gpurun_out/ab_one.log 2>&1 || { tail -5 gpurun_out/ab_one.log; exit 1; }
      echo "$1 branches=$b | $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/ab_one.log) $(grep -o '"stage_mean_ms": {[^}]*}' gpurun_out/ab_one.log)" | tee -a $out
    done
  done
}
ab table=r2 CASSMANTLE_X=0 || exit 1
cp cassmantle_amd/ops/gemm_tuning.json gpurun_out/tune_half.json
timeout -k 10 900 python -u tools/autotune_gemm.py --batch 2 --merge --out gpurun_out/tune_half.json \
  > gpurun_out/autotune_half.log 2>&1 || { tail -5 gpurun_out/autotune_half.log; exit 1; }
tail -1 gpurun_out/autotune_half.log
timeout -k 10 900 python -u tools/autotune_gemm.py --batch 1 --merge --out gpurun_out/tune_half.json \
  > gpurun_out/autotune_quarter.log 2>&1 || { tail -5 gpurun_out/autotune_quarter.log; exit 1; }
tail -1 gpurun_out/autotune_quarter.log
ab table=half CASSMANTLE_GEMM_TUNE_PATH=gpurun_out/tune_half.json || exit 1

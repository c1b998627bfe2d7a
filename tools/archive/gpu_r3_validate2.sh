#!/bin/bash
# round-3 glue kernels / CU masks / SDXL path: targeted GPU tests, SDXL + SD-1.5 traces (non-in-tree
# kernel census), same-box bench vs the round-2 tree, live round with and without CU reservation
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests/test_kernels_gpu.py tests/test_models_gpu.py -x -q --timeout 300 --timeout-method thread > gpurun_out/r3_gpu_tests2.txt 2>&1
rc=$?; tail -3 gpurun_out/r3_gpu_tests2.txt
[ $rc -ne 0 ] && { grep -E "FAIL|Error" gpurun_out/r3_gpu_tests2.txt | head -20; exit $rc; }
bash tools/gpu_profile.sh r3_sdxl_fp8 sdxl 4 8 --batch 1 --fp8-attention || exit 1
bash tools/gpu_profile.sh r3_sd15 sd15 10 24 || exit 1
grep -A12 "non-in-tree" gpurun_out/prof_r3_sd15_summary.txt gpurun_out/prof_r3_sdxl_fp8_summary.txt
for r in 1 2; do
  for tree in r2base .; do
    (cd $tree && timeout -k 10 300 python -u bench.py --steps 5 --warmup 2 --no-score --no-batch1) > gpurun_out/ab_tree.log 2>&1 || { tail -5 gpurun_out/ab_tree.log; exit 1; }
    echo "tree=$tree | $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/ab_tree.log) $(grep -o '"stage_mean_ms": {[^}]*}' gpurun_out/ab_tree.log)" | tee -a gpurun_out/r3_ab_vs_r2.txt
  done
done
for rc_ in 0 8 16; do
  timeout -k 10 300 python -u tools/bench_live.py --seconds 20 --idle-s 5 --reserve-cus $rc_ > gpurun_out/live_$rc_.log 2>&1 || { tail -5 gpurun_out/live_$rc_.log; exit 1; }
  grep '^{' gpurun_out/live_$rc_.log | tee -a gpurun_out/r3_live_cumask.jsonl
done

#!/bin/bash
# full GPU suite + smoke, SD-1.5/SDXL kernel traces (non-in-tree kernel census), and a same-box
# bench A/B of this tree against the round-2 tree (r2base/)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r3_gpu_tests.txt 2>&1
rc=$?; tail -3 gpurun_out/r3_gpu_tests.txt
[ $rc -ne 0 ] && { grep -E "FAIL|Error" gpurun_out/r3_gpu_tests.txt | head -20; exit $rc; }
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r3_smoke.txt 2>&1 || { tail -20 gpurun_out/r3_smoke.txt; exit 1; }
tail -1 gpurun_out/r3_smoke.txt
bash tools/gpu_profile.sh r3_sd15 sd15 10 24 || exit 1
bash tools/gpu_profile.sh r3_sdxl_fp8 sdxl 4 8 --batch 1 --fp8-attention || exit 1
grep -A12 "non-in-tree" gpurun_out/prof_r3_sd15_summary.txt
# r2base/: the round-2 tree (commit 02d221a: python + its own extension build), same box
for r in 1 2; do
  for tree in r2base .; do
    (cd $tree && timeout -k 10 300 python -u bench.py --steps 5 --warmup 2 --no-score --no-batch1) > gpurun_out/ab_tree.log 2>&1 || { tail -5 gpurun_out/ab_tree.log; exit 1; }
    echo "tree=$tree | $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/ab_tree.log) $(grep -o '"stage_mean_ms": {[^}]*}' gpurun_out/ab_tree.log)" | tee -a gpurun_out/r3_ab_vs_r2.txt
  done
done

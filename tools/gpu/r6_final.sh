#!/bin/bash
# round 6 final-tree check: GPU suite, the driver's bench command (with the config-4 / 5 extras),
# steady-state per-eval kernel profiles of SD-1.5 and SDXL fp8
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/r6final
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider \
  > $O/tests.txt 2>&1 || { tail -40 $O/tests.txt; exit 1; }
tail -1 $O/tests.txt
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.txt 2>&1 || { tail -20 $O/smoke.txt; exit 1; }
tail -1 $O/smoke.txt
t0=$(date +%s)
timeout -k 10 400 python bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench.json 2> $O/bench.err || { tail -30 $O/bench.err; exit 1; }
echo "bench wall $(( $(date +%s) - t0 )) s"
cat $O/bench.json
bash tools/gpu/profile.sh r6final_sd15 sd15 10 24 > /dev/null && cp gpurun_out/prof_r6final_sd15_steady.txt $O/ && head -12 $O/prof_r6final_sd15_steady.txt
bash tools/gpu/profile.sh r6final_sdxl sdxl 4 10 --batch 1 --fp8-attention > /dev/null && cp gpurun_out/prof_r6final_sdxl_steady.txt $O/ && head -12 $O/prof_r6final_sdxl_steady.txt
rm -rf gpurun_out/prof_r6final_sd15 gpurun_out/prof_r6final_sdxl

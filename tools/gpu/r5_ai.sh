#!/bin/bash
# round 5 final tree: steady-state per-eval profiles of SD-1.5 and SDXL (fp8)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
bash tools/gpu/profile.sh r5fin_sd15 sd15 10 24 || exit 1
bash tools/gpu/profile.sh r5fin_sdxl sdxl 4 10 --batch 1 --fp8-attention || exit 1
rm -rf gpurun_out/prof_r5fin_sd15 gpurun_out/prof_r5fin_sdxl

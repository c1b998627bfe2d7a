#!/bin/bash
# bench + per-eval kernel profiles + PMC tables of SD-1.5 and SDXL (fp8 attention) on one box
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
tag=${1:-r4c}
mkdir -p gpurun_out
timeout -k 10 300 python bench.py --steps 10 --warmup 2 --no-score > gpurun_out/${tag}_bench.json 2> gpurun_out/${tag}_bench.err || { tail -20 gpurun_out/${tag}_bench.err; exit 1; }
cat gpurun_out/${tag}_bench.json
bash tools/gpu/profile.sh ${tag}_sd15 sd15 10 24 || exit 1
bash tools/gpu/profile.sh ${tag}_sdxl sdxl 4 10 --batch 1 --fp8-attention || exit 1
TOP=14 bash tools/gpu/pmc_table.sh ${tag}_sd15 --model sd15 --denoise-steps 2 || exit 1
TOP=14 bash tools/gpu/pmc_table.sh ${tag}_sdxl --model sdxl --batch 1 --fp8-attention --denoise-steps 2 || exit 1

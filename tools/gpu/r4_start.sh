#!/bin/bash
# Round-4 starting point on one box: driver-contract bench, then per-eval kernel profiles of
# SD-1.5 and SDXL (fp8 attention) on the same box.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python bench.py --steps 20 --warmup 3 --no-score > gpurun_out/r4s_bench.json 2> gpurun_out/r4s_bench.err || { tail -20 gpurun_out/r4s_bench.err; exit 1; }
cat gpurun_out/r4s_bench.json
bash tools/gpu/profile.sh sd15 sd15 10 24 || exit 1
bash tools/gpu/profile.sh sdxl sdxl 4 10 --batch 1 --fp8-attention || exit 1

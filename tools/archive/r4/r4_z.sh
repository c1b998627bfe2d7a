#!/bin/bash
# full-tree check final tree of the round: GPU suite, smoke, driver-contract bench, SDXL bench
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
SKIP_PROF=1 bash tools/gpu/full_check.sh r4z || exit 1
timeout -k 10 400 python bench.py --model sdxl --batch 1 --fp8-attention --steps 5 --warmup 1 --no-score --no-batch1 > gpurun_out/r4z_sdxl.json 2> gpurun_out/r4z_sdxl.err || { tail -20 gpurun_out/r4z_sdxl.err; exit 1; }
cat gpurun_out/r4z_sdxl.json

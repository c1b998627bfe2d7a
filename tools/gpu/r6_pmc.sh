#!/bin/bash
# round 6: PMC tables of the final tree (SD-1.5 bench shape, 2 PNDM steps; SDXL fp8, 2 Euler steps)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
TOP=16 bash tools/gpu/pmc_table.sh r6_sd15 --denoise-steps 2 || exit 1
CMD="python bench.py --model sdxl --fp8-attention --batch 1 --steps 1 --warmup 0 --no-score --no-batch1 --no-live --no-sdxl --no-graphs --denoise-steps 2" TOP=16 bash tools/gpu/pmc_table.sh r6_sdxl || exit 1
rm -rf gpurun_out/pmc_r6_sd15/pmc_p* gpurun_out/pmc_r6_sd15/trace gpurun_out/pmc_r6_sdxl/pmc_p* gpurun_out/pmc_r6_sdxl/trace

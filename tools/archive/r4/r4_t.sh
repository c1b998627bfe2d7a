#!/bin/bash
# PMC tables of the final tree (SD-1.5, SDXL fp8 attention): the model steps on the final table
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
TOP=16 bash tools/gpu/pmc_table.sh r4t_sd15 --model sd15 --denoise-steps 2 || exit 1
TOP=16 bash tools/gpu/pmc_table.sh r4t_sdxl --model sdxl --batch 1 --fp8-attention --denoise-steps 2 || exit 1

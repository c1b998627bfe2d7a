#!/bin/bash
# round 6: SD-1.5 PMC table after the d40 attention staging change (compare profiles/r6_pmc_final_tables.txt)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
TOP=16 bash tools/gpu/pmc_table.sh r6_sd15b --denoise-steps 2 || exit 1
rm -rf gpurun_out/pmc_r6_sd15b/pmc_p* gpurun_out/pmc_r6_sd15b/trace

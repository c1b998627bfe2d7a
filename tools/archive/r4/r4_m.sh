#!/bin/bash
# final-table profiles: per-UNet-eval kernel traces of SD-1.5 and SDXL (fp8 attention), then PMC of
# the producer-wave tiles against the tiles they replaced
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
bash tools/gpu/profile.sh r4m_sd15 sd15 10 24 || exit 1
bash tools/gpu/profile.sh r4m_sdxl sdxl 4 10 --batch 1 --fp8-attention || exit 1
bash tools/gpu/pmc_tiles2.sh || exit 1

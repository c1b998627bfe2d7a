#!/bin/bash
# MFMA shape probe (tools/mfma_shape_probe.hip): 16x16x32 vs 32x32x16 bf16 from LDS, random data
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out /tmp/probe
hipcc --offload-arch=gfx950 -O3 -std=c++17 tools/mfma_shape_probe.hip -o /tmp/probe/mfma_shape_probe || exit 1
timeout -k 10 120 /tmp/probe/mfma_shape_probe 4000 | tee gpurun_out/mfma_shape_probe.jsonl

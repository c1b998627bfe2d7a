#!/bin/bash
# L2 -> LDS fill-rate probe (tools/lds_fill_probe.hip) on one GPU: B/cycle/CU vs waves per CU and
# DMAs in flight, from a 64 MiB (Infinity Cache) and an 8 MiB (L2) source window.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
hipcc --offload-arch=gfx950 -O3 -std=c++17 tools/lds_fill_probe.hip -o /tmp/lds_fill_probe || exit 1
timeout -k 10 120 /tmp/lds_fill_probe | tee gpurun_out/lds_fill.jsonl

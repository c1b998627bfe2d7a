#!/bin/bash
# round 5: forced-plan sweep of the level-1 / level-2 conv-shaped GEMMs + the vendor kernels' tiles
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u tools/probe_vs_blas.py --shapes 32768x320x2880,8192x640x2880,8192x640x5760 \
  --cfgs 8:1,9:1,20:1,21:1,33:1,14:1,1:1,0:1,5:1,8:2,20:2 > gpurun_out/probe_vs_blas3.jsonl 2>&1 || { tail -20 gpurun_out/probe_vs_blas3.jsonl; exit 1; }
cat gpurun_out/probe_vs_blas3.jsonl
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/blasprof -o run --output-format csv -- \
  python tools/probe_vs_blas.py --shapes 32768x320x2880,8192x640x5760,2048x1280x5120,4096x4096x4096 > gpurun_out/blasprof.log 2>&1 || { tail -20 gpurun_out/blasprof.log; exit 1; }
f=$(find gpurun_out/blasprof -name '*kernel_stats.csv' | head -1)
cut -d, -f1-4 "$f" | head -30

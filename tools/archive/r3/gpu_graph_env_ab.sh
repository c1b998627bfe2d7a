#!/bin/bash
# HIP runtime knobs vs the per-kernel floor of a replayed graph (tools/probe_small_gemm.py: empty
# kernel and a 1-k-tile GEMM, 20 dependent launches per graph), then the bench under the best
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
out=gpurun_out/graph_env_ab.txt
for r in 1 2; do
  for e in "X=0" "DEBUG_CLR_GRAPH_PACKET_CAPTURE=0" "DEBUG_CLR_GRAPH_PACKET_CAPTURE=1" "AMD_DIRECT_DISPATCH=0" "AMD_DIRECT_DISPATCH=1" "DEBUG_HIP_GRAPH_BATCH_SIZE=1" "DEBUG_HIP_GRAPH_BATCH_SIZE=256"; do
    env $e timeout -k 10 120 python -u tools/probe_small_gemm.py --ks 64,1280 --cfgs 3 > gpurun_out/ge.log 2>&1 || { tail -3 gpurun_out/ge.log; echo "$e failed" | tee -a $out; continue; }
    echo "$e | $(grep -o '"us": [0-9.]*' gpurun_out/ge.log | head -1) | $(grep -o '"auto": [0-9.]*' gpurun_out/ge.log | tr '\n' ' ')" | tee -a $out
  done
done

#!/bin/bash
# Serving-side checks on one GPU: the 64-player live round (BASELINE config 5: generation + streaming
# guess scoring, scorer tail under load) and the multi-rank bench path rehearsed with 2 ranks on the
# one GPU over gloo (the driver's N > 1 runs use RCCL; two ranks cannot share a device under RCCL)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u tools/bench_live.py --seconds 20 --idle-s 5 > gpurun_out/live.log 2>&1 \
  || { tail -8 gpurun_out/live.log; exit 1; }
grep '^{' gpurun_out/live.log | tee gpurun_out/live_round.jsonl
CASSMANTLE_DIST_BACKEND=gloo timeout -k 10 600 python -u -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \
  --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --steps 2 --warmup 1 --no-score --no-batch1 \
  > gpurun_out/dp2.log 2>&1 || { tail -8 gpurun_out/dp2.log; exit 1; }
grep '^{' gpurun_out/dp2.log | tee gpurun_out/dp2_gloo_rehearsal.json | cut -c1-600

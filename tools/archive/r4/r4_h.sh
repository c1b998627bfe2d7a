#!/bin/bash
# supervised serving topology on one GPU: worker-death recovery time (SD-1.5) and the live round
# (generation + streaming scoring) through the supervised group
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
timeout -k 10 500 python tools/bench_recovery.py --gpus 1 --model sd15 > gpurun_out/r4h_recovery.json 2> gpurun_out/r4h_recovery.err || { tail -20 gpurun_out/r4h_recovery.err; exit 1; }
cat gpurun_out/r4h_recovery.json
timeout -k 10 400 python tools/bench_live.py --gpus 1 --players 64 --seconds 25 --idle-s 6 > gpurun_out/r4h_live.json 2> gpurun_out/r4h_live.err || { tail -20 gpurun_out/r4h_live.err; exit 1; }
grep '^{' gpurun_out/r4h_live.json

#!/bin/bash
# round 5: steady-state per-eval kernel profiles (last generation only) of SD-1.5 (bench shape)
# and SDXL (fp8 attention), and the attention microbench at every shape
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out/r5h
bash tools/gpu/profile.sh sd15 sd15 10 22 && bash tools/gpu/profile.sh sdxl sdxl 5 10 --batch 1 --fp8-attention || exit 1
timeout -k 10 300 python tools/bench_attn.py --rounds 5 > gpurun_out/r5h/attn_all.jsonl 2> gpurun_out/r5h/attn_all.err || { tail -5 gpurun_out/r5h/attn_all.err; exit 1; }
cat gpurun_out/r5h/attn_all.jsonl

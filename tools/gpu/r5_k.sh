#!/bin/bash
# round 5: GEGLU probe (gated vs plain at the same width, per tile)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
timeout -k 10 300 python -u tools/probe_geglu.py > gpurun_out/probe_geglu.jsonl 2>&1 || { tail -30 gpurun_out/probe_geglu.jsonl; exit 1; }
cat gpurun_out/probe_geglu.jsonl
timeout -k 10 300 python -u tools/probe_geglu.py --m 8192 --k 640 --n 2560 > gpurun_out/probe_geglu_l2.jsonl 2>&1 || { tail -30 gpurun_out/probe_geglu_l2.jsonl; exit 1; }
cat gpurun_out/probe_geglu_l2.jsonl

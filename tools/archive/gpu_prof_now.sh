#!/bin/bash
# in-situ kernel trace of the benchmark step (10 PNDM steps = 12 UNet evals, warm-up + timed step)
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_now -o run --output-format csv -- \
  python bench.py --steps 1 --warmup 1 --denoise-steps 10 --no-score --no-batch1 > gpurun_out/prof_now.log 2>&1 || { tail -20 gpurun_out/prof_now.log; exit 1; }
grep '^{' gpurun_out/prof_now.log | head -c 300; echo
f=$(find gpurun_out/prof_now -name '*kernel_trace.csv' | head -1)
python tools/prof_summary.py "$f" --per 24 --top 45 > gpurun_out/prof_now_summary.txt && head -70 gpurun_out/prof_now_summary.txt

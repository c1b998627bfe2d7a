#!/bin/bash
# round 5: batch-1 (config 2) steady-state profile + cold/warm GEMM diag at batch 1
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
bash tools/gpu/profile.sh b1 sd15 10 24 --batch 1 > gpurun_out/prof_b1.txt 2>&1 || { tail -20 gpurun_out/prof_b1.txt; exit 1; }
head -45 gpurun_out/prof_b1_steady.txt
CASSMANTLE_DIAG_TWICE=1 CASSMANTLE_DIAG_TWICE_ACK=wrong-results timeout -k 10 500 rocprofv3 --kernel-trace -d gpurun_out/prof_twice_b1 -o run --output-format csv -- \
  python bench.py --model sd15 --batch 1 --steps 1 --warmup 1 --denoise-steps 10 --no-score --no-batch1 > gpurun_out/prof_twice_b1.log 2>&1 || { tail -20 gpurun_out/prof_twice_b1.log; exit 1; }
f=$(find gpurun_out/prof_twice_b1 -name '*kernel_trace.csv' | head -1)
python tools/diag_twice.py "$f" --top 25 > gpurun_out/diag_twice_b1.txt && cat gpurun_out/diag_twice_b1.txt
rm -rf gpurun_out/prof_twice_b1 gpurun_out/prof_b1

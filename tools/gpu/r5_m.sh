#!/bin/bash
# round 5: cold vs warm GEMM/conv cost in situ (each launch twice; timing diagnostic only)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
CASSMANTLE_DIAG_TWICE=1 CASSMANTLE_DIAG_TWICE_ACK=wrong-results timeout -k 10 500 rocprofv3 --kernel-trace -d gpurun_out/prof_twice -o run --output-format csv -- \
  python bench.py --model sd15 --steps 1 --warmup 1 --denoise-steps 10 --no-score --no-batch1 > gpurun_out/prof_twice.log 2>&1 || { tail -20 gpurun_out/prof_twice.log; exit 1; }
f=$(find gpurun_out/prof_twice -name '*kernel_trace.csv' | head -1)
python tools/diag_twice.py "$f" --top 40 > gpurun_out/diag_twice_sd15.txt && cat gpurun_out/diag_twice_sd15.txt
CASSMANTLE_DIAG_TWICE=1 CASSMANTLE_DIAG_TWICE_ACK=wrong-results timeout -k 10 500 rocprofv3 --kernel-trace -d gpurun_out/prof_twice_xl -o run --output-format csv -- \
  python bench.py --model sdxl --fp8-attention --steps 1 --warmup 1 --denoise-steps 4 --batch 1 --no-score --no-batch1 > gpurun_out/prof_twice_xl.log 2>&1 || { tail -20 gpurun_out/prof_twice_xl.log; exit 1; }
f=$(find gpurun_out/prof_twice_xl -name '*kernel_trace.csv' | head -1)
python tools/diag_twice.py "$f" --top 40 > gpurun_out/diag_twice_sdxl.txt && cat gpurun_out/diag_twice_sdxl.txt
rm -rf gpurun_out/prof_twice gpurun_out/prof_twice_xl

#!/bin/bash
# Round-4 starting point on one box: the new RCCL data-plane GPU tests, the driver-contract
# bench, then per-eval kernel profiles of SD-1.5 and SDXL (fp8 attention) on the same box.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_parallel_gpu.py -x -v --timeout 300 --timeout-method thread > gpurun_out/r4s_tests.log 2>&1 || { tail -40 gpurun_out/r4s_tests.log; exit 1; }
tail -5 gpurun_out/r4s_tests.log
timeout -k 10 300 python bench.py --steps 20 --warmup 3 --no-score > gpurun_out/r4s_bench.json 2> gpurun_out/r4s_bench.err || { tail -20 gpurun_out/r4s_bench.err; exit 1; }
cat gpurun_out/r4s_bench.json
bash tools/gpu/profile.sh sd15 sd15 10 24 || exit 1
bash tools/gpu/profile.sh sdxl sdxl 4 10 --batch 1 --fp8-attention || exit 1

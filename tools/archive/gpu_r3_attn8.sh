#!/bin/bash
# fp8 attention block variants: numerics, microbenchmark; then the captured-decode pipeline
# tests + bench and the live-round GIL switch-interval sweep
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -x -q --timeout 120 --timeout-method thread -k "fp8" > gpurun_out/r3_attn8_tests.txt 2>&1
rc=$?; tail -3 gpurun_out/r3_attn8_tests.txt; [ $rc -ne 0 ] && exit $rc
timeout -k 10 200 python -u tools/bench_attn_fp8.py > gpurun_out/r3_attn8_bench.jsonl 2>&1 || { tail -5 gpurun_out/r3_attn8_bench.jsonl; exit 1; }
cat gpurun_out/r3_attn8_bench.jsonl
bash tools/gpu_r3_live.sh

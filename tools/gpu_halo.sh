#!/bin/bash
# halo-staged conv: numerics tests, then the per-shape microbenchmark
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -x -q -k "halo" --timeout 120 --timeout-method thread \
  > gpurun_out/halo_tests.txt 2>&1
rc=$?; tail -3 gpurun_out/halo_tests.txt; [ $rc -ne 0 ] && { grep -E "FAIL|Error|assert" gpurun_out/halo_tests.txt | head -30; exit $rc; }
timeout -k 10 400 python -u tools/bench_halo.py > gpurun_out/bench_halo.jsonl 2>&1 || { tail -5 gpurun_out/bench_halo.jsonl; exit 1; }
cut -c1-400 gpurun_out/bench_halo.jsonl

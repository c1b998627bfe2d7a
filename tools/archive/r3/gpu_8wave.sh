#!/bin/bash
# 8-wave deep-ring tiles (configs 26 / 27): numerics on every forced-config test, then the
# small-GEMM probe (K sweep at M 2048 x N 1280) against the 4-wave tiles.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -x -q --timeout 120 --timeout-method thread \
  -m gpu -k "_pp" > gpurun_out/t8w.log 2>&1 || { tail -30 gpurun_out/t8w.log; exit 1; }
tail -2 gpurun_out/t8w.log
timeout -k 10 300 python -u tools/probe_small_gemm.py --cfgs 3,16,26,27,28 --ks 320,640,1280,2560 | tee gpurun_out/probe8w.jsonl
timeout -k 10 300 python -u tools/probe_small_gemm.py --m 8192 --n 640 --cfgs 3,26,27,28,21 --ks 640,1280 | tee -a gpurun_out/probe8w.jsonl

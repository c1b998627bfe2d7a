#!/bin/bash
# GroupNorm apply small-shape sizing fix: numerics, then a same-box A/B of the applies (gn_prev = before)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -x -q -m gpu -k "group_norm" --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/r4x_tests.log 2>&1 || { tail -30 gpurun_out/r4x_tests.log; exit 1; }
tail -1 gpurun_out/r4x_tests.log
bash tools/gpu/so_ab.sh gny shape us "python tools/bench_membound.py --gn-only" gn_prev tree || exit 1

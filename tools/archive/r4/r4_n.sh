#!/bin/bash
# 6-stage producer-wave rings (34/35): forced-config numerics, then the cold-weight probe (weights
# from HBM on every call, as in a UNet eval) vs warm (what the in-situ tuner measures)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_kernels_gpu.py -x -q -m gpu -k "pp or conv or producer_wave" --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/r4n_tests.log 2>&1 || { tail -30 gpurun_out/r4n_tests.log; exit 1; }
tail -1 gpurun_out/r4n_tests.log
timeout -k 10 600 python tools/cold_weight_probe.py > gpurun_out/r4n_cold.jsonl 2> gpurun_out/r4n_cold.err || { tail -20 gpurun_out/r4n_cold.err; exit 1; }
cat gpurun_out/r4n_cold.jsonl

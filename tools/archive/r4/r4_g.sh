#!/bin/bash
# epilogue change (batched residual loads, hoisted per-column operands): GEMM/conv numerics, then
# same-box A/Bs of the ResNet convs, the residual projections and the bench step (ep_old = before)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_kernels_gpu.py tests/test_models_gpu.py -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/r4g_tests.log 2>&1 || { tail -30 gpurun_out/r4g_tests.log; exit 1; }
tail -2 gpurun_out/r4g_tests.log
bash tools/gpu/so_ab.sh epc shape us "python tools/bench_resnet_convs.py" ep_old tree || exit 1
bash tools/gpu/so_ab.sh epl shape us "python tools/bench_resnet_convs.py --linear" ep_old tree || exit 1
bash tools/gpu/so_ab.sh epb config.model ms_per_step "python bench.py --steps 6 --warmup 2 --no-score --no-batch1" ep_old tree || exit 1

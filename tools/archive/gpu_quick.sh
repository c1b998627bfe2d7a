#!/bin/bash
# Quick GPU check: kernel numerics, optional op subset microbench, headline bench.
#   OPS=norm,attn BENCH=1 bash tools/gpu_quick.sh
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
set -o pipefail
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -x -q -m gpu --timeout 120 --timeout-method thread \
  > gpurun_out/q_kernels.log 2>&1 || { tail -30 gpurun_out/q_kernels.log; exit 1; }
tail -2 gpurun_out/q_kernels.log
if [ -n "${OPS}" ]; then
  timeout -k 10 600 python -u tools/bench_ops.py --only "${OPS}" > gpurun_out/q_ops.log 2>&1 || { tail -20 gpurun_out/q_ops.log; exit 1; }
  cat gpurun_out/q_ops.log | grep '^{'
fi
if [ "${MODELS:-0}" = "1" ]; then
  timeout -k 10 600 python -u -m pytest tests/test_models_gpu.py -x -q -m gpu --timeout 300 --timeout-method thread \
    > gpurun_out/q_models.log 2>&1 || { tail -30 gpurun_out/q_models.log; exit 1; }
  tail -2 gpurun_out/q_models.log
fi
if [ "${BENCH:-1}" = "1" ]; then
  timeout -k 10 600 python -u bench.py --steps 3 --warmup 1 > gpurun_out/q_bench.log 2>&1 || { tail -20 gpurun_out/q_bench.log; exit 1; }
  grep '^{' gpurun_out/q_bench.log
fi
if [ "${PROFILE:-0}" = "1" ]; then
  export TMPDIR=/tmp
  timeout -k 10 600 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_q -o run --output-format csv -- \
    python bench.py --steps 1 --warmup 1 --denoise-steps 20 --no-score > gpurun_out/q_prof.log 2>&1 || { tail -20 gpurun_out/q_prof.log; exit 1; }
fi
echo QUICKDONE

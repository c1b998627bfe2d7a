#!/bin/bash
# kernel numerics + per-op microbenchmarks vs stock PyTorch ops
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
timeout -k 10 600 python -m pytest tests/test_kernels_gpu.py -q -m gpu > gpurun_out/kernels.log 2>&1
rc=$?; tail -3 gpurun_out/kernels.log; echo "kernels rc=$rc"
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 900 python tools/bench_ops.py ${OPS_ARGS} > gpurun_out/ops.jsonl 2> gpurun_out/ops.err
rc=$?; echo "ops rc=$rc"; cat gpurun_out/ops.jsonl; tail -3 gpurun_out/ops.err
exit $rc

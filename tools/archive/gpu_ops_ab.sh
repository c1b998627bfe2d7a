#!/bin/bash
# A/B of GEMM pipeline depth: kernel tests, then gemm/conv microbench with 2 and 3 stages
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
timeout -k 10 600 python -m pytest tests/test_kernels_gpu.py -q -m gpu -k "gemm or conv or bmm" > gpurun_out/kernels.log 2>&1
rc=$?; tail -3 gpurun_out/kernels.log; echo "kernels rc=$rc"
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
CASSMANTLE_GEMM_STAGES=3 timeout -k 10 600 python -m pytest tests/test_kernels_gpu.py -q -m gpu -k "gemm or conv or bmm" > gpurun_out/kernels3.log 2>&1
rc=$?; tail -3 gpurun_out/kernels3.log; echo "kernels3 rc=$rc"
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
for st in 2 3; do
  CASSMANTLE_GEMM_STAGES=$st timeout -k 10 600 python tools/bench_ops.py --only gemm,conv > gpurun_out/ops_st$st.jsonl 2> gpurun_out/ops_st$st.err
  rc=$?; echo "ops stages=$st rc=$rc"
  if [ $rc -ne 0 ]; then tail -5 gpurun_out/ops_st$st.err; exit $rc; fi
done

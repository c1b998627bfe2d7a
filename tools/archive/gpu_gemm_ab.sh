#!/bin/bash
# GEMM/conv A/B of an env knob: kernel tests (both arms), gemm/conv microbench (both arms),
# then the full bench.  Usage: KNOB=CASSMANTLE_GEMM_BUF A=0 B=1 bash tools/gpu_gemm_ab.sh
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
for v in $B $A; do
  env $KNOB=$v timeout -k 10 600 python -m pytest tests/test_kernels_gpu.py -q -m gpu -x -k "gemm or conv or bmm" > gpurun_out/kernels_$v.log 2>&1
  rc=$?; tail -2 gpurun_out/kernels_$v.log; echo "kernels $KNOB=$v rc=$rc"
  if [ $rc -ne 0 ]; then exit $rc; fi
done
for v in $A $B; do
  env $KNOB=$v timeout -k 10 600 python tools/bench_ops.py --only gemm,conv > gpurun_out/ops_$v.jsonl 2> gpurun_out/ops_$v.err
  rc=$?; echo "ops $KNOB=$v rc=$rc"
  if [ $rc -ne 0 ]; then tail -5 gpurun_out/ops_$v.err; exit $rc; fi
done
timeout -k 10 600 python bench.py > gpurun_out/bench.log 2>&1
rc=$?; tail -1 gpurun_out/bench.log; echo "bench rc=$rc"
exit $rc

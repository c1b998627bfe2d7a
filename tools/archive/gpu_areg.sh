#!/bin/bash
# cfg-15 (A-in-registers) numerics for both variants, then the shape A/B
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
for v in 1 2; do
  CASSMANTLE_AREG_V=$v timeout -k 10 240 python -u -m pytest tests/test_kernels_gpu.py -x -v -m gpu -k "areg" --timeout 120 --timeout-method thread \
    > gpurun_out/areg_tests$v.log 2>&1
  rc=$?; tail -2 gpurun_out/areg_tests$v.log; echo "tests v=$v rc=$rc"
  [ $rc -ne 0 ] && exit $rc
done
for v in 1 2; do
  CASSMANTLE_AREG_V=$v timeout -k 10 240 python -u tools/bench_areg.py > gpurun_out/areg_bench$v.jsonl 2> gpurun_out/areg_bench$v.err
  rc=$?; echo "v=$v"; cat gpurun_out/areg_bench$v.jsonl; tail -3 gpurun_out/areg_bench$v.err; echo "bench rc=$rc"
  [ $rc -ne 0 ] && exit $rc
done
exit 0

#!/bin/bash
# stage overlap: numerics, then bench A/B (interleaved, 2 repeats each), batch-1 latency
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_models_gpu.py -x -q -m gpu -k "overlap" --timeout 240 --timeout-method thread > gpurun_out/overlap_tests.log 2>&1
rc=$?; tail -3 gpurun_out/overlap_tests.log; echo "tests rc=$rc"
[ $rc -ne 0 ] && exit $rc
for arm in "" "--overlap" "" "--overlap"; do
  timeout -k 10 400 python -u bench.py --steps 3 --warmup 1 --no-score $arm > gpurun_out/ov_bench.log 2>&1 || { tail -5 gpurun_out/ov_bench.log; exit 1; }
  echo "arm[$arm] $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/ov_bench.log) $(grep -o '"batch1_s_per_image": [0-9.]*' gpurun_out/ov_bench.log)"
done
exit 0

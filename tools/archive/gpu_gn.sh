#!/bin/bash
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -x -q -m gpu -k "group_norm or gn" --timeout 120 --timeout-method thread > gpurun_out/gn_tests.log 2>&1
rc=$?; tail -2 gpurun_out/gn_tests.log; echo "tests rc=$rc"; [ $rc -ne 0 ] && exit $rc
for m in -1 0; do
  CASSMANTLE_GN_ROWS=$m timeout -k 10 200 python -u tools/bench_gn.py > gpurun_out/gn_bench$m.jsonl 2>&1 || exit 1
  echo "mode $m"; grep -v amdgpu.ids gpurun_out/gn_bench$m.jsonl
done
for m in -1 0 -1 0; do
  CASSMANTLE_GN_ROWS=$m timeout -k 10 400 python -u bench.py --steps 3 --warmup 1 --no-score --no-batch1 > gpurun_out/gn_b.log 2>&1 || { tail -5 gpurun_out/gn_b.log; exit 1; }
  echo "gnrows=$m $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/gn_b.log)"
done

#!/bin/bash
# GroupNorm apply prologue (batched stats loads): norm tests + bandwidth; SD-1.5 bench vs the
# pre-fp8-epilogue build (ab/_C_prekv8.so: does the kv8 epilogue code cost the bf16 GEMMs?)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -x -q --timeout 120 --timeout-method thread -k "group_norm or gn or stats" > gpurun_out/r3_gn_tests.txt 2>&1
rc=$?; tail -2 gpurun_out/r3_gn_tests.txt; [ $rc -ne 0 ] && { grep -E "Error|assert" gpurun_out/r3_gn_tests.txt | head; exit $rc; }
timeout -k 10 120 python -u tools/bench_membound.py > gpurun_out/membound2.jsonl 2>&1 || { tail -5 gpurun_out/membound2.jsonl; exit 1; }
grep gn_apply gpurun_out/membound2.jsonl
for r in 1 2 3; do
  for arm in cur prekv8; do
    so=""; [ $arm = prekv8 ] && so="ab/_C_prekv8.so"
    CASSMANTLE_EXT_SO=$so timeout -k 10 200 python -u bench.py --steps 5 --warmup 2 --no-score --no-batch1 > gpurun_out/ab2.log 2>&1 || { tail -5 gpurun_out/ab2.log; exit 1; }
    echo "$arm | $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/ab2.log) $(grep -o '"stage_mean_ms": {[^}]*}' gpurun_out/ab2.log)" | tee -a gpurun_out/r3_ab_prekv8.txt
  done
done

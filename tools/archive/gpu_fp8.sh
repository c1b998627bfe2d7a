#!/bin/bash
# fp8 attention: numerics (incl. pre-packed cross K/V), microbench, SDXL end-to-end bf16 vs fp8
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
timeout -k 10 240 python -u -m pytest tests/test_kernels_gpu.py -x -q -m gpu -k "attention or set_context" --timeout 120 --timeout-method thread \
  > gpurun_out/fp8_tests.log 2>&1
rc=$?; tail -3 gpurun_out/fp8_tests.log; echo "tests rc=$rc"
[ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python -u tools/bench_attn.py --rounds 3 > gpurun_out/attn_bench.jsonl 2> gpurun_out/attn_bench.err
rc=$?; cat gpurun_out/attn_bench.jsonl; echo "bench rc=$rc"
[ $rc -ne 0 ] && exit $rc
for arm in "" "--fp8-attention" "" "--fp8-attention"; do
  timeout -k 10 400 python -u bench.py --model sdxl --batch 1 --steps 2 --warmup 1 --no-score $arm > gpurun_out/sdxl_bench.log 2>&1 || { tail -5 gpurun_out/sdxl_bench.log; exit 1; }
  echo "sdxl $arm $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/sdxl_bench.log) $(grep -o '"value": [0-9.]*' gpurun_out/sdxl_bench.log)"
done
exit 0

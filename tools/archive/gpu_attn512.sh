#!/bin/bash
# head-dim-512 flash attention: numerics, then the A/B vs SDPA and the GEMM path
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
timeout -k 10 240 python -u -m pytest tests/test_kernels_gpu.py -x -v -m gpu -k "attention" --timeout 120 --timeout-method thread \
  > gpurun_out/a512_tests.log 2>&1
rc=$?; grep -E "PASS|FAIL|Error|error" gpurun_out/a512_tests.log | tail -30; echo "tests rc=$rc"
[ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python -u tools/bench_attn_d512.py > gpurun_out/a512_bench.jsonl 2> gpurun_out/a512_bench.err
rc=$?; cat gpurun_out/a512_bench.jsonl; tail -3 gpurun_out/a512_bench.err; echo "bench rc=$rc"
exit $rc

#!/bin/bash
# attention numerics + microbenchmark (bf16 / fp8 / SDPA)
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
timeout -k 10 240 python -u -m pytest tests/test_kernels_gpu.py -x -q -m gpu -k "attention" --timeout 120 --timeout-method thread \
  > gpurun_out/attn_tests.log 2>&1
rc=$?; tail -3 gpurun_out/attn_tests.log; echo "tests rc=$rc"
[ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python -u tools/bench_attn.py ${ATTN_ARGS} > gpurun_out/attn_bench.jsonl 2> gpurun_out/attn_bench.err
rc=$?; cat gpurun_out/attn_bench.jsonl; tail -3 gpurun_out/attn_bench.err; echo "bench rc=$rc"
[ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python -u tools/bench_attn_d512.py > gpurun_out/a512_bench.jsonl 2> gpurun_out/a512_bench.err
rc=$?; cat gpurun_out/a512_bench.jsonl; echo "d512 rc=$rc"
exit $rc

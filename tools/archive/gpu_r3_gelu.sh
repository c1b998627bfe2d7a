#!/bin/bash
# cheaper GEGLU GELU: numerics (kernel + full-size model + e2e PSNR tests), then SD-1.5 bench
# A/B against the erf_fast build (ab/_C_gelu_exact.so), same box, interleaved x3
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -x -q --timeout 120 --timeout-method thread -k "geglu or gemm or linear or areg" > gpurun_out/r3_gelu_tests.txt 2>&1
rc=$?; tail -2 gpurun_out/r3_gelu_tests.txt; [ $rc -ne 0 ] && { grep -E "Error|assert" gpurun_out/r3_gelu_tests.txt | head; exit $rc; }
timeout -k 10 600 python -u -m pytest tests/test_models_gpu.py -x -q --timeout 300 --timeout-method thread -k "full_size or end_to_end or sdxl" > gpurun_out/r3_gelu_mtests.txt 2>&1
rc=$?; tail -2 gpurun_out/r3_gelu_mtests.txt; [ $rc -ne 0 ] && { grep -E "Error|assert" gpurun_out/r3_gelu_mtests.txt | head; exit $rc; }
for r in 1 2 3; do
  for arm in fast exact; do
    so=""; [ $arm = exact ] && so="ab/_C_gelu_exact.so"
    CASSMANTLE_EXT_SO=$so timeout -k 10 200 python -u bench.py --steps 5 --warmup 2 --no-score --no-batch1 > gpurun_out/gelu_ab.log 2>&1 || { tail -5 gpurun_out/gelu_ab.log; exit 1; }
    echo "gelu=$arm | $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/gelu_ab.log) $(grep -o '"stage_mean_ms": {[^}]*}' gpurun_out/gelu_ab.log)" | tee -a gpurun_out/r3_gelu_ab.txt
  done
done
# memory-bound passes: GroupNorm apply (events) + split-K reduce (kernel trace) bandwidth
timeout -k 10 120 rocprofv3 --kernel-trace -d gpurun_out/membound -o run --output-format csv -- python -u tools/bench_membound.py > gpurun_out/membound.jsonl 2>gpurun_out/membound.err || { tail -5 gpurun_out/membound.err; exit 1; }
python tools/bench_membound.py --trace "$(find gpurun_out/membound -name '*kernel_trace.csv' | head -1)" --lines gpurun_out/membound.jsonl > gpurun_out/membound_reduce.jsonl
grep gn_apply gpurun_out/membound.jsonl; cat gpurun_out/membound_reduce.jsonl

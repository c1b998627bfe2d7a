#!/bin/bash
# round 5: mixed-shape d=40 attention: numerics, then same-box A/B of the three d=40 kernels (x2)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_kernels_gpu.py -k "d40 or test_attention" > gpurun_out/r5n_tests.txt 2>&1 || { tail -30 gpurun_out/r5n_tests.txt; exit 1; }
tail -3 gpurun_out/r5n_tests.txt
for rep in 1 2; do
  timeout -k 10 300 python -u tools/bench_attn.py --only-d 40 --rounds 7 --iters 20 > gpurun_out/r5n_attn_$rep.jsonl 2>&1 || { tail -20 gpurun_out/r5n_attn_$rep.jsonl; exit 1; }
  grep shape gpurun_out/r5n_attn_$rep.jsonl
done

#!/bin/bash
# round 5: the 16x16-block d=40 attention: numerics, then A/B vs the 32x32x16 kernel (x2)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/r5d
mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread \
  tests/test_kernels_gpu.py -k "attention" > $O/tests.txt 2>&1 || { tail -40 $O/tests.txt; exit 1; }
tail -3 $O/tests.txt
for r in 1 2; do
  timeout -k 10 300 python tools/bench_attn.py --only-d 40 --rounds 7 > $O/attn_ab_$r.jsonl 2> $O/attn_ab_$r.err || { tail -20 $O/attn_ab_$r.err; exit 1; }
  cat $O/attn_ab_$r.jsonl
done

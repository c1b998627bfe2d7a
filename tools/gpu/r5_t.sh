#!/bin/bash
# round 5: adaptive rows-per-block of the split-K reduce + statistics pass: kernel tests, then
# same-box A/B (CASSMANTLE_SK_ADAPT=1 vs 0) of batch-1 latency and the batch-4 step (x2)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/r5t; mkdir -p $O
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_kernels_gpu.py -k "split or stats or conv or gemm" > $O/tests.txt 2>&1 || { tail -30 $O/tests.txt; exit 1; }
tail -2 $O/tests.txt
for rep in 1 2; do
  for ad in 1 0; do
    CASSMANTLE_SK_ADAPT=$ad timeout -k 10 300 python bench.py --steps 3 --warmup 1 --no-score > $O/bench_${ad}_$rep.json 2> $O/bench_${ad}_$rep.err || { tail -5 $O/bench_${ad}_$rep.err; exit 1; }
    python -c "import json;a=json.load(open('$O/bench_${ad}_$rep.json'));print('rep $rep adapt $ad ms_per_step', a['ms_per_step'], 'batch1_s', a.get('batch1_s_per_image'))"
  done
done

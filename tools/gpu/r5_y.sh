#!/bin/bash
# round 5: key split of the batch-1 level-1 self-attention: tests, kernel A/B, bench A/B (x2)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/r5y; mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_kernels_gpu.py -k "attention" > $O/tests.txt 2>&1 || { tail -30 $O/tests.txt; exit 1; }
tail -2 $O/tests.txt
for sp in 1 0; do
  CASSMANTLE_ATTN_SPLIT=$sp timeout -k 10 300 python -u tools/probe_attn_overhead.py > $O/attn_$sp.jsonl 2>&1 || { tail -20 $O/attn_$sp.jsonl; exit 1; }
  echo "split=$sp"; grep sd15_l1 $O/attn_$sp.jsonl
done
for rep in 1 2; do
  for sp in 1 0; do
    CASSMANTLE_ATTN_SPLIT=$sp timeout -k 10 300 python bench.py --steps 2 --warmup 1 --no-score > $O/bench_${sp}_$rep.json 2> $O/bench_${sp}_$rep.err || { tail -5 $O/bench_${sp}_$rep.err; exit 1; }
    python -c "import json;a=json.load(open('$O/bench_${sp}_$rep.json'));print('rep $rep split $sp ms_per_step', a['ms_per_step'], 'batch1_s', a.get('batch1_s_per_image'))"
  done
done

#!/bin/bash
# round 5: key split of the generic attention kernel only where the split grid fits one round
# (batch-1 levels 2 / 3): tests, kernel probe, bench A/B (x2)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/r5ag; mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_kernels_gpu.py -k "attention" > $O/tests.txt 2>&1 || { tail -30 $O/tests.txt; exit 1; }
tail -1 $O/tests.txt
for rep in 1 2; do
  for sp in 1 0; do
    CASSMANTLE_ATTN_SPLIT=$sp timeout -k 10 300 python -u tools/probe_attn_overhead.py > $O/attn_${sp}_$rep.jsonl 2>&1 || { tail -20 $O/attn_${sp}_$rep.jsonl; exit 1; }
    echo "split $sp rep $rep"; grep -E "sd15_l3|sd15_l2" $O/attn_${sp}_$rep.jsonl | grep -E '"Nk": (256|1024)'
    CASSMANTLE_ATTN_SPLIT=$sp timeout -k 10 300 python bench.py --steps 2 --warmup 1 --no-score > $O/bench_${sp}_$rep.json 2> $O/bench_${sp}_$rep.err || { tail -5 $O/bench_${sp}_$rep.err; exit 1; }
    python -c "import json;a=json.load(open('$O/bench_${sp}_$rep.json'));print('rep $rep split $sp batch1_s', a.get('batch1_s_per_image'), 'ms_per_step', a['ms_per_step'])"
  done
done

#!/bin/bash
# round 5: 4-wave vs 2-wave blocks of the generic attention on the batch-1 grids (levels 2 / 3)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/r5ah; mkdir -p $O
for rep in 1 2; do
  for t in 512 16; do
    CASSMANTLE_ATTN_NW4_MIN=$t timeout -k 10 300 python -u tools/probe_attn_overhead.py > $O/attn_${t}_$rep.jsonl 2>&1 || { tail -20 $O/attn_${t}_$rep.jsonl; exit 1; }
    echo "nw4_min $t rep $rep"; grep -E "sd15_l3_b2|sd15_l2_b2" $O/attn_${t}_$rep.jsonl | grep -E '"Nk": (256|1024)'
    CASSMANTLE_ATTN_NW4_MIN=$t timeout -k 10 300 python bench.py --steps 1 --warmup 1 --no-score > $O/bench_${t}_$rep.json 2> $O/bench_${t}_$rep.err || { tail -5 $O/bench_${t}_$rep.err; exit 1; }
    python -c "import json;a=json.load(open('$O/bench_${t}_$rep.json'));print('rep $rep nw4_min $t batch1_s', a.get('batch1_s_per_image'), 'ms_per_step', a['ms_per_step'])"
  done
done

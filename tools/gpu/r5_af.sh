#!/bin/bash
# round 5: level-1 attention block size at batch 1 (B = 2: 256 eight-wave blocks vs 512 four-wave)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/r5af; mkdir -p $O
for rep in 1 2; do
  for t in 512 128; do
    CASSMANTLE_ATTN16_NW8_MIN=$t timeout -k 10 300 python -u tools/probe_attn_overhead.py > $O/attn_${t}_$rep.jsonl 2>&1 || { tail -20 $O/attn_${t}_$rep.jsonl; exit 1; }
    echo "nw8_min $t rep $rep"; grep sd15_l1 $O/attn_${t}_$rep.jsonl | tail -1
    CASSMANTLE_ATTN16_NW8_MIN=$t timeout -k 10 300 python bench.py --steps 1 --warmup 1 --no-score > $O/bench_${t}_$rep.json 2> $O/bench_${t}_$rep.err || { tail -5 $O/bench_${t}_$rep.err; exit 1; }
    python -c "import json;a=json.load(open('$O/bench_${t}_$rep.json'));print('rep $rep nw8_min $t batch1_s', a.get('batch1_s_per_image'), 'ms_per_step', a['ms_per_step'])"
  done
done

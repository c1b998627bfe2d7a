#!/bin/bash
# round 5: same-box A/B of the merged table (batch-1 plans re-tuned cold, batch-8 keys unchanged)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/r5r; mkdir -p $O
for rep in 1 2; do
  for t in prev new; do
    tp=cassmantle_amd/ops/gemm_tuning.json; [ $t = prev ] && tp=tools/gemm_tuning_prev.json
    CASSMANTLE_GEMM_TUNE_PATH=$tp timeout -k 10 300 python bench.py --steps 2 --warmup 1 --no-score > $O/bench_${t}_$rep.json 2> $O/bench_${t}_$rep.err || { tail -5 $O/bench_${t}_$rep.err; exit 1; }
    python -c "import json;a=json.load(open('$O/bench_${t}_$rep.json'));print('rep $rep table $t ms_per_step', a['ms_per_step'], 'batch1_s', a.get('batch1_s_per_image'))"
  done
done

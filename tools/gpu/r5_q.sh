#!/bin/bash
# round 5: in-situ re-tune of the batch-1 (config 2) GEMM shapes with cold weights, then same-box
# A/B of batch-1 latency and the batch-4 step, previous table vs new (x2)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/r5q; mkdir -p $O
cp cassmantle_amd/ops/gemm_tuning.json $O/tune_prev.json
timeout -k 10 900 python -u tools/autotune_gemm.py --models sd15 --batch 1 --merge --cold 512 > $O/autotune_b1.jsonl 2> $O/autotune_b1.err || { tail -5 $O/autotune_b1.err; exit 1; }
tail -2 $O/autotune_b1.jsonl
cp cassmantle_amd/ops/gemm_tuning.json $O/tune_new.json
for rep in 1 2; do
  for t in prev new; do
    CASSMANTLE_GEMM_TUNE_PATH=$O/tune_$t.json timeout -k 10 300 python bench.py --steps 2 --warmup 1 --no-score > $O/bench_${t}_$rep.json 2> $O/bench_${t}_$rep.err || { tail -5 $O/bench_${t}_$rep.err; exit 1; }
    python -c "import json;a=json.load(open('$O/bench_${t}_$rep.json'));print('rep $rep table $t ms_per_step', a['ms_per_step'], 'batch1_s', a.get('batch1_s_per_image'))"
  done
done

#!/bin/bash
# round 5: cold (weights from HBM) in-situ re-tune of the batch-4 (CFG 8) SD-1.5 pass on top of the
# current table, then same-box A/B current vs re-tuned (x2)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/r5s; mkdir -p $O
cp cassmantle_amd/ops/gemm_tuning.json $O/tune_cur.json
cp cassmantle_amd/ops/gemm_tuning.json $O/tune_b4cold.json     # --merge reads the --out file
timeout -k 10 900 python -u tools/autotune_gemm.py --models sd15 --batch 4 --merge --cold 512 --out $O/tune_b4cold.json > $O/autotune_b4.jsonl 2> $O/autotune_b4.err || { tail -5 $O/autotune_b4.err; exit 1; }
tail -1 $O/autotune_b4.jsonl
for rep in 1 2; do
  for t in cur b4cold; do
    CASSMANTLE_GEMM_TUNE_PATH=$O/tune_$t.json timeout -k 10 300 python bench.py --steps 3 --warmup 1 --no-score > $O/bench_${t}_$rep.json 2> $O/bench_${t}_$rep.err || { tail -5 $O/bench_${t}_$rep.err; exit 1; }
    python -c "import json;a=json.load(open('$O/bench_${t}_$rep.json'));print('rep $rep table $t ms_per_step', a['ms_per_step'], 'batch1_s', a.get('batch1_s_per_image'))"
    CASSMANTLE_GEMM_TUNE_PATH=$O/tune_$t.json timeout -k 10 300 python bench.py --model sdxl --fp8-attention --batch 1 --steps 2 --warmup 1 --no-score --no-batch1 > $O/sdxl_${t}_$rep.json 2> $O/sdxl_${t}_$rep.err || { tail -5 $O/sdxl_${t}_$rep.err; exit 1; }
    python -c "import json;a=json.load(open('$O/sdxl_${t}_$rep.json'));print('rep $rep table $t sdxl ms_per_step', a['ms_per_step'])"
  done
done

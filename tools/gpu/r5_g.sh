#!/bin/bash
# round 5: in-situ re-tune of the SD-1.5 GEMM table on the grouped tile raster (merge: every
# existing table plan is an arm), then a same-box bench A/B of the old and new tables (x2)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/r5g
mkdir -p $O
cp cassmantle_amd/ops/gemm_tuning.json $O/tune_prev.json
cp cassmantle_amd/ops/gemm_tuning.json $O/tune_new.json
timeout -k 10 780 python tools/autotune_gemm.py --models ${MODEL:-sd15} --batch ${BATCH:-4} --merge --out $O/tune_new.json > $O/tune.log 2>&1 || { tail -20 $O/tune.log; exit 1; }
tail -1 $O/tune.log
for rep in 1 2; do
  for v in prev new; do
    CASSMANTLE_GEMM_TUNE_PATH=$O/tune_$v.json timeout -k 10 300 python bench.py --model ${MODEL:-sd15} --batch ${BATCH:-4} ${EXTRA} --steps 5 --warmup 1 --no-score --no-batch1 > $O/ab_${v}_$rep.json 2> $O/ab_${v}_$rep.err || { tail -5 $O/ab_${v}_$rep.err; exit 1; }
    echo "$v $rep $(python -c "import json;print(json.load(open('$O/ab_${v}_$rep.json'))['ms_per_step'])")"
  done
done

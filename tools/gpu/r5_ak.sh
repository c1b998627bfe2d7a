#!/bin/bash
# round 5: fp8 attention with two LDS stages (one barrier per key step) vs one stage:
# fp8 kernel tests (both), kernel A/B at the SDXL shapes, SDXL bench A/B (x2 interleaved)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/r5ak
mkdir -p $O
for db in 1 0; do
  CASSMANTLE_FP8_DBUF=$db timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -x -q --timeout 120 --timeout-method thread \
    -m gpu -k "fp8" -p no:cacheprovider > $O/tests_db$db.txt 2>&1 || { tail -30 $O/tests_db$db.txt; exit 1; }
  tail -1 $O/tests_db$db.txt
done
for db in 1 0 1 0; do
  CASSMANTLE_FP8_DBUF=$db timeout -k 10 180 python tools/bench_attn_fp8.py --rounds 3 --iters 30 2>>$O/err.txt \
    | sed "s/^/{\"dbuf\": $db, \"row\": /; s/\$/}/" >> $O/attn_ab.jsonl || exit 1
done
for rep in 1 2; do
  for db in 1 0; do
    CASSMANTLE_FP8_DBUF=$db timeout -k 10 300 python bench.py --model sdxl --fp8-attention --batch 1 --steps 2 --warmup 1 --no-score --no-batch1 > $O/sdxl_${db}_$rep.json 2> $O/sdxl_${db}_$rep.err || { tail -5 $O/sdxl_${db}_$rep.err; exit 1; }
    echo "db=$db rep=$rep $(python -c "import json;d=json.load(open('$O/sdxl_${db}_$rep.json'));print(d['ms_per_step'])")"
  done
done

#!/bin/bash
# round 5: fp8 attention row sums by an all-ones MFMA (key-split variants): tests, kernel probe
# and SDXL bench, same box, main build vs F8_ONES_SUM=0 build (x2)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/r5ab; mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_kernels_gpu.py -k "fp8" > $O/tests.txt 2>&1 || { tail -30 $O/tests.txt; exit 1; }
tail -2 $O/tests.txt
for rep in 1 2; do
  for v in main vsum; do
    so=""; [ $v = vsum ] && so=variants/f8_vsum.so
    CASSMANTLE_EXT_SO=$so timeout -k 10 300 python -u tools/probe_attn_overhead.py > $O/attn_${v}_$rep.jsonl 2>&1 || { tail -20 $O/attn_${v}_$rep.jsonl; exit 1; }
    echo "$v rep $rep"; grep sdxl_l3_fp8 $O/attn_${v}_$rep.jsonl
    CASSMANTLE_EXT_SO=$so timeout -k 10 300 python bench.py --model sdxl --fp8-attention --batch 1 --steps 2 --warmup 1 --no-score --no-batch1 > $O/sdxl_${v}_$rep.json 2> $O/sdxl_${v}_$rep.err || { tail -5 $O/sdxl_${v}_$rep.err; exit 1; }
    python -c "import json;a=json.load(open('$O/sdxl_${v}_$rep.json'));print('rep $rep $v sdxl ms_per_step', a['ms_per_step'], a.get('finite'))"
  done
done

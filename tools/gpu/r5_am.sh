#!/bin/bash
# round 5: fp8 attention cross-half max / sum by v_permlane32_swap (main) vs ds_bpermute (variants/f8_shfl.so, -DATTN_PERMLANE=0)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/r5am
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -x -q --timeout 120 --timeout-method thread \
  -m gpu -k "fp8" -p no:cacheprovider > $O/tests.txt 2>&1 || { tail -30 $O/tests.txt; exit 1; }
tail -1 $O/tests.txt
for v in main shfl main shfl; do
  so=""; [ $v = shfl ] && so=variants/f8_shfl.so
  CASSMANTLE_EXT_SO=$so timeout -k 10 180 python tools/bench_attn_fp8.py --rounds 3 --iters 30 2>>$O/err.txt \
    | sed "s/^/{\"v\": \"$v\", \"row\": /; s/\$/}/" >> $O/attn_ab.jsonl || exit 1
done
for rep in 1 2; do
  for v in main shfl; do
    so=""; [ $v = shfl ] && so=variants/f8_shfl.so
    CASSMANTLE_EXT_SO=$so timeout -k 10 300 python bench.py --model sdxl --fp8-attention --batch 1 --steps 2 --warmup 1 --no-score --no-batch1 > $O/sdxl_${v}_$rep.json 2> $O/sdxl_${v}_$rep.err || { tail -5 $O/sdxl_${v}_$rep.err; exit 1; }
    echo "v=$v rep=$rep $(python -c "import json;d=json.load(open('$O/sdxl_${v}_$rep.json'));print(d['ms_per_step'])")"
  done
done

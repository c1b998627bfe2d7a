#!/bin/bash
# round 5: GEMM fragment prefetch across the two k-steps of a k-tile, now actually scheduled that way
# (sched_barrier; variants/gemm_fp.so, -DGEMM_FRAG_PREFETCH=1) vs the tree: GEMM / conv kernel tests on
# the variant, SD-1.5 bench (incl. batch 1) and SDXL bench, interleaved x2
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/r5ao
mkdir -p $O
CASSMANTLE_EXT_SO=variants/gemm_fp.so timeout -k 10 400 python -u -m pytest tests/test_kernels_gpu.py -x -q --timeout 120 \
  --timeout-method thread -m gpu -k "gemm or conv or norm" -p no:cacheprovider > $O/tests.txt 2>&1 || { tail -30 $O/tests.txt; exit 1; }
tail -1 $O/tests.txt
for rep in 1 2; do
  for v in fp tree; do
    so=""; [ $v = fp ] && so=variants/gemm_fp.so
    CASSMANTLE_EXT_SO=$so timeout -k 10 300 python bench.py > $O/sd15_${v}_$rep.json 2> $O/sd15_${v}_$rep.err || { tail -5 $O/sd15_${v}_$rep.err; exit 1; }
    echo "sd15 v=$v rep=$rep $(python -c "import json;d=json.load(open('$O/sd15_${v}_$rep.json'));print(d['ms_per_step'], d['batch1_s_per_image'])")"
  done
done
for rep in 1 2; do
  for v in fp tree; do
    so=""; [ $v = fp ] && so=variants/gemm_fp.so
    CASSMANTLE_EXT_SO=$so timeout -k 10 300 python bench.py --model sdxl --fp8-attention --batch 1 --steps 2 --warmup 1 --no-score --no-batch1 > $O/sdxl_${v}_$rep.json 2> $O/sdxl_${v}_$rep.err || { tail -5 $O/sdxl_${v}_$rep.err; exit 1; }
    echo "sdxl v=$v rep=$rep $(python -c "import json;d=json.load(open('$O/sdxl_${v}_$rep.json'));print(d['ms_per_step'])")"
  done
done

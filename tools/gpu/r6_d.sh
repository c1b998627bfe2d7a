#!/bin/bash
# round 6: warm-up of the block's own W panel by the MFMA waves of the warp-specialised GEMM tiles
# (GEMM_PF_SELF 1: whole panel per block, 2: a quarter per block) vs the tree, same box, interleaved
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/r6d
mkdir -p $O
CASSMANTLE_EXT_SO=variants/gemm_pf2.so timeout -k 10 400 python -u -m pytest tests/test_kernels_gpu.py -x -q --timeout 120 \
  --timeout-method thread -m gpu -k "gemm or conv" -p no:cacheprovider > $O/tests_pf2.txt 2>&1 || { tail -30 $O/tests_pf2.txt; exit 1; }
tail -1 $O/tests_pf2.txt
timeout -k 10 400 python -u -m pytest tests/test_kernels_gpu.py tests/test_lm.py tests/test_parallel_gpu.py -x -q --timeout 200 \
  --timeout-method thread -m gpu -k "lm_sample or d40 or lm_gpu or supervised" -p no:cacheprovider > $O/tests_new.txt 2>&1 || { tail -40 $O/tests_new.txt; exit 1; }
tail -1 $O/tests_new.txt
for rep in 1 2; do
  for v in tree pf1 pf2; do
    so=""; [ $v != tree ] && so=variants/gemm_$v.so
    CASSMANTLE_EXT_SO=$so timeout -k 10 300 python bench.py --steps 10 --warmup 3 --no-score --no-live --no-sdxl > $O/sd15_${v}_$rep.json 2> $O/sd15_${v}_$rep.err || { tail -5 $O/sd15_${v}_$rep.err; exit 1; }
    echo "sd15 v=$v rep=$rep $(python -c "import json;d=json.load(open('$O/sd15_${v}_$rep.json'));print(d['ms_per_step'], d['batch1_s_per_image'])")"
  done
done
for rep in 1 2; do
  for v in tree pf1 pf2; do
    so=""; [ $v != tree ] && so=variants/gemm_$v.so
    CASSMANTLE_EXT_SO=$so timeout -k 10 300 python bench.py --model sdxl --fp8-attention --batch 1 --steps 2 --warmup 1 --no-score --no-batch1 --no-live --no-sdxl > $O/sdxl_${v}_$rep.json 2> $O/sdxl_${v}_$rep.err || { tail -5 $O/sdxl_${v}_$rep.err; exit 1; }
    echo "sdxl v=$v rep=$rep $(python -c "import json;d=json.load(open('$O/sdxl_${v}_$rep.json'));print(d['ms_per_step'])")"
  done
done
